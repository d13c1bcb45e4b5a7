"""debugging aid: the Sedov n50 trajectory with and without skin lists, energy and time vs the reference fixture"""
import sys
for p in ("tests", "oracle", "sph-exa_amd/python", "."):
    sys.path.insert(0, p)
import numpy as np
import golden_util as gu
import pyoracle as po
import sphexa_amd as sx
import trajectory as tj

fname, init, side, steps, prof_steps, rmax, nbins = tj.CASES["sedov"]
fx = gu.load(fname)
for skin in (0.0, 0.08):
    st, obox = getattr(po, init + "_state")(side)
    ctx = sx.Context(0)
    sim = sx.Sim(ctx, st.n, sx.make_box(list(obox.lim), list(obox.bnd)), params=sx.default_params())
    sim.set_skin(skin, 24 if skin else 1)
    sim.set_state(st.arrays, st.minDt, st.minDt_m1)
    t, e, mdt = [0.0], [tj.energies(st.arrays)[0]], []
    for s in range(1, steps + 1):
        sim.step()
        sc = sim.scalars()
        t.append(sc["ttot"])
        e.append(tj.energies(sim.get(tj.FIELDS))[0])
    sim.close()
    ctx.close()
    t, e = np.array(t), np.array(e)
    de = (e - fx["series_etot"]) / fx["series_etot"][0]
    dt = t[1:] / fx["series_ttot"][1:] - 1
    print("skin", skin, "max |de|", np.abs(de).max(), "at", np.abs(de).argmax(), "max |dt|", np.abs(dt).max(), flush=True)
    for s in list(range(0, 201, 20)) + list(range(180, 195)):
        print(f"  step {s}: de {de[s]:+.3e}  dt {dt[max(s - 1, 0)]:+.3e}  e {e[s]:.10f} ref {fx['series_etot'][s]:.10f}")
