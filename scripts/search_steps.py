"""Per-step search build and kernel times on one GPU: python scripts/search_steps.py {sedov|noh|evrard} SIDE STEPS."""
import sys

sys.path.insert(0, "sph-exa_amd/python")
import sphexa_amd as sx
from sphexa_amd import ic

init = sys.argv[1] if len(sys.argv) > 1 else "noh"
side = int(sys.argv[2]) if len(sys.argv) > 2 else 300
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
ctx = sx.Context(0)
if init == "sedov":
    n = side ** 3
    sim = sx.Sim(ctx, n, sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1]))
    sim.init_sedov(side)
else:
    arrays, lim, bnd, dt0 = getattr(ic, init)(side)
    n = arrays["x"].size
    sim = sx.Sim(ctx, n, sx.make_box(lim, bnd), params=sx.default_params(g=1.0 if init == "evrard" else 0.0))
    sim.set_state(arrays, dt0, dt0)
for s in range(steps):
    sim.step()
    st, kt = sim.stats(), sim.kernel_times()
    print(s, "build", st["build"], " ".join(f"{k} {v:.2f}" for k, v in kt.items() if v > 0.01),
          "stored/t %.1f" % (st["sumNeighbors"] / n), "cand/t %.1f" % (st["sumCandidates"] / n),
          "union/t %.2f" % (st["sumUnion"] / n), "max", st["maxNeighbors"], flush=True)
sim.close()
ctx.close()
