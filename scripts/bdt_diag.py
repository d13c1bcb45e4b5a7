"""ve vs ve-bdt on a small Evrard sphere: energy series per step (diagnostic)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sph-exa_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import gpu_util as gutil  # noqa: E402
import pyoracle as po  # noqa: E402
import sphexa_amd as sx  # noqa: E402

side = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = sx.Context(0)
ora = po.load_oracle()
st, obox = po.evrard_state(side)
po.converge_h(ora, st, obox)
CONS = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]
for bdt in (False, True):
    sim = sx.Sim(ctx, st.n + 64, gutil.box_to_sx(obox), params=sx.default_params(bdt=bdt, g=1.0))
    sim.set_state({k: st.arrays[k].copy() for k in CONS}, st.minDt, st.minDt)
    for s in range(10):
        sim.step()
        c = sim.conserved()
        sc = sim.scalars()
        ts = sim.timestep() if bdt else {}
        print(f"bdt={bdt} step {s} etot {c['etot']:.7f} ecin {c['ecin']:.7f} eint {c['eint']:.7f} egrav {c['egrav']:.7f}"
              f" dt {sc['minDt']:.3e} ttot {sc['ttot']:.4e} rungs {ts.get('numRungs')} sub {ts.get('substep')}")
    sim.close()
ctx.close()
