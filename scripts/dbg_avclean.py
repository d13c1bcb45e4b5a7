import sys, os
for p in ("tests", "oracle", "sph-exa_amd/python", "."):
    sys.path.insert(0, p)
import numpy as np
import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx
from test_gpu_parity import FLOATS
ora = po.load_oracle()
ctx = sx.Context(0)
for ic, side, steps in [("noh", 16, 2), ("noh", 16, 3), ("sedov", 16, 3)]:
    for av in (True, False):
        for skin in (0.0, 0.08):
            st, obox = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
            sim = sx.Sim(ctx, st.n, gutil.box_to_sx(obox), params=sx.default_params(av_clean=av))
            sim.set_skin(skin, 24 if skin else 1)
            sim.set_state(st.arrays, st.minDt, st.minDt_m1)
            try:
                gutil.shadow_steps(ctx, ora, sim, obox, steps, ora.params(av_clean=av), FLOATS)
                print(ic, side, steps, "av", av, "skin", skin, "OK", sim.skin_stats(), flush=True)
            except AssertionError as e:
                print(ic, side, steps, "av", av, "skin", skin, "FAIL", str(e)[:300], sim.skin_stats(), flush=True)
            sim.close()
ctx.close()
