"""Self-gravity step timing in a periodic box (image walk + Ewald correction) against the same lattice in an open box.

    python scripts/periodic_gravity_timing.py [side ...]

A Sedov lattice at rest with uniform temperature and self-gravity (G = 1), VE propagator, 3 steps after 1 warm-up;
prints the gravity stage's mean ms per step (sx_sim_kernel_times) and the largest |a| of the last step."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "sph-exa_amd", "python"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import pyoracle as po  # noqa: E402
import sphexa_amd as sx  # noqa: E402


def run(ctx, side, bnd, steps=3):
    st, obox = po.sedov_state(side)
    st.temp[:] = np.float64(st.temp.min())
    for k in ("vx", "vy", "vz", "x_m1", "y_m1", "z_m1"):
        st.arrays[k][:] = 0
    sim = sx.Sim(ctx, st.n, sx.make_box(list(obox.lim), [bnd] * 3), params=sx.default_params(g=1.0))
    try:
        sim.set_state(st.arrays, st.minDt, st.minDt_m1)
        sim.step()
        g = []
        for _ in range(steps):
            sim.step()
            g.append(sim.kernel_times().get("gravity", 0.0))
        f = sim.get(["ax", "ay", "az"])
        amax = float(np.sqrt(f["ax"].astype(float) ** 2 + f["ay"] ** 2 + f["az"] ** 2).max())
    finally:
        sim.close()
    return st.n, float(np.mean(g)), amax


if __name__ == "__main__":
    sides = [int(a) for a in sys.argv[1:]] or [64, 100]
    ctx = sx.Context(0)
    try:
        for side in sides:
            for bnd, name in ((0, "open"), (1, "periodic")):
                n, ms, amax = run(ctx, side, bnd)
                print(f"side {side} ({n} particles) {name}: gravity {ms:.2f} ms/step, max|a| {amax:.3g}", flush=True)
    finally:
        ctx.close()
