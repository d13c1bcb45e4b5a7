"""Fraction of local positions whose particle changes between consecutive steps (the SFC re-sort's permutation away
from identity): python scripts/perm_stats.py [side] [steps]."""
import sys

import numpy as np

sys.path.insert(0, "sph-exa_amd/python")
import sphexa_amd as sx

side = int(sys.argv[1]) if len(sys.argv) > 1 else 200
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ctx = sx.Context(0)
n = side ** 3
sim = sx.Sim(ctx, n, sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1]))
sim.init_sedov(side)
prev = None
for s in range(steps):
    sim.step()
    ids = sim.get(["id"])["id"]
    if prev is not None:
        moved = np.count_nonzero(ids != prev)
        print(f"step {s}: {moved} of {n} positions changed ({moved / n:.4f})", flush=True)
    prev = ids
sim.close()
ctx.close()
