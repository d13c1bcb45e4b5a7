"""Lane balance of the pair kernels' neighbor loops: per 64-particle group, the loop runs max(nc) iterations while
the lanes average mean(nc).  Prints sum(max) / sum(mean) for the SFC groups as they are, for groups re-formed by
sorting each 256-particle cluster by nc, and the perfectly balanced bound, with the SPLIT-share word counts:
    python scripts/nc_balance.py [side] [steps]"""
import sys

import numpy as np

sys.path.insert(0, "sph-exa_amd/python")
import sphexa_amd as sx  # noqa: E402

side = int(sys.argv[1]) if len(sys.argv) > 1 else 200
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = sx.Context(0)
n = side ** 3
sim = sx.Sim(ctx, n, sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1]))
sim.init_sedov(side)
for s in range(steps):
    sim.step()
nc = sim.get(["nc"])["nc"].astype(np.int64)
sim.close()
ctx.close()
cnt = np.minimum(nc - 1, 150)
m = (cnt.size // 256) * 256
c = cnt[:m]
for split in (1, 2, 3):
    words = (c + 1) // 2
    per = -(-words // split)  # a lane's share of words (ceil): the trip count of one share
    g = per.reshape(-1, 64)
    cl = np.sort(per.reshape(-1, 256), axis=1).reshape(-1, 64)
    mean = g.mean(axis=1).sum()
    print(f"SPLIT {split}: mean words/lane {per.mean():.2f}; sum(max)/sum(mean): SFC groups "
          f"{g.max(axis=1).sum() / mean:.3f}, cluster-sorted {cl.max(axis=1).sum() / mean:.3f}; "
          f"nc min/mean/max {nc.min()}/{nc.mean():.1f}/{nc.max()}")
h = np.bincount(cnt, minlength=151)
print("count histogram (nonzero):", {k: int(v) for k, v in enumerate(h) if v > n // 1000})
