"""debugging aid: Evrard -n 300 with gravity from the IC, step by step until a failure, with the search statistics"""
import sys
for p in ("tests", "oracle", "sph-exa_amd/python", "."):
    sys.path.insert(0, p)
import numpy as np
import sphexa_amd as sx
from sphexa_amd import ic

arrays, lim, bnd, dt0 = ic.evrard(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
n = arrays["x"].size
ctx = sx.Context(0)
sim = sx.Sim(ctx, n, sx.make_box(lim, bnd), params=sx.default_params(g=1.0))
sim.set_state(arrays, dt0, dt0)
for s in range(1, 101):
    try:
        sim.step()
    except Exception as e:
        print("step", s, "failed:", e, flush=True)
        f = sim.get(["x", "y", "z", "h", "nc"])
        r = np.sqrt(f["x"] ** 2 + f["y"] ** 2 + f["z"] ** 2)
        o = np.argsort(r)[:5]
        print("innermost r", r[o], "h", f["h"][o], "nc", f["nc"][o], "h min", f["h"].min(), "nc max", f["nc"].max())
        c = int(sys.argv[2]) if len(sys.argv) > 2 else -1
        for k in range(256) if c >= 0 else []:
            pass
        import re
        print("see stderr for the failing cluster; cluster geometry of every cluster with extent > 16 h_min:")
        x, y, z, h = f["x"], f["y"], f["z"], f["h"]
        nc_ = (x.size + 255) // 256
        ext = []
        for cc in range(nc_):
            sl = slice(cc * 256, min(x.size, cc * 256 + 256))
            e = max(x[sl].max() - x[sl].min(), y[sl].max() - y[sl].min(), z[sl].max() - z[sl].min())
            ext.append(e / np.median(h[sl]))
        ext = np.array(ext)
        o = np.argsort(ext)[::-1][:10]
        print("largest cluster extents in units of their median h:", [(int(i), round(float(ext[i]), 1)) for i in o])
        break
    st = sim.stats()
    if s % 5 == 0 or s < 4:
        h = sim.get(["h"])["h"]
        print("step", s, "t", sim.scalars()["ttot"], st, "hmin", h.min(), flush=True)
sim.close()
ctx.close()
