"""Per-step search build and kernel times of Noh -n 300 on one GPU (which search build runs when, and its cost)."""
import sys

sys.path.insert(0, "sph-exa_amd/python")
import sphexa_amd as sx
from sphexa_amd import ic

arrays, lim, bnd, dt0 = ic.noh(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
n = arrays["x"].size
ctx = sx.Context(0)
sim = sx.Sim(ctx, n, sx.make_box(lim, bnd))
sim.set_state(arrays, dt0, dt0)
for s in range(int(sys.argv[2]) if len(sys.argv) > 2 else 12):
    sim.step()
    st, kt = sim.stats(), sim.kernel_times()
    print(s, "build", st["build"], "search %.2f" % kt["findNeighbors"], "momentum %.2f" % kt["momentumEnergy"],
          "stored/t %.1f" % (st["sumNeighbors"] / n), "union/t %.2f" % (st["sumUnion"] / n), "max", st["maxNeighbors"],
          flush=True)
sim.close()
ctx.close()
