"""Full-size property test on the metric's own configuration: Sedov -n 400 (64M particles) on ONE MI355X.

The oracle cannot run 64M particles in test time, so this checks size-independent properties of the GPU path on
the full problem (BASELINE.json metric, `main/src/init/sedov_init.hpp:106-130` IC):
  * every particle of the periodic lattice has the same neighborhood: nc == 93 (92 neighbors + self, the value the
    oracle gives at n=50, test_gpu_parity.py::test_sedov_n50_energy_and_counts) after the first step's h iteration,
  * no search capacity error, no non-converged h, ids remain a permutation of 0..n-1 after two SFC re-sorts,
  * total energy (computeConservedQuantities) drifts < 1e-6 over two steps.
"""
import numpy as np
import pytest

import sphexa_amd as sx

pytestmark = pytest.mark.gpu

SIDE = 400


def test_sedov_n400_two_steps_one_gpu():
    n = SIDE ** 3
    ctx = sx.Context(0)
    box = sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1])
    sim = sx.Sim(ctx, n, box)
    try:
        sim.init_sedov(SIDE)
        e0 = sim.conserved()
        sim.step()
        st = sim.stats()
        assert st["numFailed"] == 0
        nc = sim.get(["nc"])["nc"]
        vals, cnts = np.unique(nc, return_counts=True)
        assert np.array_equal(vals, [93]), dict(zip(vals.tolist(), cnts.tolist()))
        assert st["sumNeighbors"] == 92 * n and st["maxNeighbors"] == 92
        sim.step()
        e2 = sim.conserved()
        assert abs(e2["etot"] / e0["etot"] - 1) < 1e-6, (e0, e2)
        ids = np.sort(sim.get(["id"])["id"])
        assert np.array_equal(ids, np.arange(n, dtype=np.uint64))
        h = sim.get(["h"])["h"]
        assert np.all(np.isfinite(h)) and np.all(h > 0)
    finally:
        sim.close()
        ctx.close()
