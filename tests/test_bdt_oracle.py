"""CPU checks of the block time-step cycle restatement (oracle/bdt_oracle.py) and of the host helpers of
sphexa_amd.ve_bdt (no GPU calls).

* butterfly / activeRung reproduce cstone::butterfly's 1 2 1 3 1 2 1 4 pattern (primitives/math.hpp:26-31) and the
  hierarchy boundaries of ve_hydro_bdt.hpp:108-112;
* a Sedov run through one and a half hierarchies: the hierarchy has several rungs, a substep touches only the
  active rungs' particles, every rung has been kicked (no pending drift) at the end of a hierarchy, h/nc of
  inactive particles are untouched on partial substeps, energy is conserved.
"""
import numpy as np

import bdt_oracle as bo
import pyoracle as po
from sphexa_amd import ve_bdt


def test_butterfly_and_active_rung():
    want = [0, 1, 2, 1, 3, 1, 2, 1, 4, 1, 2, 1, 3]
    assert [bo.butterfly(i) for i in range(13)] == want
    assert [ve_bdt.butterfly(i) for i in range(13)] == want
    for nr in range(1, 5):
        for s in range(20):
            assert bo.active_rung(s, nr) == ve_bdt.active_rung(s, nr)
            if s == 0 or s >= 1 << (nr - 1):
                assert bo.active_rung(s, nr) == 0
    assert ve_bdt.sliced(ve_bdt.Groups(4096, 8192, 10, 0, 0).view(), 3, 7).groupStart == 4096 + 12


def test_oracle_cycle_sedov():
    ora = po.load_oracle()
    st, box = po.sedov_state(14)
    po.converge_h(ora, st, box)
    e0 = po.total_energy(st)
    o = bo.BdtOracle(ora, st, box, st.minDt)
    o.step()  # new hierarchy: every group active
    assert o.act.all()
    nr = o.ts["numRungs"]
    assert nr >= 3
    for s in range(1, 1 << (nr - 1)):
        h0, nc0 = st.h.copy(), st.nc.copy()
        o.step()
        act = o.act
        assert 0 < act.sum() < st.n
        # the h-nc iteration and updateH touch only the active rungs
        assert np.array_equal(st.h[~act], h0[~act]) and np.array_equal(st.nc[~act], nc0[~act])
    assert o.ts["substep"] == 1 << (nr - 1)
    assert np.all(o.ts["dt_drift"][:nr] == 0)  # every rung kicked at the hierarchy's end
    o.step()
    assert o.act.all()  # next hierarchy: full sync
    assert abs(po.total_energy(st) / e0 - 1) < 1e-7
