"""The oracle's numpy restatement of the block time-step rung bookkeeping (sph/include/sph/ts_rungs.hpp:67-157,
sph/groups.hpp:31-48) on hand-checked cases, and its findRungRanges against the reference's own (compiled into
oracle/_ref).  The rest of ts_rungs.hpp (sortGroupDt, computeMinTimestep, rungTimestep, minimumGroupDt) runs only
on the GPU in the reference: it calls cstone::sortByKeyGpu / sequenceGpu / memcpyD2H, defined in the reference's
CUDA sources, and its host-vector branch leaves minGroupDt unset, so those parts are pinned by the reference text
(cited per line in oracle/pyoracle.py) and by these cases."""
import numpy as np
import pytest

import pyoracle as po


def test_rung_timestep_two_rungs():
    g = np.array([4e-4, 1e-4, 3e-4, 1e-4, 9e-4, 2e-4, 5e-4], np.float32)
    dt, idx, ts = po.rung_timestep(g, 7, 1.0)
    assert np.array_equal(dt, np.sort(g))
    assert list(idx) == [1, 3, 5, 2, 0, 6, 4]  # stable: the two 1e-4 keep their order
    # fast fraction: LocalIndex(0.4f * 7) = 2 -> dt 2e-4, log2(2) = 1 -> 2 rungs
    assert ts["numRungs"] == 2
    assert ts["rungRanges"] == [0, 2, 7, 7, 7]  # lower_bound(2 * 1e-4) = 2
    assert ts["nextDt"] == np.float32(1e-4) and ts["totDt"] == np.float32(1e-4) * np.float32(4)
    assert ts["elapsedDt"] == 0 and ts["substep"] == 0


def test_rung_timestep_caps_and_max_dt():
    g = np.array([1.0, 1e-3] + [1.0] * 8, np.float32)  # 0.4 * 10 = 4 -> dt 1.0: log2(1000) = 9.97 -> capped at 4
    dt, idx, ts = po.rung_timestep(g, 10, 5e-4)
    assert ts["numRungs"] == 4
    assert ts["rungRanges"] == [0, 1, 1, 1, 10]  # ranges use the minimum before min(maxDt, .)
    assert ts["nextDt"] == np.float32(5e-4) and ts["totDt"] == np.float32(5e-4) * np.float32(16)
    assert idx[0] == 1


def test_rung_timestep_single_group():
    dt, idx, ts = po.rung_timestep(np.array([3e-5], np.float32), 1, 1.0)
    assert ts["numRungs"] == 1 and ts["rungRanges"] == [0, 1, 1, 1, 1] and list(idx) == [0]


def test_minimum_group_dt_time_left():
    g = np.array([4e-4, 1e-4, 3e-4, 1e-4, 9e-4, 2e-4, 5e-4], np.float32)
    _, _, ts = po.rung_timestep(g, 7, 1.0)
    ts = dict(ts, substep=1, elapsedDt=np.float32(1e-4))
    act = np.array([2.5e-4, 1.5e-4], np.float32)  # the two rung-0 groups after a substep
    dt, idx, d, rr = po.minimum_group_dt(ts, act, 2)
    assert list(idx) == [1, 0] + list(range(2, 7))  # sequence past the active groups up to rungRanges.back()
    # time left totDt - elapsedDt (float) over 4 - 1 = 3 substeps, below the active minimum 1.5e-4
    left = np.float32(ts["totDt"] - np.float32(1e-4))
    assert d == np.float32(left / np.float32(3)) and d < np.float32(1.5e-4)
    assert rr == [0, 2, 2, 2, 2]


def test_extract_groups():
    gs = np.array([0, 10, 20, 30], np.uint32)
    ge = np.array([10, 20, 30, 35], np.uint32)
    s, e = po.extract_groups(gs, ge, np.array([3, 0, 2, 1], np.uint32), 1, 3)
    assert list(s) == [0, 20] and list(e) == [10, 30]


@pytest.mark.ref
@pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", range(8))
def test_find_rung_ranges_vs_reference(seed):
    """findRungRanges<false> (ts_rungs.hpp:116-130) is host code: compiled from /root/reference into oracle/_ref (with
    the image's MPICH for the header's <mpi.h>) and compared with the restatement on sorted random group time-steps,
    including ties at the 2^r minDt boundaries"""
    import ctypes as C

    ref = C.CDLL(po.REF_SO)
    f = ref.ref_find_rung_ranges
    f.restype = None
    f.argtypes = [C.c_float, C.POINTER(C.c_float), C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 3000))
    dt = np.sort((10.0 ** rng.uniform(-6, -3, n)).astype(np.float32))
    if seed % 2:  # exact multiples of minDt at the rung boundaries
        dt[rng.integers(0, n, n // 4)] = dt[0] * np.float32(2 ** rng.integers(1, 4))
        dt = np.sort(dt)
    for num_rungs in range(1, po.MAX_NUM_RUNGS + 1):
        out = np.zeros(po.MAX_NUM_RUNGS + 1, np.uint32)
        f(float(dt[0]), dt.ctypes.data_as(C.POINTER(C.c_float)), n, num_rungs, out.ctypes.data_as(C.POINTER(C.c_uint32)))
        assert out.tolist() == po.find_rung_ranges(dt[0], dt, n, num_rungs)
