"""Target groups (computeGroupSplits<64>, cstone/traversal/groups.cuh:55-310, caller sph/groups.cu:30-47) in the
oracle, pinned by the reference's own known-answer tests (domain/test/unit_cuda/traversal/groups.cu) restated for
the 64-wide wavefront (GpuConfig::warpSize = 64 on AMD: one 64-bit split mask per fixed group).  The reference
implements this seam only for the GPU (its CPU path uses one group, sph/groups.hpp:24-28), so these KATs are the
pin: no oracle/_ref build exists for it."""
import numpy as np
import pytest

import pyoracle as po


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def test_make_splits_kat(ora):
    """TEST(TargetGroups, makeSplits), groups.cu:136-213 (masks given as (low, high) 32-bit halves)"""
    m = lambda lo, hi: (hi << 32) + lo
    assert ora.make_splits(m(0, 0)) == [64]
    assert ora.make_splits(m(1, 0)) == [1, 63]
    assert ora.make_splits(m(0, 1 << 30)) == [63, 1]
    assert ora.make_splits(m(2, 0)) == [2, 62]
    assert ora.make_splits(m(3, 0)) == [1, 1, 62]
    assert ora.make_splits(m(1 << 31, 1)) == [32, 1, 31]
    assert ora.make_splits(m(0, 8)) == [36, 28]
    r = ora.make_splits(m(0xFFFFFFFF, 0x6FFFFFFF))
    assert all(v == (2 if i == 60 else 1) for i, v in enumerate(r[:63]))
    assert ora.make_splits(m(0xFFFFFFFF, 0x7FFFFFFF))[:63] == [1] * 63


def kat_tree():
    """OctreeMaker<uint64_t>{}.divide().divide(2).makeTree() (groups.cu:223): 8 level-1 octants, octant 2 split"""
    L1, L2 = 8 ** 20, 8 ** 19
    leaves = [k * L1 for k in range(3)] + [2 * L1 + c * L2 for c in range(1, 8)] + [k * L1 for k in range(3, 9)]
    return np.array(leaves, np.uint64)


def kat_group_volumes():
    """inputs of TEST(TargetGroups, groupVolumes), groups.cu:215-293"""
    first, last = 4, 128
    leaves = kat_tree()
    counts = [4, 1, 8, 8, 8, 8, 31, 8, 8, 8, 16, 16, 16, 0, 0]
    layout = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    x = np.arange(last, dtype=np.float64)
    x[5] -= 0.01  # split between particles 5 and 6
    box = po.make_box(0.0, float(last), True)
    dist_crit = np.cbrt(128.0 ** 3 / 64)
    return first, last, leaves, layout, x, box, dist_crit


@pytest.mark.parametrize("factor", [1.01, 0.99])
def test_group_volumes_kat(ora, factor):
    """15 leaves, particles on the diagonal of a [0,128]^3 box; tolFactor just above / below the spacing"""
    first, last, leaves, layout, x, box, dist_crit = kat_group_volumes()
    tol = float(np.float32(np.sqrt(3.0) / dist_crit * factor))
    g = ora.group_splits(first, last, x, x.copy(), x.copy(), leaves, layout, box, tol)
    if factor > 1:
        assert g.tolist() == [4, 6, 68, 128]  # EXPECT groups {4, 6, 68, 128} (groupDiv {2, 1})
    else:
        assert g.tolist() == list(range(first, last + 1))  # groupDiv {64, 60}: every pair splits


def test_find_splits_kat(ora):
    """TEST(TargetGroups, findSplits), groups.cu:69-118: splits exactly at lanes 0, 31 and 33 (distCritSq 3.01 on
    unit-spaced diagonal points), through one 64-particle fixed group in a unit box with a single level-0 leaf"""
    n = 64
    x = np.arange(n, dtype=np.float64)
    y, z = x.copy(), x.copy()
    x[0] = y[0] = z[0] = -1.0
    for l in (31, 33):
        x[l] -= 0.5
        y[l] -= 0.5
        z[l] -= 0.5
    leaves = np.array([0, 8 ** 21], np.uint64)
    layout = np.array([0, n], np.uint32)
    box = po.make_box(0.0, 1.0, True)
    g = ora.group_splits(0, n, x, y, z, leaves, layout, box, float(np.float32(np.sqrt(3.01))))
    assert g.tolist() == [0, 1, 32, 34, 64]  # splits after lanes 0, 31, 33
