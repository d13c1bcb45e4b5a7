"""sx_spatial_groups (computeSpatialGroups, sph/groups.cu:30-47 -> computeGroupSplits<64>,
cstone/traversal/groups.cuh:195-310) on the GPU: bit-exact group boundaries against the oracle restatement, which
tests/test_groups_oracle.py pins to the reference's own known-answer tests (domain/test/unit_cuda/traversal/
groups.cu); the same KATs are also run on the GPU directly."""
import ctypes as C

import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx
from test_groups_oracle import kat_group_volumes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def gpu_groups(ctx, first, last, x, y, z, leaves, layout, obox, tol):
    box = gutil.box_to_sx(obox)
    dx, dy, dz = ctx.upload(np.ascontiguousarray(x)), ctx.upload(np.ascontiguousarray(y)), \
        ctx.upload(np.ascontiguousarray(z))
    dl, dlay = ctx.upload(np.ascontiguousarray(leaves, np.uint64)), ctx.upload(np.ascontiguousarray(layout, np.uint32))
    tree = sx.SxTree(numLeafNodes=leaves.size - 1, leaves=dl.ptr, layout=dlay.ptr)
    cap = last - first + 2
    out = ctx.alloc(cap, np.uint32)
    g = sx.SxGroups()
    ctx.check(ctx.L.sx_spatial_groups(ctx.h, first, last, dx.ptr, dy.ptr, dz.ptr, C.byref(tree), C.byref(box),
                                      float(tol), out.ptr, cap, C.byref(g)), "spatial_groups")
    assert g.firstBody == first and g.lastBody == last
    res = out.get()[:g.numGroups + 1].copy()
    ctx.free_all()
    return res


@pytest.mark.parametrize("factor", [1.01, 0.99])
def test_group_volumes_kat_gpu(ctx, factor):
    first, last, leaves, layout, x, box, dist_crit = kat_group_volumes()
    tol = float(np.float32(np.sqrt(3.0) / dist_crit * factor))
    g = gpu_groups(ctx, first, last, x, x.copy(), x.copy(), leaves, layout, box, tol)
    assert g.tolist() == ([4, 6, 68, 128] if factor > 1 else list(range(first, last + 1)))


@pytest.mark.parametrize("case", ["sedov", "noh", "clustered", "evrard"])
def test_spatial_groups_match_oracle(ctx, ora, case):
    """tolFactor 2 (sph/groups.cu:38) on SFC-sorted states with their converged trees; sub-ranges included"""
    if case == "sedov":
        st, obox = po.sedov_state(24)
    elif case == "noh":
        st, obox = po.noh_state(24)
    elif case == "evrard":
        st, obox = po.evrard_state(20)
    else:
        rng = np.random.default_rng(9)
        n = 30000
        st = po.HostState(n)
        st.x[:] = rng.uniform(-0.5, 0.5, n)
        st.y[:] = rng.uniform(-0.5, 0.5, n)
        st.z[:] = np.clip(rng.normal(0, 0.1, n), -0.5, 0.4999)
        obox = po.make_box(-0.5, 0.5, True)
    gutil.sorted_state(st, obox, ora)
    t = ora.octree(st.keys, 64)
    layout = np.concatenate([[0], np.cumsum(t["counts"])]).astype(np.uint32)
    n = st.n
    for first, last in ((0, n), (37, n - 11), (n // 3, n // 3 + 130)):
        ref = ora.group_splits(first, last, st.x, st.y, st.z, t["leaves"], layout, obox, 2.0)
        got = gpu_groups(ctx, first, last, st.x, st.y, st.z, t["leaves"], layout, obox, 2.0)
        assert np.array_equal(got, ref), (case, first, last, got.size, ref.size)
        assert np.all(np.diff(got) > 0) and np.all(np.diff(got) <= 64)
