"""The two neighbor-search builds and the device-side fallback between them (sx_neighbors.hip findNeighbors).

The compact build (four workgroups per CU) runs first; a cluster that exceeds its capacities is left unwritten (h,
nc, lists, union) and listed, and the large build then redoes exactly the listed clusters, without a host sync.
All paths must give bit-identical h, nc, neighbor lists, union sizes and statistics:
  mode 1 large only, mode 2 compact (on Noh some sphere-surface clusters go to the large build), mode 3 compact
  with a forced overflow of every cluster (every cluster redone by the large build from the untouched h), with the
  h-nc iteration on, on inputs where it actually iterates (h0 far from the converged value), plus the reference
  oracle's sets as the anchor.
"""
import ctypes as C

import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


def search(ctx, st, obox, mode, h0):
    box = gutil.box_to_sx(obox)
    n = st.n
    host = gutil.host_dict(st)
    host["h"] = h0.copy()
    ds = sx.DeviceState(ctx, host)
    tree, _ = gutil.device_tree(ctx, ds.dev["keys"], n, 64, box)
    p = sx.default_params()
    stats = sx.SxNbStats()
    ctx.check(ctx.L.sx_set_search_mode(ctx.h, mode), "mode")
    rc = ctx.L.sx_find_neighbors(ctx.h, C.byref(ds.fields), C.byref(tree), C.byref(box), C.byref(p), 0, n, 1,
                                 C.byref(stats))
    ctx.check(ctx.L.sx_set_search_mode(ctx.h, 0), "mode")
    assert rc == sx.SX_OK, ctx.L.sx_last_error(ctx.h)
    nc, h = ds.get("nc"), ds.get("h")
    out = ctx.alloc(n * 150, np.uint32)
    ctx.check(ctx.L.sx_export_neighbors(ctx.h, ds.dev["nc"].ptr, 0, n, 150, out.ptr), "export")
    nbr = out.get().reshape(n, 150)
    ctx.free_all()
    return dict(nc=nc, h=h, nbr=nbr, sum=stats.sumNeighbors, max=stats.maxNeighbors, failed=stats.numFailed,
                union=stats.sumUnion, cand=stats.sumCandidates, build=stats.build)


@pytest.mark.parametrize("case", ["sedov", "noh"])
def test_builds_and_fallback_identical(ctx, case):
    ora = po.load_oracle()
    if case == "sedov":
        st, obox = po.sedov_state(26)
    else:
        st, obox = po.noh_state(26)
    gutil.sorted_state(st, obox, ora)
    h0 = (st.h * np.float32(1.35)).astype(np.float32)  # ~2.5x the neighbors: the h-nc iteration runs
    big = search(ctx, st, obox, 1, h0)
    small = search(ctx, st, obox, 2, h0)
    fb = search(ctx, st, obox, 3, h0)
    assert big["build"] == 1 and fb["build"] == 2 and small["build"] in ((0,) if case == "sedov" else (0, 2))
    assert not np.array_equal(big["h"], h0)  # the iteration changed h
    for other in (small, fb):
        assert np.array_equal(other["h"], big["h"])
        assert np.array_equal(other["nc"], big["nc"])
        assert np.array_equal(other["nbr"], big["nbr"])  # same lists, same (stream) order
        for k in ("sum", "max", "failed", "union", "cand"):
            assert other[k] == big[k], k
    # anchor: the reference's h-nc iteration and neighbor sets
    ref = st.copy()
    ref.h[:] = h0
    rn, rnc = ora.find_neighbors(ref, obox, iterate_h=True)
    assert np.array_equal(big["h"], ref.h) and np.array_equal(big["nc"], rnc)
    a = gutil.rows_sorted(big["nbr"].ravel(), big["nc"], 150)
    b = gutil.rows_sorted(rn, rnc, 150)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
