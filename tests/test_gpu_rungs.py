"""Block time-step rung bookkeeping through the C-ABI (sx_rung_timestep, sx_minimum_group_dt, sx_extract_groups)
against the oracle's restatement of sph/include/sph/ts_rungs.hpp:67-157 and sph/groups.hpp:31-48: sorted group
time-steps, the permutation, numRungs, rungRanges, nextDt / totDt and the substep dt all bit-identical."""
import ctypes as C

import numpy as np
import pytest

import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


def group_dts(n, seed, spread):
    """Courant-like group time-steps: log-uniform over `spread` decades, with ties and FLT_MAX (untouched groups)"""
    rng = np.random.default_rng(seed)
    g = (1e-4 * 10.0 ** (spread * rng.random(n))).astype(np.float32)
    if n > 8:
        g[rng.integers(0, n, n // 8)] = g[0]  # ties: the stable order must match
        g[rng.integers(0, n, n // 50 + 1)] = np.finfo(np.float32).max
    return g


@pytest.mark.parametrize("n,seed,spread", [(1, 0, 1.0), (7, 1, 0.5), (1000, 2, 1.5), (65537, 3, 0.8),
                                           (300000, 4, 3.0)])
def test_rung_timestep_and_substeps(ctx, n, seed, spread):
    L, h = ctx.L, ctx.h
    g = group_dts(n, seed, spread)
    max_dt = np.float32(np.median(g) if seed % 2 else 1.0)
    dg, di = ctx.upload(g), ctx.alloc(n, np.uint32)
    ts = sx.SxTimestep()
    ctx.check(L.sx_rung_timestep(h, dg.ptr, di.ptr, n, max_dt, None, C.byref(ts)), "rung timestep")
    rdt, ridx, rts = po.rung_timestep(g, n, max_dt)
    assert np.array_equal(dg.get(), rdt)
    assert np.array_equal(di.get(), ridx)
    assert ts.numRungs == rts["numRungs"] and list(ts.rungRanges) == rts["rungRanges"]
    assert np.float32(ts.nextDt) == rts["nextDt"] and np.float32(ts.totDt) == rts["totDt"]
    assert ts.substep == 0 and ts.elapsedDt == 0.0

    # a substep: the groups of the lowest rungs get new time-steps, minimumGroupDt over them
    rng = np.random.default_rng(seed + 10)
    for sub in (1, 2):
        if sub >= (1 << ts.numRungs):  # the hierarchy ends there (the next step computes new rungs)
            break
        hi = min(sub, ts.numRungs)
        na = rts["rungRanges"][hi] or n
        act = (np.float32(rts["nextDt"]) * (0.5 + 3 * rng.random(na))).astype(np.float32)
        ts.substep, ts.elapsedDt = sub, np.float32(sub * rts["nextDt"])
        rts2 = dict(rts, substep=sub, elapsedDt=np.float32(sub * rts["nextDt"]))
        dg.set(np.concatenate([act, g[na:]]))
        dt = C.c_float()
        rr = (C.c_uint32 * 5)()
        ctx.check(L.sx_minimum_group_dt(h, C.byref(ts), dg.ptr, di.ptr, na, None, C.byref(dt), rr), "minimumGroupDt")
        rdt2, ridx2, rd, rrr = po.minimum_group_dt(rts2, np.concatenate([act, g[na:]]), na)
        assert np.array_equal(dg.get()[:na], rdt2[:na])
        assert np.array_equal(di.get()[:rts["rungRanges"][4]], ridx2)
        assert np.float32(dt.value) == rd and list(rr) == rrr


def test_extract_groups(ctx):
    rng = np.random.default_rng(7)
    b = np.concatenate([[0], np.cumsum(rng.integers(1, 65, 5000))]).astype(np.uint32)
    gs, ge = b[:-1].copy(), b[1:].copy()
    idx = rng.permutation(gs.size).astype(np.uint32)
    db, di = ctx.upload(np.concatenate([gs, ge])), ctx.upload(idx)
    grp = sx.SxGroups(firstBody=0, lastBody=int(b[-1]), numGroups=gs.size, groupStart=db.ptr,
                      groupEnd=db.ptr + 4 * gs.size)
    first, last = 100, 4321
    os_, oe = ctx.alloc(last - first, np.uint32), ctx.alloc(last - first, np.uint32)
    ctx.check(ctx.L.sx_extract_groups(ctx.h, C.byref(grp), di.ptr, first, last, os_.ptr, oe.ptr), "extract")
    rs, re_ = po.extract_groups(gs, ge, idx, first, last)
    assert np.array_equal(os_.get(), rs) and np.array_equal(oe.get(), re_)
    # fixed 64-blocks (groupStart NULL): group j = [64 j, min(64 j + 64, lastBody))
    g64 = sx.SxGroups(firstBody=0, lastBody=1000, numGroups=16)
    i2 = ctx.upload(np.array([15, 0, 3], np.uint32))
    a, e = ctx.alloc(3, np.uint32), ctx.alloc(3, np.uint32)
    ctx.check(ctx.L.sx_extract_groups(ctx.h, C.byref(g64), i2.ptr, 0, 3, a.ptr, e.ptr), "extract 64")
    assert list(a.get()) == [960, 0, 192] and list(e.get()) == [1000, 64, 256]
