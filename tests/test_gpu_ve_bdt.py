"""Block time-steps end to end: sphexa_amd.ve_bdt.HydroVeBdtProp (the ve-bdt propagator, ve_hydro_bdt.hpp:51-378,
driven through the C-ABI seam on the GPU) against oracle/bdt_oracle.py (the same cycle on the CPU oracle).

Exact variant, lockstep over whole hierarchies (full syncs, partial syncs with drifting inactive rungs, rung
re-sorting with extractGroupGpu, the last substep's periodic wrap): after every computeForces the search of the
active view must hold exactly the oracle's neighbor sets and h/nc, and every field, groupDt, and after every
integrate the conserved fields, rungs and the Timestep, must be bit-identical.  The oracle sums each target's
neighbors in the GPU list's order (sets checked first), so float sums agree bit for bit.

Fast variant (the production cluster kernels): the same cycle over a hierarchy conserves energy to float rounding
and reproduces the exact run's rung structure.
"""
import ctypes as C

import numpy as np
import pytest

import bdt_oracle as bo
import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx
from sphexa_amd.ve_bdt import HydroVeBdtProp

pytestmark = pytest.mark.gpu
NGMAX = 150
FIELDS = ["h", "nc", "xm", "kx", "gradh", "prho", "c", "c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv",
          "alpha", "du", "ax", "ay", "az"]
CONS = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


def initial(ic, side, ora):
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    po.converge_h(ora, st, box)
    return st, box


def view_groups(ctx, v):
    n = v.numGroups
    if n == 0:
        return np.zeros(0, np.uint32), np.zeros(0, np.uint32)
    s, e = np.empty(n, np.uint32), np.empty(n, np.uint32)
    ctx.check(ctx.L.sx_memcpy(ctx.h, s.ctypes.data, v.groupStart, 4 * n, 2), "view")
    ctx.check(ctx.L.sx_memcpy(ctx.h, e.ctypes.data, v.groupEnd, 4 * n, 2), "view")
    return s, e


class Exporter:
    """on_search hook: the GPU's neighbor lists of the active view, in the oracle's layout"""

    def __init__(self, ctx):
        self.ctx, self.lists = ctx, None

    def __call__(self, prop, v):
        ctx = self.ctx
        gs, ge = view_groups(ctx, v)
        n = prop.n
        full = np.zeros(n * NGMAX, np.uint32)
        if gs.size:
            a, b = int(gs.min()), int(ge.max())
            out = ctx.alloc((b - a) * NGMAX, np.uint32)
            ctx.check(ctx.L.sx_export_neighbors(ctx.h, prop.fields.nc, a, b, NGMAX, out.ptr), "export")
            full[a * NGMAX:b * NGMAX] = out.get()
        self.lists, self.nc, self.view = full, prop.get("nc"), (gs, ge)

    def provide(self, orc, act, rows):
        gs, ge = self.view
        got = orc.active_mask((gs, ge))
        assert np.array_equal(got, act), "active view differs"
        m = self.lists.reshape(-1, NGMAX)
        for i in np.nonzero(act)[0]:
            c = min(int(self.nc[i]) - 1, NGMAX)
            assert np.array_equal(np.sort(m[i, :c]), rows[i]), ("neighbor set", int(i))
        return self.lists


def compare(prop, orc, names, what):
    st = orc.st
    for k in names:
        g = prop.get(k)
        r = st.arrays[k] if k in st.arrays else None
        assert np.array_equal(g, r.astype(g.dtype)), (what, k, int(np.sum(g != r)))


@pytest.mark.parametrize("ic,side,substeps,min_rungs", [("sedov", 14, 12, 3), ("noh", 14, 10, 2)])
def test_ve_bdt_cycle_exact_bitwise(ctx, ic, side, substeps, min_rungs):
    ora = po.load_oracle()
    st, obox = initial(ic, side, ora)
    host = {k: st.arrays[k].copy() for k in CONS}
    ctx.set_exact(True)
    try:
        prop = HydroVeBdtProp(ctx, host, gutil.box_to_sx(obox), st.minDt)
        ex = Exporter(ctx)
        prop.on_search = ex
        orc = bo.BdtOracle(ora, st.copy(), obox, st.minDt)
        partial = 0
        for s in range(substeps):
            synced = prop.is_synced()
            partial += not synced
            prop.compute_forces()
            orc.compute_forces(lists=ex.provide)
            compare(prop, orc, FIELDS, f"forces {s}")
            ng = prop.groups.num if synced else None
            gdt = prop.group_dt.get()[:orc.group_dt.size]
            assert np.array_equal(gdt, orc.group_dt), ("groupDt", s, ng)
            prop.integrate()
            orc.integrate()
            compare(prop, orc, CONS, f"integrate {s}")
            assert np.array_equal(prop.get("rung"), orc.rung), ("rung", s)
            ts = prop.ts
            assert ts.numRungs == orc.ts["numRungs"] and ts.substep == orc.ts["substep"]
            assert list(ts.rungRanges) == list(orc.ts["rungRanges"])
            assert np.float32(ts.nextDt) == orc.ts["nextDt"]
            assert np.array_equal(np.array(ts.dt_m1[:], np.float32), orc.ts["dt_m1"])
            assert np.array_equal(np.array(ts.dt_drift[:], np.float32), orc.ts["dt_drift"])
        assert partial > 0, "no partial substep ran: the hierarchy had a single rung"
        assert max(e["numRungs"] for e in prop.log) >= min_rungs  # Noh 14^3 (1472 particles): two rungs
    finally:
        ctx.set_exact(False)
        ctx.free_all()


def test_ve_bdt_fast_hierarchy(ctx):
    """production kernels: two hierarchies of Sedov, total energy conserved, rung structure of the exact run"""
    ora = po.load_oracle()
    st, obox = initial("sedov", 16, ora)
    host = {k: st.arrays[k].copy() for k in CONS}
    e0 = po.total_energy(st)
    runs = {}
    for exact in (True, False):
        ctx.set_exact(exact)
        prop = HydroVeBdtProp(ctx, host, gutil.box_to_sx(obox), st.minDt)
        hier = 0
        while hier < 2:
            prop.step()
            hier += prop.is_synced()
        runs[exact] = prop
        g = {k: prop.get(k) for k in ("vx", "vy", "vz", "m", "temp")}
        v2 = sum(g[k].astype(np.float64) ** 2 for k in ("vx", "vy", "vz"))
        e = np.sum(0.5 * g["m"] * v2) + np.sum(g["m"] * np.float64(po.ideal_gas_cv()) * g["temp"])
        assert abs(e / e0 - 1) < 1e-6, (exact, e / e0 - 1)
    ctx.set_exact(False)
    a, b = runs[True], runs[False]
    assert [e["numRungs"] for e in a.log] == [e["numRungs"] for e in b.log]
    ia, ib = a.get("id"), b.get("id")
    oa, ob = np.argsort(ia), np.argsort(ib)
    assert np.array_equal(ia[oa], ib[ob])
    for k in ("x", "y", "z"):
        assert np.max(np.abs(a.get(k)[oa] - b.get(k)[ob])) < 1e-6, k
    ctx.free_all()
