"""CPU restatement of one HydroVeBdtProp substep cycle -- TEST INFRASTRUCTURE ONLY.

The block-time-step VE propagator (`main/src/propagator/ve_hydro_bdt.hpp:51-378`, avClean = false, one rank, no
gravity) on the plain-C oracle (`sph_oracle.c`, pinned bit-for-bit to the reference CPU path) and the numpy rung
bookkeeping of `pyoracle` (restating `ts_rungs.hpp`).  Only tests import this module, as the checker of
`sphexa_amd.ve_bdt.HydroVeBdtProp`; the product path never calls it.

The reference runs this propagator only on GPUs (`:118`), so there is no reference CPU cycle to pin against; every
piece it is built from is pinned on its own (kernels, search and h iteration, spatial groups, positions/drift, group
time-steps: `_ref` and the reference KATs; rung bookkeeping: the reference text, tests/test_rungs_oracle.py).

Semantics restated per substep:
  * full sync (substep 0 of a hierarchy): keys, stable key sort of the conserved fields (+ rung, id), converged
    tree, computeGroupSplits<64> groups (tolFactor 2), groupDt = FLT_MAX, active view = all groups;
  * partial sync: order and tree kept, searchExtFactor *= 1.012, active view = rung-sorted groups
    [rungRanges[0], rungRanges[butterfly(substep)]);
  * each kernel over the view's targets only (the reference's GPU kernels visit only the view's groups): the oracle
    evaluates every target and restores the ones outside the view, which is the same map;
  * the h-nc iteration of the view's targets is the exact neighbor search on the current positions (a target's
    iteration depends only on its own h and the positions; the reference's stale tree + searchExtFactor is meant to
    find the same sets);
  * Courant minimum per view group (momentum_energy_gpu.cu:98-104), groupDivv/groupAcc time-steps per group.
`lists` (optional) supplies the neighbor ORDER of the view's targets (the GPU's exported lists, checked here to hold
exactly the oracle's neighbor sets), so that float sums run in the same order and the cycle can be compared bit for
bit with the exact GPU variant.
"""
import ctypes as C

import numpy as np

import pyoracle as po

MAX_RUNGS = po.MAX_NUM_RUNGS
FLT_MAX = np.float32(np.finfo(np.float32).max)
SORTED = po.CONSERVED + ["rung"]
P = C.c_void_p


def butterfly(i):
    """cstone::butterfly (domain/include/cstone/primitives/math.hpp:27-31)"""
    return 0 if i == 0 else 1 + ((i & -i).bit_length() - 1)


def active_rung(substep, num_rungs):
    """HydroVeBdtProp::activeRung (ve_hydro_bdt.hpp:108-112)"""
    if substep == 0 or substep >= (1 << (num_rungs - 1)):
        return 0
    return butterfly(substep)


def _bind(lib):
    lib.ox_positions_rungs.argtypes = [C.POINTER(po.OxState), P, P, C.c_uint, C.c_float, P, P, C.c_double,
                                       C.POINTER(po.OxBox)]
    lib.ox_drift_positions.argtypes = [C.POINTER(po.OxState), P, P, C.c_uint, C.c_float, C.c_float, P, P, C.c_double]
    lib.ox_group_divv_dt.argtypes = [C.c_float, P, P, C.c_uint, P, P]
    lib.ox_group_acc_dt.argtypes = [C.c_float, P, P, C.c_uint, P, P, P, P]
    return lib


def exact_search(ora, st, box, ngmax, ng0, bucket=64):
    """the oracle's findNeighborsSph with the h-nc iteration on the CURRENT positions of every particle (a key-sorted
    copy, mapped back): returns (h, nc, rows) in the state's own order, rows[i] = sorted neighbor indices of i"""
    tmp = st.copy()
    keys = ora.sfc_keys(tmp, box).copy()
    srt = np.argsort(keys, kind="stable")
    for name in ("x", "y", "z", "h"):
        tmp.arrays[name][:] = st.arrays[name][srt]
    tmp.keys[:] = keys[srt]
    nbr, nc = ora.find_neighbors(tmp, box, bucket=bucket, iterate_h=True, ngmax=ngmax, ng0=ng0)
    n = st.n
    h = np.empty(n, np.float32)
    h[srt] = tmp.h
    ncs = np.empty(n, np.uint32)
    ncs[srt] = nc
    m = nbr.reshape(n, ngmax)
    rows = [None] * n
    for k in range(n):
        c = min(int(nc[k]) - 1, ngmax)
        rows[srt[k]] = np.sort(srt[m[k, :c]].astype(np.uint32))
    return h, ncs, rows


class BdtOracle:
    def __init__(self, ora, st, box, min_dt, params=None, bucket=64, ngmax=150, ng0=100):
        self.ora, self.lib = ora, _bind(ora.lib)
        self.st, self.box, self.bucket = st, box, bucket
        self.p = params or ora.params()
        self.ngmax, self.ng0 = ngmax, ng0
        self.n = st.n
        self.rung = np.zeros(self.n, np.uint8)
        self.ts = dict(nextDt=np.float32(0), elapsedDt=np.float32(0), totDt=np.float32(0), numRungs=1, substep=0,
                       rungRanges=[0] * (MAX_RUNGS + 1), dt_m1=np.zeros(MAX_RUNGS, np.float32),
                       dt_drift=np.zeros(MAX_RUNGS, np.float32))
        self.ts["dt_m1"][0] = np.float32(min_dt)
        self.prev = None
        st.minDt = float(min_dt)
        self.groups = self.ts_groups = None
        self.group_dt = np.zeros(0, np.float32)
        self.group_idx = np.zeros(0, np.uint32)
        self.rungs = [None] * MAX_RUNGS
        self.search_ext = np.float32(1.0)
        self.neighbors = None  # the lists the kernels of the last substep ran on (oracle layout)

    # ---- sync ----------------------------------------------------------------------------------------------
    def _full_sync(self):
        st, ora = self.st, self.ora
        keys = ora.sfc_keys(st, self.box).copy()
        o = np.argsort(keys, kind="stable")
        for k in po.CONSERVED:
            st.arrays[k][:] = st.arrays[k][o]
        self.rung[:] = self.rung[o]
        st.keys[:] = keys[o]
        t = ora.octree(st.keys, self.bucket)
        layout = np.concatenate([[0], np.cumsum(t["counts"])]).astype(np.uint32)
        g = ora.group_splits(0, self.n, st.x, st.y, st.z, t["leaves"], layout, self.box, 2.0)
        self.groups = (g[:-1].copy(), g[1:].copy())
        self.active = self.groups
        self.group_dt = np.full(self.groups[0].size, FLT_MAX, np.float32)
        self.group_idx = np.zeros(self.groups[0].size, np.uint32)
        self.search_ext = np.float32(1.0)

    def _partial_sync(self):
        self.search_ext = np.float32(np.float64(self.search_ext) * 1.012)
        hr = butterfly(self.ts["substep"])
        rr = self.ts["rungRanges"]
        self.active = (self.ts_groups[0][rr[0]:rr[hr]], self.ts_groups[1][rr[0]:rr[hr]])

    def active_mask(self, view=None):
        gs, ge = self.active if view is None else view
        act = np.zeros(self.n, bool)
        for s, e in zip(gs, ge):
            act[s:e] = True
        return act

    # ---- computeForces -------------------------------------------------------------------------------------
    def compute_forces(self, lists=None):
        """lists(oracle, act, rows) -> the view's neighbor lists (n x ngmax, oracle layout) or None for the oracle's
        own sorted rows"""
        if active_rung(self.ts["substep"], self.ts["numRungs"]) == 0:
            self._full_sync()
        else:
            self._partial_sync()
        st, ora, box, p = self.st, self.ora, self.box, self.p
        gs, ge = self.active
        act = self.active_mask()
        h, nc, rows = exact_search(ora, st, box, self.ngmax, self.ng0, self.bucket)
        st.h[act] = h[act]
        st.nc[act] = nc[act]
        self.rows, self.act = rows, act
        nbr = lists(self, act, rows) if lists is not None else None
        if nbr is not None:
            # the kernels below run over every target and keep only the active ones; an external list holds
            # whatever an earlier search left for inactive targets (indices possibly beyond n), so those rows get
            # the oracle's own in-range rows before the C oracle reads them
            nbr = nbr.copy()
            m = nbr.reshape(-1, self.ngmax)
            for i in np.nonzero(~act)[0]:
                r = rows[i]
                m[i] = 0
                m[i, :r.size] = r
        else:
            nbr = np.zeros(self.n * self.ngmax, np.uint32)
            for i in np.nonzero(act)[0]:
                r = rows[i]
                nbr[i * self.ngmax:i * self.ngmax + r.size] = r
        self.neighbors = nbr
        for name, fields in (("xmass", ["xm"]), ("ve_def_gradh", ["kx", "gradh"])):
            self._view_kernel(name, fields, nbr, act)
        ora.eos(st, params=p)  # computeEOS(first, last): every target
        self._view_kernel("iad_divv_curlv", ["c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv"], nbr, act)
        ng = np.uint32(gs.size)
        self.lib.ox_group_divv_dt(np.float32(p.Krho), gs.ctypes.data, ge.ctypes.data, ng, st.divv.ctypes.data,
                                  self.group_dt.ctypes.data)
        self._view_kernel("av_switches", ["alpha"], nbr, act)
        before = st.copy()
        self._view_kernel("momentum_energy", ["du", "ax", "ay", "az"], nbr, act)
        for k, (s, e) in enumerate(zip(gs, ge)):  # Courant minimum per view group, min with the previous value
            tmp = before.copy()
            dt = ora.momentum_energy(tmp, box, nbr[int(s) * self.ngmax:int(e) * self.ngmax], int(s), int(e),
                                     params=p)
            self.group_dt[k] = min(self.group_dt[k], np.float32(dt))
        eta = np.float32(np.float64(p.etaAcc) * np.sqrt(np.float64(p.eps)))
        self.lib.ox_group_acc_dt(eta, gs.ctypes.data, ge.ctypes.data, ng, st.ax.ctypes.data, st.ay.ctypes.data,
                                 st.az.ctypes.data, self.group_dt.ctypes.data)

    def _view_kernel(self, name, fields, nbr, act):
        st = self.st
        keep = {k: st.arrays[k].copy() for k in fields}
        getattr(self.ora, name)(st, self.box, nbr, params=self.p)
        for k in fields:
            st.arrays[k][~act] = keep[k][~act]

    # ---- computeRungs --------------------------------------------------------------------------------------
    def compute_rungs(self):
        ts = self.ts
        high = active_rung(ts["substep"], ts["numRungs"])
        if high == 0:
            self.prev = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in ts.items()}
            max_dt = np.float32(np.float64(ts["dt_m1"][0]) * np.float64(self.p.maxDtIncrease))
            ng = self.groups[0].size
            dt, idx, new = po.rung_timestep(self.group_dt, ng, max_dt)
            self.group_dt[:ng] = dt[:ng]
            self.group_idx[:idx.size] = idx
            new.update(dt_m1=np.zeros(MAX_RUNGS, np.float32), dt_drift=np.zeros(MAX_RUNGS, np.float32))
            self.ts = ts = new
        else:
            num = ts["rungRanges"][high]
            dt_sorted, idx, dt, rr = po.minimum_group_dt(ts, self.group_dt, num)
            self.group_dt[:num] = dt_sorted[:num]
            self.group_idx[:idx.size] = idx
            ts["nextDt"] = np.float32(dt)
            for r in range(high):
                ts["rungRanges"][r] = rr[r]
        if high == 0 or high > 1:
            if high > 1:
                self.groups, self.ts_groups = self.ts_groups, self.groups
            self.ts_groups = po.extract_groups(self.groups[0], self.groups[1], self.group_idx, 0,
                                               ts["rungRanges"][MAX_RUNGS])
        rr = ts["rungRanges"]
        for r in range(ts["numRungs"]):
            self.rungs[r] = (self.ts_groups[0][rr[r]:rr[r + 1]].copy(), self.ts_groups[1][rr[r]:rr[r + 1]].copy())

    # ---- integrate -----------------------------------------------------------------------------------------
    def integrate(self):
        self.compute_rungs()
        ts, st, lib, f32 = self.ts, self.st, self.lib, np.float32
        lowest_drift = butterfly(ts["substep"] + 1)
        last_substep = active_rung(ts["substep"] + 1, ts["numRungs"]) == 0
        sub_box = self.box if last_substep else po.make_box(0.0, 1.0, False)
        cv = float(po.ideal_gas_cv(np.float32(self.p.muiConst), self.p.gamma))
        rp = self.rung.ctypes.data
        for i in range(ts["numRungs"]):
            use_rung = ts["substep"] == ts["substep"] % (1 << i)
            advance = i < lowest_drift
            dt = f32(ts["nextDt"])
            dt_m1 = np.ascontiguousarray((self.prev if use_rung else ts)["dt_m1"], np.float32)
            gs, ge = self.rungs[i]
            ng = gs.size
            s = st.struct()
            if advance:
                if ts["dt_drift"][i] > 0 and ng:
                    lib.ox_drift_positions(C.byref(s), gs.ctypes.data, ge.ctypes.data, ng, f32(0),
                                           f32(ts["dt_drift"][i]), dt_m1.ctypes.data, rp, cv)
                if ng:
                    lib.ox_positions_rungs(C.byref(s), gs.ctypes.data, ge.ctypes.data, ng,
                                           f32(f32(ts["dt_drift"][i]) + dt), dt_m1.ctypes.data, rp, cv,
                                           C.byref(sub_box))
                ts["dt_m1"][i] = f32(f32(ts["dt_drift"][i]) + dt)
                ts["dt_drift"][i] = f32(0)
                for a, b in zip(gs, ge):
                    self.rung[a:b] = i
            else:
                if ng:
                    lib.ox_drift_positions(C.byref(s), gs.ctypes.data, ge.ctypes.data, ng,
                                           f32(f32(ts["dt_drift"][i]) + dt), f32(ts["dt_drift"][i]),
                                           dt_m1.ctypes.data, rp, cv)
                ts["dt_drift"][i] = f32(f32(ts["dt_drift"][i]) + dt)
        for a, b in zip(*self.active):
            self.ora.update_h_range(st, self.ng0, int(a), int(b))
        ts["substep"] += 1
        ts["elapsedDt"] = f32(f32(ts["elapsedDt"]) + f32(ts["nextDt"]))
        st.ttot += float(f32(ts["nextDt"]))
        st.minDt_m1 = st.minDt
        st.minDt = float(f32(ts["nextDt"]))

    def step(self, lists=None):
        self.compute_forces(lists)
        self.integrate()
