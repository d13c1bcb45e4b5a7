"""HydroVeBdtProp on one GPU: the VE propagator with block time-steps, driven through the C-ABI seam.

Mirror of `main/src/propagator/ve_hydro_bdt.hpp:51-378` on one rank (avClean and self-gravity included): the reference's
host control flow -- full/partial syncs, the rung hierarchy, the substep drift/kick cycle -- calling the HIP
kernels of libsphexa_hip.so through the same seam functions the reference's propagator calls (`sph_gpu.hpp`):

  computeForces  (:222-290)  sync; computeXMass(activeRungs) [search + h-nc iteration on the view]; VeDefGradh;
                             computeEOS(first, last); IAD+divv/curlv; groupDivvTimestep; AV switches;
                             momentum/energy (Courant per view group into groupDt); self-gravity (upsweep + traversal of
                             gravGroup: every target on a new hierarchy, else the active view); groupAccTimestep
  computeRungs   (:292-331)  rungTimestep on a new hierarchy, minimumGroupDt on a substep; extractGroupGpu
  integrate      (:333-378)  per rung: drift, or drift back + computePositions + storeRung; updateSmoothingLength

A full sync (substep 0 of a hierarchy) is the single-rank `Domain::sync`: SFC keys, stable key sort and the gather
of the conserved fields (x, y, z, h, m, temp, v, x_m1, du_m1, alpha, rung and the particle id), the converged
cornerstone tree + linked octree + node geometry, then computeSpatialGroups (`groups.cu:30-47`).  A partial sync
keeps order and tree and grows `searchExtFactor` by 1.012 (:196-211).  Everything stays on the device; the host
sees the group count, the rung ranges and the time-step scalars, as in the reference.

The product path is the HIP library: nothing here computes particle data on the CPU.  The production driver is the
native one (sx_sim with propagator 2, sph-exa_amd/csrc/sx_bdt.cpp); this one stays as its bit-for-bit reference
(tests/test_gpu_ve_bdt_native.py) and as the seam-level mirror the CPU oracle is checked against.
"""
import ctypes as C

import numpy as np

from . import (SX_OK, DTYPES, FIELD_ORDER, SxBox, SxError, SxFields, SxGroups, SxOctree, SxTimestep, SxTree,
               default_params)

MAX_RUNGS = 4  # sph::Timestep::maxNumRungs (sph/timestep.h:19)
FLT_MAX = np.float32(np.finfo(np.float32).max)
# Domain::sync reorders these (x, y, z, h, m + ConservedFields of ve_hydro_bdt.hpp:94) and the particle id
CONSERVED = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "rung",
             "id"]
DEPENDENT = ["ax", "ay", "az", "prho", "c", "du", "c11", "c12", "c13", "c22", "c23", "c33", "xm", "kx", "nc", "divv",
             "curlv", "gradh", "keys"]
GRAD_V = ["dV11", "dV12", "dV13", "dV22", "dV23", "dV33"]  # GradVFields of HydroVeBdtProp<avClean = true>
DT = dict(DTYPES, id=np.uint64)


def butterfly(i):
    """cstone::butterfly (primitives/math.hpp:27-31): 0 for 0, else 1 + count of trailing zeros"""
    if i == 0:
        return 0
    return 1 + ((i & -i).bit_length() - 1)


def active_rung(substep, num_rungs):
    """HydroVeBdtProp::activeRung (ve_hydro_bdt.hpp:108-112)"""
    if substep == 0 or substep >= (1 << (num_rungs - 1)):
        return 0
    return butterfly(substep)


class Groups:
    """GroupData: device groupStart/groupEnd (+ host copies for the host decisions), firstBody/lastBody"""

    def __init__(self, start, end, num, first_body, last_body, keep=()):
        self.start, self.end, self.num = start, end, int(num)
        self.first_body, self.last_body = first_body, last_body
        self.keep = keep  # device arrays that own start/end

    def view(self):
        return SxGroups(firstBody=self.first_body, lastBody=self.last_body, numGroups=self.num,
                        groupStart=self.start, groupEnd=self.end)


def sliced(v, first, last):
    """makeSlicedView (sph/groups.hpp:51-58)"""
    return SxGroups(firstBody=v.firstBody, lastBody=v.lastBody, numGroups=int(last) - int(first),
                    groupStart=(v.groupStart or 0) + 4 * int(first), groupEnd=(v.groupEnd or 0) + 4 * int(first))


class HydroVeBdtProp:
    """one block-time-step substep per `step()`; `state` holds the device fields (SxFields) and `ts` the Timestep"""

    def __init__(self, ctx, host, box, min_dt, params=None, bucket=64, min_dt_m1=None):
        """host: dict of numpy arrays with the conserved fields (rung optional, zeros); box: SxBox"""
        self.ctx, self.L, self.h = ctx, ctx.L, ctx.h
        self.p = params or default_params()
        if self.p.propagator not in (0, 2):
            raise SxError("HydroVeBdtProp is the VE propagator")
        if self.p.g != 0.0 and any(box.bnd[k] == 1 for k in range(3)):
            raise SxError("self-gravity needs an open box (no Ewald replicas)")
        self.box, self.bucket = box, bucket
        n = len(host["x"])
        self.n = n
        self.dev, self.fields = {}, SxFields()
        self.fields.n = n
        for name in CONSERVED + DEPENDENT + (GRAD_V if self.p.avClean else []):
            dt = DT[name]
            d = ctx.alloc(n, dt)
            if name in host:
                d.set(np.asarray(host[name], dtype=dt))
            else:
                self.L.sx_memset(self.h, d.ptr, 0, n * np.dtype(dt).itemsize)
            self.dev[name] = d
            if name != "id":
                setattr(self.fields, name, d.ptr)
        self.order = ctx.alloc(n, np.uint32)
        self.scratch = ctx.alloc(n, np.uint64)
        self.gbuf = ctx.alloc(n + 1, np.uint32)
        self.group_dt = ctx.alloc(max(1, n), np.float32)
        self.group_idx = ctx.alloc(max(1, n), np.uint32)
        self.ts_start, self.ts_end = ctx.alloc(max(1, n), np.uint32), ctx.alloc(max(1, n), np.uint32)
        self.ts2_start, self.ts2_end = ctx.alloc(max(1, n), np.uint32), ctx.alloc(max(1, n), np.uint32)
        # Timestep timestep_, prevTimestep_ (timestep_.dt_m1[0] = settings "minDt", :122)
        self.ts = SxTimestep(numRungs=1, substep=0)
        self.ts.dt_m1[0] = np.float32(min_dt)
        self.prev = SxTimestep()
        self.min_dt = float(min_dt)  # d.minDt, d.minDt_m1, d.ttot
        self.min_dt_m1 = float(min_dt if min_dt_m1 is None else min_dt_m1)
        self.ttot = 0.0
        self.groups = self.ts_groups = None
        self.rungs = [None] * MAX_RUNGS
        self.active = None
        self.tree = None
        self.egrav = 0.0
        self.on_search = None  # test hook: called after the search of computeForces with the active view
        self.log = []

    # ---- helpers -------------------------------------------------------------------------------------------
    def _ck(self, rc, what):
        self.ctx.check(rc, what)

    def get(self, name):
        return self.dev[name].get()

    def _const_cv(self):
        """idealGasCv<float, double>(muiConst, gamma) (sph/eos.hpp:13-18: float R / mui, divided by gamma - 1 in
        double, returned as float), widened to the double constCv of computePositions (positions.hpp:168, 185)"""
        R = np.float32(8.317e7)
        return float(np.float32(np.float64(R / np.float32(self.p.muiConst)) / (self.p.gamma - 1.0)))

    # ---- sync (:171-218) -----------------------------------------------------------------------------------
    def _full_sync(self):
        L, h, n, d = self.L, self.h, self.n, self.dev
        keys = d["keys"]
        self._ck(L.sx_sfc_keys(h, d["x"].ptr, d["y"].ptr, d["z"].ptr, keys.ptr, n, C.byref(self.box)), "keys")
        self._ck(L.sx_sort_keys(h, keys.ptr, self.order.ptr, n), "sort")
        for name in CONSERVED:
            a = d[name]
            eb = a.dtype.itemsize
            self._ck(L.sx_gather(h, self.order.ptr, n, a.ptr, self.scratch.ptr, eb), "gather " + name)
            self._ck(L.sx_memcpy(h, a.ptr, self.scratch.ptr, n * eb, 3), "copy " + name)
        self._build_tree()
        # computeGroups(first, last, d, box, groups_) (groups.cu:30-47, tolFactor 2)
        out = SxGroups()
        self._ck(L.sx_spatial_groups(h, 0, n, d["x"].ptr, d["y"].ptr, d["z"].ptr, C.byref(self.tree), C.byref(self.box),
                                     2.0, self.gbuf.ptr, n + 1, C.byref(out)), "spatial groups")
        self.groups = Groups(out.groupStart, out.groupEnd, out.numGroups, 0, n)
        self.active = self.groups.view()
        # groupDt_ = FLT_MAX (:192-193)
        self.group_dt.set(np.concatenate([np.full(out.numGroups, FLT_MAX, np.float32),
                                          np.zeros(self.group_dt.n - out.numGroups, np.float32)]))

    def _build_tree(self):
        ctx, L, h, n = self.ctx, self.L, self.h, self.n
        cap = max(64, 2 * n // max(1, self.bucket) * 8 + 64)
        if getattr(self, "_tree_cap", 0) < cap:
            self._tree_cap = cap
            nn = cap + (cap - 1) // 7 + 1
            self._t = dict(leaves=ctx.alloc(cap + 1, np.uint64), counts=ctx.alloc(cap + 1, np.uint32),
                           prefixes=ctx.alloc(nn, np.uint64), childOffsets=ctx.alloc(nn + 1, np.int32),
                           parents=ctx.alloc(max(1, nn // 8), np.int32), levelRange=ctx.alloc(23, np.int32),
                           internalToLeaf=ctx.alloc(nn, np.int32), leafToInternal=ctx.alloc(nn, np.int32),
                           centers=ctx.alloc(3 * nn, np.float64), sizes=ctx.alloc(3 * nn, np.float64),
                           layout=ctx.alloc(cap + 1, np.uint32))
        t = self._t
        nleaf = C.c_int32()
        self._ck(L.sx_compute_octree(h, self.dev["keys"].ptr, n, self.bucket, t["leaves"].ptr, t["counts"].ptr, cap,
                                     C.byref(nleaf)), "octree")
        nl = nleaf.value
        nn = nl + (nl - 1) // 7
        oc = SxOctree(**{k: t[k].ptr for k in ("prefixes", "childOffsets", "parents", "levelRange", "internalToLeaf",
                                               "leafToInternal")})
        self._ck(L.sx_build_octree(h, t["leaves"].ptr, nl, C.byref(oc)), "link octree")
        self._ck(L.sx_node_centers(h, t["prefixes"].ptr, nn, C.byref(self.box), t["centers"].ptr, t["sizes"].ptr),
                 "centers")
        self._ck(L.sx_leaf_layout(h, t["counts"].ptr, nl, t["layout"].ptr), "layout")
        # d.treeView = domain.octreeProperties(): searchExtFactor back to 1
        self.tree = SxTree(numLeafNodes=nl, numNodes=nn, prefixes=t["prefixes"].ptr,
                           childOffsets=t["childOffsets"].ptr, internalToLeaf=t["internalToLeaf"].ptr,
                           levelRange=t["levelRange"].ptr, leaves=t["leaves"].ptr, layout=t["layout"].ptr,
                           centers=t["centers"].ptr, sizes=t["sizes"].ptr, searchExtFactor=1.0)

    def _partial_sync(self):
        # one rank: no halos to exchange (:199); the tree-cell search radius grows per substep (:207)
        self.tree.searchExtFactor = float(np.float32(np.float64(np.float32(self.tree.searchExtFactor)) * 1.012))
        hr = butterfly(self.ts.substep)
        self.active = sliced(self.ts_groups.view(), self.ts.rungRanges[0], self.ts.rungRanges[hr])

    def is_synced(self):
        return active_rung(self.ts.substep, self.ts.numRungs) == 0

    # ---- computeForces (:222-290) --------------------------------------------------------------------------
    def compute_forces(self):
        L, h, f, p, box = self.L, self.h, self.fields, self.p, self.box
        if self.is_synced():
            self._full_sync()
        else:
            self._partial_sync()
        v = self.active
        gdt = self.group_dt.ptr
        self._ck(L.sx_xmass(h, C.byref(v), C.byref(f), C.byref(p), C.byref(box), C.byref(self.tree)), "xmass")
        if self.on_search is not None:
            self.on_search(self, v)
        self._ck(L.sx_ve_def_gradh(h, C.byref(v), C.byref(f), C.byref(p), C.byref(box)), "VeDefGradh")
        self._ck(L.sx_eos(h, 0, self.n, p.muiConst, p.gamma, f.temp, f.m, f.kx, f.xm, f.gradh, f.prho, f.c, None,
                          None), "EOS")
        self._ck(L.sx_iad_divv_curlv(h, C.byref(v), C.byref(f), C.byref(p), C.byref(box)), "IAD")
        # groupDivvTimestep: groupDivvTimestepGpu(d.Krho, ...) (ts_rungs.hpp:48-54)
        self._ck(L.sx_group_divv_timestep(h, np.float32(p.Krho), C.byref(v), f.divv, gdt), "group divv dt")
        self._ck(L.sx_av_switches(h, C.byref(v), C.byref(f), C.byref(p), C.byref(box), self.min_dt), "AV switches")
        me = L.sx_momentum_energy_avclean if p.avClean else L.sx_momentum_energy
        self._ck(me(h, C.byref(v), gdt, C.byref(f), C.byref(p), C.byref(box), None), "momentum")
        if p.g != 0.0:
            self._gravity(self.is_synced())
        # groupAccTimestep: etaAcc * sqrt(eps) (ts_rungs.hpp:58-65)
        eta = np.float32(np.float64(p.etaAcc) * np.sqrt(np.float64(p.eps)))
        self._ck(L.sx_group_acc_timestep(h, eta, C.byref(v), f.ax, f.ay, f.az, gdt), "group acc dt")

    def _gravity(self, new_hierarchy):
        """mHolder_.upsweep + traverse(gravGroup) (:272-286): gravGroup is every target on a new hierarchy
        (computeSpatialGroups of the MultipoleHolder), else the active rungs"""
        L, h, t = self.L, self.h, self.tree
        nn = t.numNodes
        if getattr(self, "_gcap", 0) < nn:
            self._gcap = nn
            self._gc, self._gm = self.ctx.alloc(4 * nn, np.float64), self.ctx.alloc(8 * nn, np.float32)
        self._ck(L.sx_gravity_upsweep(h, C.byref(self.fields), C.byref(t), self.p.theta, self._gc.ptr, self._gm.ptr),
                 "upsweep")
        g = SxGroups(firstBody=0, lastBody=self.n) if new_hierarchy else self.active
        e = C.c_double()
        self._ck(L.sx_gravity_traverse(h, C.byref(g), C.byref(self.fields), C.byref(t), C.byref(self.box),
                                       self._gc.ptr, self._gm.ptr, np.float32(self.p.g), C.byref(e)), "gravity")
        self.egrav = e.value

    # ---- computeRungs (:292-331) ---------------------------------------------------------------------------
    def compute_rungs(self):
        L, h = self.L, self.h
        high = active_rung(self.ts.substep, self.ts.numRungs)
        if high == 0:
            C.memmove(C.byref(self.prev), C.byref(self.ts), C.sizeof(SxTimestep))
            max_dt = np.float32(np.float64(self.ts.dt_m1[0]) * np.float64(self.p.maxDtIncrease))
            ts = SxTimestep()
            self._ck(L.sx_rung_timestep(h, self.group_dt.ptr, self.group_idx.ptr, self.groups.num, max_dt, None,
                                        C.byref(ts)), "rungTimestep")
            self.ts = ts
        else:
            dt = C.c_float()
            rr = (C.c_uint32 * (MAX_RUNGS + 1))()
            self._ck(L.sx_minimum_group_dt(h, C.byref(self.ts), self.group_dt.ptr, self.group_idx.ptr,
                                           self.ts.rungRanges[high], None, C.byref(dt), rr), "minimumGroupDt")
            self.ts.nextDt = dt.value
            for r in range(high):
                self.ts.rungRanges[r] = rr[r]
        if high == 0 or high > 1:
            if high > 1:
                self.groups, self.ts_groups = self.ts_groups, self.groups
            # extractGroupGpu(groups_.view(), groupIndices_, 0, rungRanges.back(), tsGroups_) into the spare buffers
            if self.groups.start == self.ts_start.ptr:  # never overwrite the groups being extracted from
                s, e = self.ts2_start, self.ts2_end
            else:
                s, e = self.ts_start, self.ts_end
            g = self.groups.view()
            last = self.ts.rungRanges[MAX_RUNGS]
            self._ck(L.sx_extract_groups(h, C.byref(g), self.group_idx.ptr, 0, last, s.ptr, e.ptr), "extract groups")
            self.ts_groups = Groups(s.ptr, e.ptr, last, 0, 0)
        for r in range(self.ts.numRungs):
            self.rungs[r] = sliced(self.ts_groups.view(), self.ts.rungRanges[r], self.ts.rungRanges[r + 1])
        self.log.append(dict(substep=self.ts.substep, high=high, numRungs=self.ts.numRungs, nextDt=self.ts.nextDt,
                             rungRanges=list(self.ts.rungRanges)))

    # ---- integrate (:333-378) ------------------------------------------------------------------------------
    def integrate(self):
        self.compute_rungs()
        L, h, f, ts = self.L, self.h, self.fields, self.ts
        f32 = np.float32
        lowest_drift = butterfly(ts.substep + 1)
        last_substep = active_rung(ts.substep + 1, ts.numRungs) == 0
        open_box = SxBox()
        open_box.lim[:] = [0.0, 1.0, 0.0, 1.0, 0.0, 1.0]  # cstone::Box<T>(0, 1, open)
        sub_box = self.box if last_substep else open_box
        gamma, cv = self.p.gamma, self._const_cv()
        rung = self.dev["rung"].ptr
        for i in range(ts.numRungs):
            use_rung = ts.substep == ts.substep % (1 << i)  # drift back to the start of the hierarchy
            advance = i < lowest_drift
            dt = f32(ts.nextDt)
            src = self.prev if use_rung else ts
            dt_m1 = np.array([src.dt_m1[k] for k in range(MAX_RUNGS)], np.float32)
            g = self.rungs[i]
            live = g.numGroups > 0  # a kernel over zero groups does nothing
            if advance:
                if ts.dt_drift[i] > 0 and live:
                    self._ck(L.sx_drift_positions(h, C.byref(g), 0.0, f32(ts.dt_drift[i]), dt_m1.ctypes.data, rung,
                                                  C.byref(f), gamma, cv), "drift back")
                if live:
                    self._ck(L.sx_positions_rungs(h, C.byref(g), f32(f32(ts.dt_drift[i]) + dt), dt_m1.ctypes.data,
                                                  rung, C.byref(f), gamma, cv, C.byref(sub_box)), "positions")
                ts.dt_m1[i] = f32(f32(ts.dt_drift[i]) + dt)
                ts.dt_drift[i] = 0.0
                if live:
                    self._ck(L.sx_store_rung(h, C.byref(g), i, rung), "store rung")
            else:
                if live:
                    self._ck(L.sx_drift_positions(h, C.byref(g), f32(f32(ts.dt_drift[i]) + dt), f32(ts.dt_drift[i]),
                                                  dt_m1.ctypes.data, rung, C.byref(f), gamma, cv), "drift")
                ts.dt_drift[i] = f32(f32(ts.dt_drift[i]) + dt)
        self._ck(L.sx_update_h_groups(h, C.byref(self.active), self.p.ng0, f.nc, f.h), "update h")
        ts.substep += 1
        ts.elapsedDt = f32(f32(ts.elapsedDt) + f32(ts.nextDt))
        self.ttot += float(f32(ts.nextDt))
        self.min_dt_m1 = self.min_dt
        self.min_dt = float(f32(ts.nextDt))

    def step(self):
        """Propagator::computeForces + integrate: one substep of the block time-step hierarchy"""
        self.compute_forces()
        self.integrate()
        self.ctx.sync()
