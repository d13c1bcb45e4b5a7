"""Multi-rank CPU restatement of the SFC domain decomposition + VE step (TEST INFRASTRUCTURE ONLY).

Never imported by the product path: tests/ use it as the checker of the multi-GPU algorithm on the CPU, with
torch.distributed (gloo) standing in for RCCL.  It runs the same decomposition as sx_sim.cpp (distributedSync and
the halo exchanges of sx_sim_step), which replaces the reference's Domain::sync (domain/include/cstone/domain/
domain.hpp:196-244) and the halo exchanges of HydroVeProp (main/src/propagator/ve_hydro.hpp:150-186):

  1. SFC keys, local sort;
  2. global histogram of 2^18 key bins (all-reduce) -> equal-count splitters, computed by the product library's
     host function sx_domain_splitters (the same code the GPU path calls);
  3. particle exchange (all-to-all of the conserved fields) to the SFC owner, re-sort;
  4. halo discovery: an AABB per 2048 SFC-consecutive locals grown by 2*hmax*margin + key-quantisation margin,
     all-gathered; every rank sends the locals inside a peer's boxes (minimum image); receive layout
     [lower ranks | locals | higher ranks] from sx_domain_halo_layout (key-sorted, one tree for all);
  5. x,y,z,h,m of the halos; neighbor search with the h iteration on the locals; if a local's h grew past its
     chunk's request radius (decided globally) the discovery is redone with a 1.5x margin;
  6. the five halo exchanges between the kernels (xm | v,prho,c,kx | c_ij,divv | alpha), global dt = min over
     ranks, positions + h update on the locals.

With overlap=True each exchange is overlapped as sx_sim.cpp does it (classifyClustersKernel + the comm-stream
exchanges): clusters of 256 SFC-consecutive locals whose neighbor union holds no halo are "interior" and are
computed BEFORE the exchange, with the halo copies of the exchanged fields poisoned (NaN); the "boundary" clusters
after it.  A wrong classification lets a NaN into an interior result, so overlap == serial bitwise is the check.

The per-particle kernels are the plain-C oracle (sph_oracle.c) on [first, last) of the rank's arrays.
"""
import math

import numpy as np

import pyoracle as po

HIST_BITS = 18
CHUNK = 2048
HALO_MARGIN = 1.05
MAX_LEVEL = 21


def _dist():
    import torch.distributed as dist

    return dist


def _a2a_bytes(send, send_counts, item):
    """all-to-all of a 1-D array segmented by send_counts (elements, rank order) -> received array, counts"""
    import torch

    dist = _dist()
    P = dist.get_world_size()
    sc = torch.tensor([int(c) for c in send_counts], dtype=torch.int64)
    rc = torch.empty(P, dtype=torch.int64)
    dist.all_to_all_single(rc, sc)
    rcounts = [int(v) for v in rc]
    sb = np.ascontiguousarray(send).view(np.uint8)
    out = torch.empty(sum(rcounts) * item, dtype=torch.uint8)
    dist.all_to_all_single(out, torch.from_numpy(sb.copy()), [c * item for c in rcounts],
                           [int(c) * item for c in send_counts])
    return out.numpy().view(send.dtype).copy(), rcounts


def quant_margin(box):
    L = [box.lim[2 * k + 1] - box.lim[2 * k] for k in range(3)]
    return 4.0 * max(L) / float(1 << MAX_LEVEL)


def _fold(d, box, k):
    if box.bnd[k] != 1:
        return d
    L = box.lim[2 * k + 1] - box.lim[2 * k]
    return d - L * np.rint(d / L)


class DistOracle:
    """one rank of the decomposed oracle; `local` is a po.HostState with this rank's particles"""

    CLUSTER = 256  # targets sharing one neighbor union (sx_device.hpp kCluster)

    def __init__(self, ora, box, local, bucket=64, overlap=False):
        dist = _dist()
        self.ora, self.box, self.bucket, self.overlap = ora, box, bucket, overlap
        self.cluster_counts = [0, 0]  # interior, boundary clusters of the last step
        self.rank, self.size = dist.get_rank(), dist.get_world_size()
        self.local = local
        self.p = ora.params()
        self.halo_retries = 0

    # ---- sync ------------------------------------------------------------------------------------------------
    def _sort(self, st):
        keys = self.ora.sfc_keys(st, self.box).copy()
        o = np.argsort(keys, kind="stable")
        for k in st.arrays:
            st.arrays[k][:] = st.arrays[k][o]
        st.keys[:] = keys[o]
        return st

    def _exchange_particles(self, st):
        import sphexa_amd as sx
        import torch

        dist = _dist()
        P = self.size
        bins = (st.keys >> np.uint64(63 - HIST_BITS)).astype(np.int64)
        hist = torch.from_numpy(np.bincount(bins, minlength=1 << HIST_BITS).astype(np.int64))
        dist.all_reduce(hist, op=dist.ReduceOp.SUM)
        split = sx.domain_splitters(hist.numpy().astype(np.uint32), HIST_BITS, P)
        seg = np.searchsorted(st.keys, split, side="left")
        seg[0], seg[P] = 0, st.n
        counts = np.diff(seg)
        arrays = {}
        for name in po.CONSERVED:
            a = st.arrays[name]
            arrays[name], rc = _a2a_bytes(a, counts, a.itemsize)
        out = po.HostState(sum(rc))
        for name in po.CONSERVED:
            out.arrays[name][:] = arrays[name]
        out.minDt, out.minDt_m1, out.ttot = st.minDt, st.minDt_m1, st.ttot
        self.split = split
        return self._sort(out)

    def _chunk_boxes(self, st, margin):
        qm = quant_margin(self.box)
        boxes = []
        for c0 in range(0, st.n, CHUNK):
            c1 = min(st.n, c0 + CHUNK)
            lo = np.array([st.x[c0:c1].min(), st.y[c0:c1].min(), st.z[c0:c1].min()])
            hi = np.array([st.x[c0:c1].max(), st.y[c0:c1].max(), st.z[c0:c1].max()])
            hmax = float(st.h[c0:c1].max())
            R = 2.0 * hmax * margin + qm
            boxes.append(np.concatenate([0.5 * (lo + hi), 0.5 * (hi - lo) + R, [hmax]]))
        return np.array(boxes, np.float64).reshape(-1, 7)

    def _discover(self, st, margin):
        import sphexa_amd as sx
        import torch

        dist = _dist()
        P, r = self.size, self.rank
        mine = self._chunk_boxes(st, margin)
        self.my_boxes = mine
        cnt = torch.tensor([mine.shape[0]], dtype=torch.int64)
        allc = [torch.zeros(1, dtype=torch.int64) for _ in range(P)]
        dist.all_gather(allc, cnt)
        mx = max(int(c) for c in allc)
        pad = np.zeros((mx, 7), np.float64)
        pad[: mine.shape[0]] = mine
        gathered = [torch.zeros((mx, 7), dtype=torch.float64) for _ in range(P)]
        dist.all_gather(gathered, torch.from_numpy(pad))
        qm = quant_margin(self.box)
        self.send_idx = []
        for q in range(P):
            if q == r:
                self.send_idx.append(np.zeros(0, np.int64))
                continue
            boxes = gathered[q].numpy()[: int(allc[q])]
            inside = np.zeros(st.n, bool)
            for b in boxes:
                d = [np.abs(_fold(c - b[k], self.box, k)) for k, c in enumerate((st.x, st.y, st.z))]
                inside |= (d[0] <= b[3] + qm) & (d[1] <= b[4] + qm) & (d[2] <= b[5] + qm)
            self.send_idx.append(np.nonzero(inside)[0])
        send_counts = [len(s) for s in self.send_idx]
        sc = torch.tensor(send_counts, dtype=torch.int64)
        rc = torch.empty(P, dtype=torch.int64)
        dist.all_to_all_single(rc, sc)
        self.recv_counts = [int(v) for v in rc]
        self.recv_counts[r] = 0
        off, (first, last, total) = sx.halo_layout(self.recv_counts, r, st.n)
        self.recv_off, self.first, self.last, self.total = off, first, last, total
        full = po.HostState(total)
        for name in po.CONSERVED:
            full.arrays[name][first:last] = st.arrays[name]
        full.minDt, full.minDt_m1, full.ttot = st.minDt, st.minDt_m1, st.ttot
        self.full = full
        self.halo_exchange(["x", "y", "z", "h", "m"])
        self.ora.sfc_keys(full, self.box)
        return full

    def halo_exchange(self, fields):
        r = self.rank
        full = self.full
        for name in fields:
            a = full.arrays[name]
            send = np.concatenate([a[self.first + idx] for idx in self.send_idx]) if self.send_idx else a[:0]
            recv, rcounts = _a2a_bytes(send, [len(s) for s in self.send_idx], a.itemsize)
            pos = 0
            for q, c in enumerate(rcounts):
                if q != r and c:
                    o = int(self.recv_off[q])
                    a[o:o + c] = recv[pos:pos + c]
                pos += c

    def _classify(self, nbr, nc, f, l):
        """interior / boundary clusters as (c0, c1) target ranges (classifyClustersKernel, sx_sim.cpp)"""
        ng = self.p.ngmax
        inner, bound = [], []
        for c0 in range(f, l, self.CLUSTER):
            c1 = min(l, c0 + self.CLUSTER)
            halo = False
            for i in range(c0, c1):
                cnt = min(int(nc[i - f]) - 1, ng)
                row = nbr[(i - f) * ng:(i - f) * ng + cnt]
                if cnt and (row.min() < f or row.max() >= l):
                    halo = True
                    break
            (bound if halo else inner).append((c0, c1))
        self.cluster_counts = [len(inner), len(bound)]
        return inner, bound

    def _phase(self, fields, kern, nbr, f, l):
        """exchange `fields`, then run kern(nbr rows, first, last) on the locals; with overlap: interior clusters
        first against poisoned halo copies, then the exchange, then the boundary clusters"""
        if not self.overlap:
            if fields:
                self.halo_exchange(fields)
            kern(nbr, f, l)
            return
        full, ng = self.full, self.p.ngmax
        for name in fields:
            full.arrays[name][:f] = np.nan
            full.arrays[name][l:] = np.nan
        for c0, c1 in self.interior:
            kern(nbr[(c0 - f) * ng:], c0, c1)
        if fields:
            self.halo_exchange(fields)
        for c0, c1 in self.boundary:
            kern(nbr[(c0 - f) * ng:], c0, c1)

    # ---- one VE step (ve_hydro.hpp:132-218) ---------------------------------------------------------------------
    def step(self):
        import torch

        dist = _dist()
        ora, box, p = self.ora, self.box, self.p
        st = self._sort(self.local)
        st = self._exchange_particles(st)
        margin = HALO_MARGIN
        h_pre = st.h.copy()
        for attempt in range(4):
            st.h[:] = h_pre
            full = self._discover(st, margin)
            f, l = self.first, self.last
            nbr, nc = ora.find_neighbors(full, box, f, l, bucket=self.bucket, iterate_h=True, ngmax=p.ngmax,
                                         ng0=p.ng0)
            full.nc[f:l] = nc
            # every local's final h within its chunk's request radius (sx_sim.cpp chunkCheckKernel), decided globally
            hm = np.repeat(self.my_boxes[:, 6], CHUNK)[: l - f]
            bad = torch.tensor([int(np.any(full.h[f:l].astype(np.float64) > hm * margin))], dtype=torch.int64)
            dist.all_reduce(bad, op=dist.ReduceOp.SUM)
            if int(bad) == 0:
                break
            margin *= 1.5
            self.halo_retries += 1
        else:
            raise RuntimeError("halo discovery did not converge")
        if self.overlap:
            self.interior, self.boundary = self._classify(nbr, nc, f, l)
        ora.xmass(full, box, nbr, f, l)
        self._phase(["xm"], lambda nb, a, b: ora.ve_def_gradh(full, box, nb, a, b), nbr, f, l)
        ora.eos(full, f, l)
        self._phase(["vx", "vy", "vz", "prho", "c", "kx"], lambda nb, a, b: ora.iad_divv_curlv(full, box, nb, a, b),
                    nbr, f, l)
        max_divv = float(np.max(full.divv[f:l])) if l > f else -math.inf
        self._phase(["c11", "c12", "c13", "c22", "c23", "c33", "divv"],
                    lambda nb, a, b: ora.av_switches(full, box, nb, a, b), nbr, f, l)
        courant = []

        def momentum(nb, a, b):
            ora.momentum_energy(full, box, nb, a, b)
            courant.append(full.minDtCourant)

        self._phase(["alpha"], momentum, nbr, f, l)
        full.minDtCourant = min(courant) if courant else math.inf
        # rhoTimestep + computeTimestep (ts_global.hpp:72-112) with the MPI_Allreduce(min) as a gloo all-reduce
        dt_rho = p.Krho / abs(max_divv) if max_divv != 0 else math.inf  # C: division by zero -> inf
        dt_loc = min(full.minDtCourant, dt_rho, p.maxDtIncrease * full.minDt)
        t = torch.tensor([dt_loc], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        dt = float(t)
        full.ttot += dt
        full.minDt_m1 = full.minDt
        full.minDt = dt
        ora.positions(full, box, f, l)
        s = full.struct()
        ora.lib.update_h_range(C_byref(s), p.ng0, f, l)
        out = po.HostState(l - f)
        for k in out.arrays:
            out.arrays[k][:] = full.arrays[k][f:l]
        out.minDt, out.minDt_m1, out.ttot = full.minDt, full.minDt_m1, full.ttot
        out.minDtCourant, out.minDtRho = full.minDtCourant, dt_rho
        self.local = out
        return out


def C_byref(s):
    import ctypes

    return ctypes.byref(s)


# ---- multi-rank self-gravity (restates distributedGravity, sph-exa_amd/csrc/sx_sim.cpp) ----------------------------
CELL_SHIFT = 63 - HIST_BITS  # level-6 SFC cells = the splitter bins: one owner per cell


def _cell_geometry(st, box, sel):
    """geometric center and half size of the level-6 cell holding the particles sel (all in one cell)"""
    c, s = np.zeros(3), np.zeros(3)
    for k, name in enumerate(("x", "y", "z")):
        lo, hi = box.lim[2 * k], box.lim[2 * k + 1]
        L = (hi - lo) / float(1 << (HIST_BITS // 3))
        ic = np.floor((st.arrays[name][sel][0] - lo) / L)
        c[k], s[k] = lo + (ic + 0.5) * L, 0.5 * L
    return c, s


def _cell_moments(st, box, idx, inv_theta):
    """com, mass, MAC radius^2 (setMac) and traceless quadrupole (Cqi order) of one cell, float64"""
    x, y, z = st.x[idx], st.y[idx], st.z[idx]
    m = st.m[idx].astype(np.float64)
    M = m.sum()
    com = np.array([np.sum(m * x), np.sum(m * y), np.sum(m * z)]) / M
    gc, gs = _cell_geometry(st, box, idx)
    mac = 2.0 * gs.max() * inv_theta + np.linalg.norm(com - gc)
    r = np.stack([x - com[0], y - com[1], z - com[2]], 1)
    Q = np.einsum("i,ia,ib->ab", m, r, r)
    tr = np.trace(Q)
    q = np.array([M, 3 * Q[0, 0] - tr, 3 * Q[0, 1], 3 * Q[0, 2], 3 * Q[1, 1] - tr, 3 * Q[1, 2], 3 * Q[2, 2] - tr, tr])
    return np.concatenate([com, [mac * mac], q])


def _m2p(targets, cells):
    """quadrupole M2P (cartesian_qpole.hpp:175-201) of every cell on every target, float64; returns (n, 4)"""
    out = np.zeros((targets.shape[0], 4))
    for c in cells:
        r = targets - c[0:3]
        rr = np.sum(r * r, 1)
        rm1 = 1.0 / np.sqrt(rr)
        rm2 = rm1 * rm1
        rm5 = rm2 * rm2 * rm1
        M = c[4:12]
        Qr = np.stack([r[:, 0] * M[1] + r[:, 1] * M[2] + r[:, 2] * M[3],
                       r[:, 0] * M[2] + r[:, 1] * M[4] + r[:, 2] * M[5],
                       r[:, 0] * M[3] + r[:, 1] * M[5] + r[:, 2] * M[6]], 1)
        rQr = np.sum(r * Qr, 1)
        mono = (-2.5 * rQr * rm5 - M[0] * rm1) * rm2
        out[:, 0] += -(M[0] * rm1 + 0.5 * rm5 * rQr)
        out[:, 1:] += rm5[:, None] * Qr + mono[:, None] * r
    return out


def distributed_gravity(d, full, G, theta):
    """gravity of the locals [d.first, d.last) of `full` (key sorted, after DistOracle._discover): own level-6 cells'
    moments all-gathered; remote cells passing the vector MAC against every request box of this rank are far-field
    multipoles, the particles of the others are fetched from their owners and traversed with the locals (oracle
    Barnes-Hut on their own tree).  Returns accelerations (nl, 3), egrav and {halos, far_cells, remote_cells}."""
    import torch

    dist = _dist()
    P, r = d.size, d.rank
    f, l = d.first, d.last
    nl = l - f
    keys = full.keys[f:l]
    cells = (keys >> np.uint64(CELL_SHIFT)).astype(np.int64)
    ucell, start = np.unique(cells, return_index=True)
    ends = np.append(start[1:], nl)
    inv_theta = 1.0 / theta
    mine = np.array([np.concatenate([[c], _cell_moments(full, d.box, np.arange(f + b, f + e), inv_theta)])
                     for c, b, e in zip(ucell, start, ends)]).reshape(-1, 13)
    # all-gather (rank order = key order)
    cnt = torch.tensor([mine.shape[0]], dtype=torch.int64)
    allc = [torch.zeros(1, dtype=torch.int64) for _ in range(P)]
    dist.all_gather(allc, cnt)
    mx = max(int(c) for c in allc)
    pad = np.zeros((mx, 13))
    pad[: mine.shape[0]] = mine
    gathered = [torch.zeros((mx, 13), dtype=torch.float64) for _ in range(P)]
    dist.all_gather(gathered, torch.from_numpy(pad))
    remote = [gathered[q].numpy()[: int(allc[q])] for q in range(P)]
    # near / far against the request boxes of this rank (center, half size + search radius)
    boxes = d.my_boxes
    near = []
    for q in range(P):
        if q == r:
            near.append(np.zeros(0, bool))
            continue
        nq = np.zeros(remote[q].shape[0], bool)
        for b in boxes:
            dd = np.maximum(np.abs(b[0:3][None, :] - remote[q][:, 1:4]) - b[3:6][None, :], 0.0)
            nq |= np.sum(dd * dd, 1) < remote[q][:, 4]
        near.append(nq)
    # requests: cell ids to each owner; owners answer with x, y, z, m, h of those cells (ascending = key order)
    req = [remote[q][near[q], 0].astype(np.int64) if q != r else np.zeros(0, np.int64) for q in range(P)]
    got, rcounts = _a2a_bytes(np.concatenate(req) if req else np.zeros(0, np.int64), [len(x) for x in req], 8)
    pos = np.cumsum([0] + rcounts)
    send = []
    for q in range(P):
        ids = got[pos[q]:pos[q + 1]]
        sel = [np.arange(f + start[k], f + ends[k]) for k in np.searchsorted(ucell, ids)] if len(ids) else []
        send.append(np.concatenate(sel) if sel else np.zeros(0, np.int64))
    parts = {}
    for name in ("x", "y", "z", "m", "h"):
        a = full.arrays[name]
        src = np.concatenate([a[s] for s in send]) if send else a[:0]
        parts[name], pc = _a2a_bytes(src, [len(s) for s in send], a.itemsize)
    po_ = np.cumsum([0] + pc)
    nlow = int(sum(pc[:r]))
    nh = int(sum(pc)) - nlow
    g = po.HostState(nlow + nl + nh)
    for name in ("x", "y", "z", "m", "h"):
        g.arrays[name][:nlow] = parts[name][:nlow]
        g.arrays[name][nlow:nlow + nl] = full.arrays[name][f:l]
        g.arrays[name][nlow + nl:] = parts[name][nlow:]
    d.ora.sfc_keys(g, d.box)
    assert np.all(np.diff(g.keys.astype(np.float64)) >= 0), "gravity sources not key sorted"
    prm = d.ora.params(g=G, theta=theta)
    eg, _, _ = d.ora.gravity(g, d.box, prm, first=nlow, last=nlow + nl)
    acc = np.stack([g.ax[nlow:nlow + nl], g.ay[nlow:nlow + nl], g.az[nlow:nlow + nl]], 1).astype(np.float64)
    far = [remote[q][~near[q]] for q in range(P) if q != r]
    far = np.concatenate(far) if far else np.zeros((0, 13))
    tg = np.stack([full.x[f:l], full.y[f:l], full.z[f:l]], 1)
    fa = _m2p(tg, far[:, 1:]) if far.shape[0] else np.zeros((nl, 4))
    acc += G * fa[:, 1:]
    eg += 0.5 * G * float(np.sum(full.m[f:l].astype(np.float64) * fa[:, 0]))
    stats = {"halos": nlow + nh, "far_cells": int(far.shape[0]), "remote_cells": int(sum(x.shape[0] for x in remote))
             - mine.shape[0]}
    return acc, eg, stats


# ---- skin lists on several ranks: the argument behind reuse steps (sx_skin.hpp, DESIGN 4c, sx_sim.cpp skinHaloRefresh)

SKIN_GRID_N = 16  # displacement-grid cells per axis here (the GPU's 64^3; any resolution gives a valid bound)


def _grid_cells(pos, box, n):
    """cell index per particle of an n^3 grid over the box (gridCell: floor, periodic axes wrapped, others clamped)"""
    idx = []
    for k in range(3):
        lo, L = box.lim[2 * k], box.lim[2 * k + 1] - box.lim[2 * k]
        c = np.floor((pos[:, k] - lo) * (n / L)).astype(np.int64)
        idx.append(np.mod(c, n) if box.bnd[k] == 1 else np.clip(c, 0, n - 1))
    return idx


def _mi_dist2(a, b, box):
    d2 = 0.0
    for k in range(3):
        d2 = d2 + _fold(a[..., k] - b[..., k], box, k) ** 2
    return d2


def skin_premise(d, full, glob_pos0, h_of, s, disps, global_grid=True):
    """Restatement of the multi-rank skin argument on this rank (test infrastructure).

    Build: the halos of `full` were requested with the skin radius (d._discover(..., HALO_MARGIN * (1 + s))); every
    local target a gets its skin list S_a = the particles of locals + halos within R_a = 2 h_a (1 + s).  Returned check
    1: S_a equals the global truth within R_a (the halo set of the build holds every skin neighbour).
    Reuse steps t = 1, 2, ...: every particle moves by disps[t-1] (rows by id, the same on every rank); this rank
    scatters its LOCALS' displacements into a grid of per-cell component ranges (cells of the end-of-step positions),
    reduced over all ranks with min / max when global_grid (the GPU's all-reduce of the grid) or left local; per
    cluster of 256 consecutive locals, with u = the displacement of its first particle, the filter's bound
    2 h_a + d_a + A_C <= R_a (1 - 2^-16) (d_a = sum_t |d_a(t) - u(t)|, A_C = sum_t max over the cells around the
    cluster's targets grown by max R of the largest |d - u|).  Check 2: every target of every cluster the bound admits
    has all its current neighbours (global truth within 2 h_a, minimum image) in S_a.
    Returns (skin_mismatch, admitted clusters per step, violations per step)."""
    import torch

    dist = _dist()
    box, f, l = d.box, d.first, d.last
    d.halo_exchange(["id"])  # the halos' ids (the sync's setup exchange carries x, y, z, h, m only)
    ids_full = full.id.astype(np.int64)
    loc = ids_full[f:l]
    n_glob = glob_pos0.shape[0]
    # skin lists at the build, by id, over locals + halos; the truth over every particle
    R = 2.0 * h_of[loc] * (1.0 + s)
    pf = glob_pos0[ids_full]
    skin, mismatch = [], 0
    for q, a in enumerate(loc):
        d2 = _mi_dist2(pf, glob_pos0[a][None, :], box)
        sa = set(ids_full[(d2 < R[q] ** 2)].tolist()) - {int(a)}
        dg = _mi_dist2(glob_pos0, glob_pos0[a][None, :], box)
        truth = set(np.nonzero(dg < R[q] ** 2)[0].tolist()) - {int(a)}
        mismatch += sa != truth
        skin.append(sa)
    pos = glob_pos0.copy()
    rel = np.zeros(len(loc))
    ncl = (len(loc) + DistOracle.CLUSTER - 1) // DistOracle.CLUSTER
    acc = np.zeros(ncl)
    G = SKIN_GRID_N
    admitted, violations = [], []
    for disp in disps:
        pos = pos + disp
        for k in range(3):
            if box.bnd[k] == 1:
                lo, L = box.lim[2 * k], box.lim[2 * k + 1] - box.lim[2 * k]
                pos[:, k] = lo + np.mod(pos[:, k] - lo, L)
        # this rank's grid of its locals' displacements, reduced over the ranks
        cx, cy, cz = _grid_cells(pos[loc], box, G)
        cell = (cz * G + cy) * G + cx
        lo_ = np.full((3, G ** 3), np.inf)
        hi_ = np.full((3, G ** 3), -np.inf)
        for k in range(3):
            np.minimum.at(lo_[k], cell, disp[loc, k])
            np.maximum.at(hi_[k], cell, disp[loc, k])
        if global_grid:
            tl, th = torch.from_numpy(lo_), torch.from_numpy(hi_)
            dist.all_reduce(tl, op=dist.ReduceOp.MIN)
            dist.all_reduce(th, op=dist.ReduceOp.MAX)
            lo_, hi_ = tl.numpy(), th.numpy()
        n_ok, n_bad = 0, 0
        for c in range(ncl):
            sel = np.arange(c * DistOracle.CLUSTER, min(len(loc), (c + 1) * DistOracle.CLUSTER))
            ids = loc[sel]
            u = disp[ids[0]]
            rel[sel] += np.sqrt(np.sum((disp[ids] - u) ** 2, axis=1))
            # cells around the targets (minimum image relative to the cluster's first particle) grown by max R
            o = pos[ids[0]]
            rr = np.stack([_fold(pos[ids, k] - o[k], box, k) for k in range(3)], axis=1)
            Rm = float(R[sel].max())
            ranges = []
            for k in range(3):
                lo, L = box.lim[2 * k], box.lim[2 * k + 1] - box.lim[2 * k]
                k0 = int(np.floor((o[k] + rr[:, k].min() - Rm - lo) * (G / L)))
                k1 = int(np.floor((o[k] + rr[:, k].max() + Rm - lo) * (G / L)))
                if box.bnd[k] == 1:
                    ranges.append(np.mod(np.arange(k0, k1 + 1), G) if k1 - k0 + 1 < G else np.arange(G))
                else:
                    ranges.append(np.arange(max(0, k0), min(G - 1, k1) + 1))
            cz_, cy_, cx_ = np.meshgrid(ranges[2], ranges[1], ranges[0], indexing="ij")
            cells = ((cz_ * G + cy_) * G + cx_).ravel()
            g = 0.0
            for q_ in cells:
                if np.isfinite(lo_[0, q_]):
                    e = [max(abs(lo_[k, q_] - u[k]), abs(hi_[k, q_] - u[k])) for k in range(3)]
                    g = max(g, float(np.sqrt(e[0] ** 2 + e[1] ** 2 + e[2] ** 2)))
            acc[c] += g
            if not np.all(2.0 * h_of[ids] + rel[sel] + acc[c] <= R[sel] * (1.0 - 2.0 ** -16)):
                continue
            n_ok += 1
            for q_, a in zip(sel, ids):
                dg = _mi_dist2(pos, pos[a][None, :], box)
                truth = set(np.nonzero(dg < (2.0 * h_of[a]) ** 2)[0].tolist()) - {int(a)}
                n_bad += not truth <= skin[q_]
        admitted.append(n_ok)
        violations.append(n_bad)
    return mismatch, admitted, violations
