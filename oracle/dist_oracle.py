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

    def __init__(self, ora, box, local, bucket=64):
        dist = _dist()
        self.ora, self.box, self.bucket = ora, box, bucket
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
        ora.xmass(full, box, nbr, f, l)
        self.halo_exchange(["xm"])
        ora.ve_def_gradh(full, box, nbr, f, l)
        ora.eos(full, f, l)
        self.halo_exchange(["vx", "vy", "vz", "prho", "c", "kx"])
        ora.iad_divv_curlv(full, box, nbr, f, l)
        max_divv = float(np.max(full.divv[f:l])) if l > f else -math.inf
        self.halo_exchange(["c11", "c12", "c13", "c22", "c23", "c33", "divv"])
        ora.av_switches(full, box, nbr, f, l)
        self.halo_exchange(["alpha"])
        ora.momentum_energy(full, box, nbr, f, l)
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
