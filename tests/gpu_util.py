"""Helpers for the GPU parity tests: build the device tree through the C-ABI, run single kernels, compare."""
import ctypes as C

import numpy as np

import pyoracle as po
import sphexa_amd as sx


def box_to_sx(obox):
    return sx.make_box(list(obox.lim), list(obox.bnd))


def device_tree(ctx, keys_dev, n, bucket, box):
    L = ctx.L
    cap = max(64, 2 * n // max(1, bucket) * 8 + 64)
    leaves = ctx.alloc(cap + 1, np.uint64)
    counts = ctx.alloc(cap + 1, np.uint32)
    nleaf = C.c_int32()
    ctx.check(L.sx_compute_octree(ctx.h, keys_dev.ptr, n, bucket, leaves.ptr, counts.ptr, cap, C.byref(nleaf)),
              "compute_octree")
    nl = nleaf.value
    nint = (nl - 1) // 7
    nn = nl + nint
    arrs = dict(prefixes=ctx.alloc(nn, np.uint64), childOffsets=ctx.alloc(nn + 1, np.int32),
                parents=ctx.alloc(max(1, (nn - 1) // 8), np.int32), levelRange=ctx.alloc(23, np.int32),
                internalToLeaf=ctx.alloc(nn, np.int32), leafToInternal=ctx.alloc(nn, np.int32))
    oc = sx.SxOctree(**{k: v.ptr for k, v in arrs.items()})
    ctx.check(L.sx_build_octree(ctx.h, leaves.ptr, nl, C.byref(oc)), "build_octree")
    centers = ctx.alloc(3 * nn, np.float64)
    sizes = ctx.alloc(3 * nn, np.float64)
    ctx.check(L.sx_node_centers(ctx.h, arrs["prefixes"].ptr, nn, C.byref(box), centers.ptr, sizes.ptr), "centers")
    layout = ctx.alloc(nl + 1, np.uint32)
    ctx.check(L.sx_leaf_layout(ctx.h, counts.ptr, nl, layout.ptr), "layout")
    tree = sx.SxTree(numLeafNodes=nl, numNodes=nn, prefixes=arrs["prefixes"].ptr,
                     childOffsets=arrs["childOffsets"].ptr, internalToLeaf=arrs["internalToLeaf"].ptr,
                     levelRange=arrs["levelRange"].ptr, leaves=leaves.ptr, layout=layout.ptr, centers=centers.ptr,
                     sizes=sizes.ptr, searchExtFactor=1.0)
    host = {k: v.get() for k, v in arrs.items()}
    host["leaves"] = leaves.get()[:nl + 1]
    host["counts"] = counts.get()[:nl]
    host["centers"] = centers.get().reshape(-1, 3)
    host["sizes"] = sizes.get().reshape(-1, 3)
    host["layout"] = layout.get()
    return tree, host


def host_dict(st):
    return {k: st.arrays[k] for k, _ in po.STATE_FIELDS if k in sx.DTYPES}


def sorted_state(st, box, ora):
    """sort a host state by Hilbert key (the sync the reference does before every step)"""
    keys = ora.sfc_keys(st, box).copy()
    o = np.argsort(keys, kind="stable")
    for k in po.CONSERVED:
        st.arrays[k][:] = st.arrays[k][o]
    st.keys[:] = keys[o]
    return st


def rows_sorted(nbr, nc, ngmax):
    """neighbor lists as sorted rows (CPU layout), only the first min(nc-1, ngmax) entries"""
    out = []
    n = nc.size
    m = nbr.reshape(n, ngmax)
    for i in range(n):
        c = min(int(nc[i]) - 1, ngmax)
        out.append(np.sort(m[i, :c]))
    return out


def close(a, b, rtol, atol_frac=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.max(np.abs(b)) if b.size else 0.0
    tol = rtol * np.abs(b) + atol_frac * scale
    bad = np.abs(a - b) > tol
    return not bad.any(), (np.nonzero(bad)[0][:5], np.max(np.abs(a - b) / (np.abs(b) + 1e-300)) if b.size else 0)


class StepChecker:
    """Per-particle, scale-aware comparison of one GPU step with one oracle step taken FROM THE SAME STATE
    (SURVEY.md 8(c) tiers 1-3; no global max-based floor).  Multi-step tests shadow the GPU trajectory: before every
    step the oracle is handed the GPU's conserved state, so each step is checked as a map from identical inputs
    (the divergence of two independent float trajectories is a property of the dynamics, not of the kernels).

    The oracle exports, for the step it just ran, the magnitude of the terms of every float sum per particle
    (pyoracle Lib.scales_on: du, a, divv/curlv, gradh, alpha).  Rates and fields formed from neighbor sums must
    agree within rtol*scale_i.  The integrated fields carry the per-particle bounds propagated through the
    reference integrator (positions.hpp:77-88 positionUpdate, :54-61 energyUpdate) from identical inputs:
        E_v  = t_a (dt_m1/2 + dt),   E_dX = t_a (dt_m1 + dt) dt / 2,   t_a = rtol*S_a
        E_x  = E_dX (positions compared as minimum-image displacements: the tier-3 |dx| bound),
        E_u  = t_du (dt + dt^2/(2 dt_m1)),  temp: E_u / cv,   t_du = rtol*S_du
    plus the float32 storage rounding of each stored value.  nc and h must be bit-exact.
    """

    RATE_SCALES = {"du": "du", "ax": "a", "ay": "a", "az": "a", "divv": "dv", "curlv": "dv", "dV11": "dv",
                   "dV12": "dv", "dV13": "dv", "dV22": "dv", "dV23": "dv", "dV33": "dv", "gradh": "gradh"}
    CONSERVED = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]

    def __init__(self, ora, rtol=2e-5, cv=None, periodic=(True, True, True), box_len=(1.0, 1.0, 1.0)):
        self.ora, self.rtol = ora, rtol
        self.cv = cv if cv is not None else po.ideal_gas_cv()
        self.periodic, self.L = periodic, box_len
        self.worst = {}
        self.steps = 0

    def step_oracle_from(self, sim, box, params=None):
        """hand the oracle the GPU's current conserved state and advance it one step, exporting the error
        scales; returns the oracle state"""
        g = sim.get(self.CONSERVED)
        ref = po.HostState(g["id"].size)
        for k in self.CONSERVED:
            ref.arrays[k][:] = g[k]
        sc = sim.scalars()
        ref.minDt, ref.minDt_m1, ref.ttot = sc["minDt"], sc["minDt_m1"], sc["ttot"]
        scales = self.ora.scales_on(ref.n)
        try:
            self.ora.step(ref, box, params=params)
        finally:
            self.ora.scales_off()
        self.ref, self.sc = ref, {k: v.copy() for k, v in scales.items()}
        self.steps += 1
        return ref

    def _bound(self, name, got, b, scale):
        a = np.asarray(got, np.float64)
        b = np.asarray(b, np.float64)
        err = np.abs(a - b)
        bad = err > scale
        w = float(np.max(err / (scale + 1e-300))) if a.size else 0.0
        self.worst[name] = max(self.worst.get(name, 0.0), w)
        assert not bad.any(), (f"step {self.steps}", name, int(bad.sum()), np.nonzero(bad)[0][:5], w)

    def check(self, got, fields):
        ref, sc, rt = self.ref, self.sc, self.rtol
        og, orf = np.argsort(got["id"]), np.argsort(ref.id)
        assert np.array_equal(got["id"][og], ref.id[orf])
        assert np.array_equal(got["nc"][og], ref.nc[orf])
        assert np.array_equal(got["h"][og], ref.h[orf])
        R = {f: ref.arrays[f][orf] for f in ref.arrays}
        G = {f: got[f][og] for f in got}
        S = {kk: v[orf] for kk, v in sc.items()}
        f32 = 2.0 ** -23
        dt, dtm1 = ref.minDt, ref.minDt_m1
        ta, tdu = rt * S["a"], rt * S["du"]
        for f in fields:
            if f in self.RATE_SCALES:
                self._bound(f, G[f], R[f], rt * S[self.RATE_SCALES[f]] + f32 * np.abs(R[f]))
            elif f in ("xm", "kx", "prho", "c", "rho", "p"):
                self._bound(f, G[f], R[f], rt * np.abs(R[f]) + 1e-30)
            elif f in ("c11", "c12", "c13", "c22", "c23", "c33"):
                diag = np.maximum(np.maximum(np.abs(R["c11"]), np.abs(R["c22"])), np.abs(R["c33"]))
                self._bound(f, G[f], R[f], rt * diag)
            elif f == "alpha":
                self._bound(f, G[f], R[f], rt * (np.abs(R[f]) + S["alpha"]))
        Ev = ta * (0.5 * dtm1 + dt)
        EdX = ta * 0.5 * (dtm1 + dt) * dt
        Eu = tdu * (dt + dt * dt / (2 * dtm1))
        for c, comp in enumerate("xyz"):
            if "v" + comp in fields:
                self._bound("v" + comp, G["v" + comp], R["v" + comp], Ev + f32 * np.abs(R["v" + comp]))
            if comp + "_m1" in fields:
                self._bound(comp + "_m1", G[comp + "_m1"], R[comp + "_m1"], EdX + f32 * np.abs(R[comp + "_m1"]))
            if comp in fields:
                d = G[comp].astype(np.float64) - R[comp]
                if self.periodic[c]:
                    d -= self.L[c] * np.rint(d / self.L[c])
                self._bound(comp, d, np.zeros_like(d), EdX + 2.0 ** -52 * np.abs(R[comp]) + 1e-300)
        if "temp" in fields:
            self._bound("temp", G["temp"], R["temp"], Eu / self.cv + 1e-15 * np.abs(R["temp"]))
        if "du_m1" in fields:
            self._bound("du_m1", G["du_m1"], R["du_m1"], tdu + f32 * np.abs(R["du_m1"]))


def shadow_steps(ctx, ora, sim, obox, steps, params, fields, on_step=None):
    """run `steps` GPU steps of sim, each checked per particle against one oracle step from the same state"""
    lim = list(obox.lim)
    chk = StepChecker(ora, periodic=tuple(bool(obox.bnd[d] == 1) for d in range(3)),
                      box_len=tuple(lim[2 * d + 1] - lim[2 * d] for d in range(3)))
    for s in range(steps):
        ref = chk.step_oracle_from(sim, obox, params)
        sim.step()
        chk.check(sim.get(["id", "nc", "h"] + fields), fields)
        sc = sim.scalars()
        assert sc["minDt"] == np.float64(ref.minDt) or abs(sc["minDt"] / ref.minDt - 1) < 1e-5
        assert abs(sc["ttot"] / ref.ttot - 1) < 1e-5
        if on_step is not None:
            on_step(s, sim, ref)
    print({k: f"{v:.2g}" for k, v in chk.worst.items()})
    return chk
