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
