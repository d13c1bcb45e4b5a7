"""Golden vectors of the reference's periodic Barnes-Hut walk (TEST INFRASTRUCTURE): ryoanji::computeGravity with
numShells = 1 (traversal_cpu.hpp:166-230, the 27 images of the box; oracle/_ref, ref_set_gravity_shells) on a
key-sorted, perturbed lattice with varying masses in a periodic cube, plus the root expansion for the Ewald correction
(sx_gravity_ewald).  Writes tests/golden/grav_pbc_ref.npz.
    python oracle/gen_grav_pbc.py"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402


def state(side=14, seed=7):
    st, box = po.sedov_state(side)
    rng = np.random.default_rng(seed)
    dx = 1.0 / side
    for k in ("x", "y", "z"):
        a = st.arrays[k]
        a[:] = np.clip(a + rng.uniform(-0.3, 0.3, a.size) * dx, -0.5 + 1e-9, 0.5 - 1e-9)
    st.m[:] = (rng.uniform(0.5, 1.5, st.n) / st.n).astype(np.float32)
    st.ax[:] = 0
    st.ay[:] = 0
    st.az[:] = 0
    return st, box


if __name__ == "__main__":
    ora = po.load_oracle()
    ref = po.load_ref()
    st, box = state()
    keys = ora.sfc_keys(st, box).copy()
    o = np.argsort(keys, kind="stable")
    for k in po.CONSERVED:
        st.arrays[k][:] = st.arrays[k][o]
    st.keys[:] = keys[o]
    out = {k: st.arrays[k].copy() for k in ("x", "y", "z", "h", "m")}
    out["box"] = np.array(list(box.lim) + list(box.bnd), np.float64)
    for shells in (1, 0):
        C.CDLL(po.REF_SO).ref_set_gravity_shells(shells)
        a = st.copy()
        eg, cen, mp = ref.gravity(a, box, ref.params(g=1.0, theta=0.5))
        out[f"shells{shells}_acc"] = np.stack([a.ax, a.ay, a.az])
        out[f"shells{shells}_egrav"] = np.array([eg])
        if shells == 1:
            out["centers"], out["multipoles"] = cen, mp
    C.CDLL(po.REF_SO).ref_set_gravity_shells(0)
    path = os.path.join(HERE, "..", "tests", "golden", "grav_pbc_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", os.path.normpath(path), st.n, "particles; |a| max shells 1/0:",
          np.abs(out["shells1_acc"]).max(), np.abs(out["shells0_acc"]).max())
