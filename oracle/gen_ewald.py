"""Golden vectors of the reference's Ewald correction (TEST INFRASTRUCTURE): runs oracle/_ref/libewald_ref.so
(ryoanji::computeGravityEwald compiled from /root/reference, oracle/ewald_ref.cpp) on a seeded periodic cube and writes
tests/golden/ewald_ref.npz (inputs, root moments, and per setting the accelerations and energy).
    python oracle/gen_ewald.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ewald as ew  # noqa: E402

CASES = {"nrs1": dict(numReplicaShells=1), "nrs0": dict(numReplicaShells=0),
         "nrs2_l1": dict(numReplicaShells=2, lCut=1.0, hCut=2.0, alpha_scale=1.5)}


def ref_lib():
    import ctypes
    lib = ctypes.CDLL(os.path.join(HERE, "_ref", "libewald_ref.so"))
    lib.ref_gravity_ewald.restype = ctypes.c_double
    return lib


def run_ref(lib, x, y, z, m, M, c, lo, hi, G, s):
    import ctypes
    P = ctypes.c_void_p
    ax = np.zeros(len(x), np.float32)
    ay, az = ax.copy(), ax.copy()
    s = {**ew.SETTINGS, **s}
    e = lib.ref_gravity_ewald(c.ctypes.data_as(P), M.ctypes.data_as(P), ctypes.c_uint(len(x)), x.ctypes.data_as(P),
                              y.ctypes.data_as(P), z.ctypes.data_as(P), m.ctypes.data_as(P), ctypes.c_double(lo),
                              ctypes.c_double(hi), ctypes.c_float(G), ctypes.c_int(s["numReplicaShells"]),
                              ctypes.c_double(s["lCut"]), ctypes.c_double(s["hCut"]), ctypes.c_double(s["alpha_scale"]),
                              ctypes.c_double(s["small_R_scale_factor"]), ax.ctypes.data_as(P), ay.ctypes.data_as(P),
                              az.ctypes.data_as(P))
    return e, ax, ay, az


def root_moments(x, y, z, m):
    """mass, center of mass and traceless quadrupole (CartesianQuadrupole layout, P2M of cartesian_qpole.hpp)"""
    mt = m.astype(np.float64).sum()
    c = np.array([(x * m).sum(), (y * m).sum(), (z * m).sum()]) / mt
    rx, ry, rz = x - c[0], y - c[1], z - c[2]
    g = np.zeros(8, np.float32)
    g[0] = mt
    g[1], g[2], g[3] = (rx * rx * m).sum(), (rx * ry * m).sum(), (rx * rz * m).sum()
    g[4], g[5], g[6] = (ry * ry * m).sum(), (ry * rz * m).sum(), (rz * rz * m).sum()
    tr = g[1] + g[4] + g[6]
    g[7] = tr
    g[1], g[4], g[6] = 3 * g[1] - tr, 3 * g[4] - tr, 3 * g[6] - tr
    return g, c


def cube(n=400, seed=5, lo=-0.5, hi=0.5):
    rng = np.random.default_rng(seed)
    x, y, z = (rng.uniform(lo, hi, n) for _ in range(3))
    # targets near the expansion center exercise the small-R series (ewald.hpp:270-291)
    x[:20], y[:20], z[:20] = (rng.normal(0, 0.01, 20) for _ in range(3))
    m = (rng.uniform(0.5, 1.5, n) / n).astype(np.float32)
    return x, y, z, m


if __name__ == "__main__":
    lo, hi, G = -0.5, 0.5, 1.0
    x, y, z, m = cube()
    M, c = root_moments(x, y, z, m)
    lib = ref_lib()
    out = dict(x=x, y=y, z=z, m=m, M=M, center=c, box=np.array([lo, hi]), G=np.array([G]))
    for k, s in CASES.items():
        e, ax, ay, az = run_ref(lib, x, y, z, m, M, c, lo, hi, G, s)
        out[f"{k}_egrav"] = np.array([e])
        out[f"{k}_acc"] = np.stack([ax, ay, az])
    path = os.path.join(HERE, "..", "tests", "golden", "ewald_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", os.path.normpath(path))
