"""Ewald periodic-gravity correction: numpy restatement -- TEST INFRASTRUCTURE ONLY (the checker of the GPU's
sx_gravity_ewald; never imported by the product path).

Follows ryoanji/src/ryoanji/nbody/ewald.hpp with the types of the GPU seam's instantiation
(ryoanji/interface/ewald.cu:104: CartesianQuadrupole<float>, double coordinates, float accelerations):
  * ewald_params      -- ewaldInitParameters (ewald.hpp:149-214): the k-space coefficients, each gamma and mfac
                         evaluated in float (EwaldParameters<double, float>, ewaldEvalMultipoleComplete<float,...>)
  * real_space        -- computeEwaldRealSpace (ewald.hpp:224-325): image sum in double, gamma rounded to float
  * k_space           -- computeEwaldKSpace (ewald.hpp:327-351)
  * gravity_ewald     -- computeGravityEwald (ewald.hpp:380-413): a += G (real + k), returns 0.5 G sum m phi
Pinned to the reference compiled from its own header (oracle/ewald_ref.cpp -> oracle/_ref/libewald_ref.so) by
tests/test_ewald_oracle.py, and through the committed fixture tests/golden/ewald_ref.npz where the reference is absent.
"""
import math

import numpy as np

F = np.float32
SETTINGS = dict(numReplicaShells=1, lCut=2.6, hCut=2.8, alpha_scale=2.0, small_R_scale_factor=3.0e-3)  # ewald.h:17-21
MASS, QXX, QXY, QXZ, QYY, QYZ, QZZ, TRACE = range(8)  # Cqi (cartesian_qpole.hpp:59-71)


def _quad(M):
    """the traceless moments / 3 as the reference forms them (float): qxx, qyy, qzz, qxy, qxz, qyz"""
    t3 = F(3)
    return ((M[QXX] + M[TRACE]) / t3, (M[QYY] + M[TRACE]) / t3, (M[QZZ] + M[TRACE]) / t3, M[QXY] / t3, M[QXZ] / t3,
            M[QYZ] / t3)


def _eval_potential_f32(hr, gamma, M):
    """ewaldEvalMultipoleComplete<Ta = float, Tc = double, Tmm = float>(...)[0] (ewald.hpp:106-131) for one hr"""
    r = [F(v) for v in hr]
    qxx, qyy, qzz, qxy, qxz, qyz = _quad(M)
    Qr = (r[0] * qxx + r[1] * qxy + r[2] * qxz, r[0] * qxy + r[1] * qyy + r[2] * qyz,
          r[0] * qxz + r[1] * qyz + r[2] * qzz)
    rQr = F(0.5 * float(r[0] * Qr[0] + (r[1] * Qr[1] + r[2] * Qr[2])))  # dot: a right fold (util/array.hpp:255)
    Qtr = F(0.5 * float(M[TRACE]))
    return float((-gamma[0]) * M[MASS] + gamma[1] * Qtr - gamma[2] * rQr)


def ewald_params(Mroot, center, L, numReplicaShells=1, lCut=2.6, hCut=2.8, alpha_scale=2.0,
                 small_R_scale_factor=3.0e-3):
    """ewaldInitParameters (ewald.hpp:149-214): dict with the shells and the k-space table hs (K x 3, double) and
    hfac (K x 2: cos, sin)"""
    M = np.asarray(Mroot, dtype=F)
    if lCut == 0 and hCut == 0 and alpha_scale == 0:
        numReplicaShells = 0
    p = dict(M=M, center=np.asarray(center, dtype=np.float64), L=float(L), numReplicaShells=numReplicaShells,
             numEwaldShells=max(int(math.ceil(lCut)), numReplicaShells), lCut=lCut, hCut=hCut,
             alpha_scale=alpha_scale, small_R_scale_factor=small_R_scale_factor, hs=np.zeros((0, 3)),
             hfac=np.zeros((0, 2)))
    if p["numEwaldShells"] == 0:
        return p
    hReps = int(math.ceil(hCut))
    alpha = alpha_scale / L
    k4 = math.pi * math.pi / (alpha * alpha * L * L)
    hCut2 = hCut * hCut
    hs, hfac = [], []
    for hx in range(-hReps, hReps + 1):
        for hy in range(-hReps, hReps + 1):
            for hz in range(-hReps, hReps + 1):
                h2 = float(hx * hx + hy * hy + hz * hz)
                if h2 == 0 or h2 > hCut2:
                    continue
                g0 = F(math.exp(-k4 * h2) / (math.pi * h2 * L))
                g1 = F(2 * math.pi / L * float(g0))
                g2 = F(-2 * math.pi / L * float(g1))
                g3 = F(2 * math.pi / L * float(g2))
                g4 = F(-2 * math.pi / L * float(g3))
                g5 = F(2 * math.pi / L * float(g4))
                z = F(0)
                hr = (float(hx), float(hy), float(hz))
                mcos = _eval_potential_f32(hr, (g0, z, g2, z, g4, z), M)
                msin = _eval_potential_f32(hr, (z, g1, z, g3, z, g5), M)
                hs.append([2 * math.pi / L * hr[0], 2 * math.pi / L * hr[1], 2 * math.pi / L * hr[2]])
                hfac.append([mcos, msin])
    p["hs"] = np.array(hs, dtype=np.float64)
    p["hfac"] = np.array(hfac, dtype=np.float64)
    return p


def _c_libm():
    import ctypes
    import ctypes.util
    lib = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
    fns = {}
    for name in ("exp", "erf", "erfc", "cos", "sin"):
        f = getattr(lib, name)
        f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
        fns[name] = f
    return fns


_LIBM = _c_libm()


def _libm(name, x):
    """the C library's function per element, as the reference calls it (numpy's vectorized exp/cos/sin and Python's
    own erf may round differently from the C library's)"""
    f = _LIBM[name]
    return np.array([f(float(v)) for v in np.ravel(x)], dtype=np.float64).reshape(np.shape(x))


def _erf(x):
    return _libm("erf", x)


def _erfc(x):
    return _libm("erfc", x)


def real_space(x, y, z, p):
    """computeEwaldRealSpace (ewald.hpp:224-325) for arrays of targets: (phi, ax, ay, az) in double"""
    M, L = p["M"], p["L"]
    nE, nR = p["numEwaldShells"], p["numReplicaShells"]
    lCut2 = p["lCut"] * p["lCut"] * L * L
    alpha = p["alpha_scale"] / L
    alpha2 = alpha * alpha
    k1 = math.pi / (alpha2 * L * L * L)
    ka = 2.0 * alpha / math.sqrt(math.pi)
    smallR2 = p["small_R_scale_factor"] * L * L
    qxx, qyy, qzz, qxy, qxz, qyz = _quad(M)
    Qtr = np.float64(0.5 * float(M[TRACE]))  # Ta = double (a float times it is promoted)
    n = len(x)
    pot = np.full(n, k1 * float(M[MASS]))
    acc = [np.zeros(n), np.zeros(n), np.zeros(n)]
    r = [np.asarray(x, np.float64) - p["center"][0], np.asarray(y, np.float64) - p["center"][1],
         np.asarray(z, np.float64) - p["center"][2]]
    for ix in range(-nE, nE + 1):
        for iy in range(-nE, nE + 1):
            for iz in range(-nE, nE + 1):
                pre = max(abs(ix), abs(iy), abs(iz)) <= nR
                R = [r[0] + ix * L, r[1] + iy * L, r[2] + iz * L]
                R2 = R[0] * R[0] + (R[1] * R[1] + R[2] * R[2])  # norm2 = dot, a right fold
                use = np.ones(n, bool) if pre else (R2 <= lCut2)
                if not use.any():
                    continue
                g = [np.zeros(n, F) for _ in range(6)]
                small = (R2 < smallR2) & (ka > 0) & use
                big = use & ~small
                if small.any():
                    R2a2 = R2[small] * alpha2
                    c0 = ka
                    for k, (num, den) in enumerate([(3.0, 1.0), (5.0, 1.0 / 3.0), (7.0, 1.0 / 5.0), (9.0, 1.0 / 7.0),
                                                    (11.0, 1.0 / 9.0), (13.0, 1.0 / 11.0)]):
                        if k > 0:
                            c0 *= 2 * alpha2
                        g[k][small] = (c0 * (R2a2 / num - den)).astype(F)
                if big.any():
                    Rb = R2[big]
                    Rmag = np.sqrt(Rb)
                    invR = 1.0 / Rmag
                    invR2 = invR * invR
                    a = _libm("exp", -Rb * alpha2) * ka * invR2
                    fn = -_erf(alpha * Rmag) if pre else _erfc(alpha * Rmag)
                    alphan = 1.0
                    gb = [None] * 6
                    gb[0] = (fn * invR).astype(F)
                    gb[1] = (gb[0] * invR2 + a).astype(F)
                    for k, c in ((2, 3), (3, 5), (4, 7), (5, 9)):
                        alphan *= 2 * alpha2
                        gb[k] = ((c * gb[k - 1]) * invR2 + alphan * a).astype(F)
                    for k in range(6):
                        g[k][big] = gb[k]
                # ewaldEvalMultipoleComplete<double, double, float> (ewald.hpp:106-131)
                Qr = [R[0] * qxx + R[1] * qxy + R[2] * qxz, R[0] * qxy + R[1] * qyy + R[2] * qyz,
                      R[0] * qxz + R[1] * qyz + R[2] * qzz]
                rQr = 0.5 * (R[0] * Qr[0] + (R[1] * Qr[1] + R[2] * Qr[2]))
                ug = ((-g[0]) * M[MASS]).astype(np.float64) + g[1] * Qtr - g[2] * rQr
                inner = (g[1] * M[MASS]).astype(np.float64) - g[2] * Qtr + g[3] * rQr
                pot = np.where(use, pot + ug, pot)
                for d in range(3):
                    acc[d] = np.where(use, acc[d] + (g[2] * Qr[d] - R[d] * inner), acc[d])
    return pot, acc[0], acc[1], acc[2]


def k_space(x, y, z, p):
    """computeEwaldKSpace (ewald.hpp:327-351)"""
    n = len(x)
    pot = np.zeros(n)
    acc = [np.zeros(n), np.zeros(n), np.zeros(n)]
    dr = [np.asarray(x, np.float64) - p["center"][0], np.asarray(y, np.float64) - p["center"][1],
          np.asarray(z, np.float64) - p["center"][2]]
    for (h0, h1, h2), (fc, fs) in zip(p["hs"], p["hfac"]):
        hx = h0 * dr[0] + (h1 * dr[1] + h2 * dr[2])  # dot, a right fold (util/array.hpp:255)
        c, s = _libm("cos", hx), _libm("sin", hx)
        cs_sum = fc * c + fs * s
        cs_diff = fc * s - fs * c
        pot -= cs_sum
        acc[0] += cs_diff * h0
        acc[1] += cs_diff * h1
        acc[2] += cs_diff * h2
    return pot, acc[0], acc[1], acc[2]


def gravity_ewald(x, y, z, m, Mroot, center, L, G, ax, ay, az, **settings):
    """computeGravityEwald (ewald.hpp:380-413): ax, ay, az (float32 arrays) += G (real + k); returns the energy
    0.5 G sum m phi"""
    G = float(np.float32(G))  # the seam's G is a float (computeGravityEwald(..., float G, ...))
    s = dict(SETTINGS)
    s.update(settings)
    p = ewald_params(Mroot, center, L, **s)
    if p["numEwaldShells"] == 0:
        return 0.0
    pr = real_space(x, y, z, p)
    pk = k_space(x, y, z, p)
    pot = pr[0] + pk[0]
    for d, a in enumerate((ax, ay, az)):
        a[:] = (a.astype(np.float64) + G * (pr[d + 1] + pk[d + 1])).astype(F)
    return 0.5 * G * float(np.sum(pot * np.asarray(m, np.float64)))
