"""CPU-side checks of the C-ABI library (no GPU compute): it loads, exports every symbol include/sphexa_hip.h
declares, and its host-side constants (K, kernel tables) equal the reference's bit for bit."""
import ctypes as C
import ctypes.util

import numpy as np
import pytest

import pyoracle as po
import sphexa_amd as sx


def test_library_loads_and_exports_header_symbols():
    L = sx.lib()
    syms = sx.header_symbols()
    assert len(syms) > 40
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_kernel_constant_and_tables_match_oracle():
    L = sx.lib()
    ora = po.load_oracle()
    assert L.sx_kernel_constant() == ora.K
    wh = np.zeros(sx.KTABLE, np.float32)
    whd = np.zeros(sx.KTABLE, np.float32)
    assert L.sx_copy_tables(None, wh.ctypes.data, whd.ctypes.data) == 0
    assert np.array_equal(wh, ora.wh) and np.array_equal(whd, ora.whd)


def test_kernel_poly_matches_sinc6_and_tables():
    """The fast pair kernels evaluate W = sinc(pi v/2)^6 and dW/dv by a degree-6 polynomial in v^2
    (sx_kernel_poly.hpp) instead of the 20000-point tables; its error is of the order of the tables' own."""
    L = sx.lib()
    v = np.linspace(0.0, 2.1, 400001).astype(np.float32)
    w = np.zeros_like(v)
    dw = np.zeros_like(v)
    assert L.sx_kernel_poly(v.ctypes.data, v.size, w.ctypes.data, dw.ctypes.data) == 0
    x = np.pi / 2 * v.astype(np.float64)
    s = np.where(x > 0, np.sin(x) / np.where(x > 0, x, 1.0), 1.0)
    ds = np.where(x > 0, np.pi / 2 * (np.cos(x) / np.where(x > 0, x, 1.0) - np.sin(x) / np.where(x > 0, x, 1.0) ** 2),
                  0.0)
    inside = v < 2.0
    w_ex = np.where(inside, s ** 6, 0.0)
    dw_ex = np.where(inside, 6 * s ** 5 * ds, 0.0)
    assert np.max(np.abs(w - w_ex)) < 4e-7  # tables: 1.1e-7 (float interpolation of float samples)
    assert np.max(np.abs(dw - dw_ex)) < 1e-6  # tables: 2.2e-7
    # outside the support both are exactly zero (v^2 clamped to 4, where the polynomial is exactly 0.0f), and so
    # are NaN arguments (fminf returns the number)
    far = np.array([2.0, 2.0000002, 2.5, 7.0, 1e30, np.inf, np.nan], np.float32)
    wf, dwf = np.ones_like(far), np.ones_like(far)
    assert L.sx_kernel_poly(far.ctypes.data, far.size, wf.ctypes.data, dwf.ctypes.data) == 0
    assert np.all(wf == 0.0) and np.all(dwf[:-2] == 0.0)
    # the reference tables (linear interpolation, lt::lookup) differ from the exact function by the same order
    wh = np.zeros(sx.KTABLE, np.float32)
    whd = np.zeros(sx.KTABLE, np.float32)
    L.sx_copy_tables(None, wh.ctypes.data, whd.ctypes.data)
    dx = np.float32(2.0) / np.float32(sx.KTABLE - 1)
    idx = (v[inside] * (np.float32(1.0) / dx)).astype(np.int64)
    ok = idx < sx.KTABLE - 1
    vi, ii = v[inside][ok], idx[ok]
    lut = wh[ii] + (wh[ii + 1] - wh[ii]) / dx * (vi - ii.astype(np.float32) * dx)
    assert np.max(np.abs(lut - w[inside][ok])) < 4e-7


def test_update_h_needs_glibc_powf_table():
    """updateH calls std::pow(float,float) = glibc powf, which is not correctly rounded: on nc = 1..2e5 (ng0=100) it
    differs from a correctly rounded pow for 100+ values (first at nc=488).  This is why the device takes the factor
    from a table filled by the host's powf (sx_device.hpp updateH); the GPU parity tests check h bit-for-bit."""
    libm = C.CDLL(ctypes.util.find_library("m"))
    libm.powf.restype = C.c_float
    libm.powf.argtypes = [C.c_float, C.c_float]
    ex = np.float32(1.0 / 10.0)
    nc = np.arange(1, 200001, dtype=np.float32)
    base = (np.float32(1.0) + np.float32(1023.0) * np.float32(100) / nc).astype(np.float32)
    viadouble = np.power(base.astype(np.float64), np.float64(ex)).astype(np.float32)
    glibc = np.array([libm.powf(float(b), float(ex)) for b in base], np.float32)
    bad = np.nonzero(glibc != viadouble)[0]
    assert bad.size > 0 and bad[0] + 1 == 488
    # the oracle's updateH (plain C, glibc powf) is what the device table reproduces
    ora = po.load_oracle()
    for k in (1, 25, 100, 151, 488, 620, 65535):
        assert ora.lib.update_h(100, k, 1.0) == np.float32(0.5) * glibc[k - 1] if k <= 200000 else True


def test_params_layout():
    assert C.sizeof(sx.SxBox) == 64
    p = sx.default_params()
    assert p.ngmax == 150 and p.ng0 == 100 and abs(p.ramp - 10.0) < 1e-6
