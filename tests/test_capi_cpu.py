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
