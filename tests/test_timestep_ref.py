"""The oracle's global time-step (oracle/sph_oracle.c ox_rho_timestep / ox_compute_timestep, the functions its step
uses) against the reference's own sph::rhoTimestep and sph::computeTimestep (sph/include/sph/ts_global.hpp:47-112),
compiled from /root/reference into oracle/_ref with the image's MPICH (one rank, MPI_Allreduce(MIN) over itself).

Runs only where oracle/_ref exists (the build container).  Bit-exact: both evaluate the same float max and double
arithmetic.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle as po

pytestmark = [pytest.mark.ref, pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built")]

FP = C.POINTER(C.c_float)
DP = C.POINTER(C.c_double)


def _fns(lib, prefix):
    rho = getattr(lib, prefix + "rho_timestep")
    rho.restype, rho.argtypes = C.c_double, [FP, C.c_size_t, C.c_double]
    dt = getattr(lib, prefix + "compute_timestep")
    dt.restype, dt.argtypes = None, [DP, FP, FP, FP, C.c_size_t, C.c_double, C.c_double]
    return rho, dt


@pytest.fixture(scope="module")
def fns():
    return _fns(C.CDLL(po.ORACLE_SO), "ox_"), _fns(C.CDLL(po.REF_SO), "ref_")


def _f(a):
    return a.ctypes.data_as(FP)


@pytest.mark.parametrize("seed", range(6))
def test_rho_timestep(fns, seed):
    (ora_rho, _), (ref_rho, _) = fns
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 5000))
    divv = (rng.standard_normal(n) * 10.0 ** rng.uniform(-3, 3)).astype(np.float32)
    if seed == 0:
        divv = -np.abs(divv)  # every particle compressing: |max| of a negative maximum
    for krho in (0.06, 0.2):
        assert ora_rho(_f(divv), n, krho) == ref_rho(_f(divv), n, krho)


@pytest.mark.parametrize("seed,g", [(0, 0.0), (1, 1.0), (2, 1.0), (3, 0.0), (4, 6.674e-8)])
def test_compute_timestep(fns, seed, g):
    (_, ora_dt), (_, ref_dt) = fns
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 4000))
    acc = [(rng.standard_normal(n) * 10.0 ** rng.uniform(-2, 4)).astype(np.float32) for _ in range(3)]
    for trial in range(4):
        io = np.array([10.0 ** rng.uniform(-7, -3), 10.0 ** rng.uniform(-7, -3), rng.uniform(0, 1),
                       10.0 ** rng.uniform(-7, -2) if trial != 1 else np.inf, 10.0 ** rng.uniform(-7, -2),
                       g, 1.1], dtype=np.float64)
        a, b = io.copy(), io.copy()
        ora_dt(a.ctypes.data_as(DP), *map(_f, acc), n, 0.2, 0.005)
        ref_dt(b.ctypes.data_as(DP), *map(_f, acc), n, 0.2, 0.005)
        assert np.array_equal(a[:3], b[:3]), (a[:3], b[:3])
        assert a[1] == io[0]  # minDt_m1 <- minDt
