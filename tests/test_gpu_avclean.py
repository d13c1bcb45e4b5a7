"""AV cleaning (HydroVeProp<avClean=true>, ve_hydro.hpp:50-85) on the GPU against the CPU oracle, whose avClean
path is pinned bit-for-bit to the reference template in tests/test_oracle_vs_ref.py::test_full_steps_av_clean.

* kernels on the oracle's own neighbor list (imported): velocity gradient dV11..dV33 from the IAD kernel
  (divv_curlv_kern.hpp:113-121) and the avClean momentum kernel (avRvCorrection, momentum_energy_kern.hpp:43-63).
  Exact variant: bitwise, except that exp() inside avRvCorrection is evaluated in double and rounded once (glibc's
  expf agrees wherever it is correctly rounded), so du/a are allowed a few float ulps (4e-7 relative to |term|);
  fast variant: the FMA tolerance of test_gpu_parity.py.
* full avClean steps of sx_sim (own search, cluster kernels) within the full-step tolerance.
"""
import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx
from test_gpu_parity import fast_tolerance_scale, kernel_chain, run_checked_steps, FLOATS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def avclean_fixture(ora, side=14, steps=2):
    """a Sedov state with flow (after `steps` avClean oracle steps), its neighbor list and the oracle outputs"""
    st, box = po.sedov_state(side)
    p = ora.params(av_clean=True)
    for _ in range(steps):
        ora.step(st, box, params=p)
    gutil.sorted_state(st, box, ora)
    d = {"box": np.array(list(box.lim) + list(box.bnd), np.float64)}
    for k, _ in po.STATE_FIELDS:
        d["in_" + k] = st.arrays[k].copy()
    d["in_scalars"] = np.array([st.minDt, st.minDt_m1, st.ttot, st.minDtCourant, st.minDtRho])
    nbr, nc = ora.find_neighbors(st, box)
    st.nc[:] = nc
    d["nbr"], d["nc"], d["h_after_iter"] = nbr, nc, st.h.copy()
    ora.xmass(st, box, nbr, params=p)
    ora.ve_def_gradh(st, box, nbr, params=p)
    ora.eos(st, params=p)
    ora.iad_divv_curlv(st, box, nbr, params=p)
    ora.av_switches(st, box, nbr, params=p)
    mdt = ora.momentum_energy(st, box, nbr, params=p)
    for k in ["xm", "kx", "gradh", "prho", "c", "c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv", "alpha",
              "du", "ax", "ay", "az", "dV11", "dV12", "dV13", "dV22", "dV23", "dV33"]:
        d[k] = st.arrays[k].copy()
    d["minDtCourant"] = np.array([mdt])
    return d


GRAD = ["dV11", "dV12", "dV13", "dV22", "dV23", "dV33"]
OUT = ["xm", "kx", "gradh", "prho", "c", "c11", "c22", "c33", "divv", "alpha"] + GRAD + ["du", "ax", "ay", "az"]


def test_avclean_kernels_exact(ctx, ora):
    d = avclean_fixture(ora)
    assert np.any(d["dV11"] != 0)
    out = kernel_chain(ctx, d, exact=True, av_clean=True)
    for k in OUT:
        a, b = out[k], d[k].astype(out[k].dtype)
        if k in ("du", "ax", "ay", "az"):
            scale = fast_tolerance_scale(k, d)
            assert np.all(np.abs(a.astype(np.float64) - b) <= 4e-7 * scale + 1e-9 * np.max(np.abs(b))), k
        else:
            assert np.array_equal(a, b), (k, np.max(np.abs(a.astype(np.float64) - b)))
    ctx.free_all()


def test_avclean_kernels_fast(ctx, ora):
    d = avclean_fixture(ora)
    out = kernel_chain(ctx, d, exact=False, av_clean=True)
    for k in OUT:
        a, b = out[k].astype(np.float64), d[k].astype(np.float64)
        scale = fast_tolerance_scale(k, d) if not k.startswith("dV") else np.full(b.size, 10 * np.max(np.abs(b)))
        assert np.all(np.abs(a - b) <= 2e-5 * scale + 1e-6 * np.max(np.abs(b))), (k, np.max(np.abs(a - b)))
    ctx.free_all()


def test_avclean_changes_momentum(ctx, ora):
    d = avclean_fixture(ora)
    a = kernel_chain(ctx, d, exact=True, av_clean=True)
    b = kernel_chain(ctx, d, exact=True, av_clean=False)
    assert not np.array_equal(a["ax"], b["ax"])
    ctx.free_all()


@pytest.mark.parametrize("ic,side,steps", [("sedov", 16, 3), ("noh", 16, 2)])
def test_avclean_full_steps(ctx, ora, ic, side, steps):
    """per-particle checks (gpu_util.StepChecker) of whole avClean steps against the oracle"""
    st, obox = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    run_checked_steps(ctx, ora, st, obox, steps, av_clean=True).close()
