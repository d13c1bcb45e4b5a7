"""The oracle restatement against the live reference build (oracle/_ref) on fresh inputs.

Runs only where oracle/_ref/libsphexa_ref.so exists (the build container); on the GPU box the golden
fixtures (test_oracle_golden.py) carry the same checks.
"""
import numpy as np
import pytest

import pyoracle as po

pytestmark = [pytest.mark.ref, pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built")]


@pytest.fixture(scope="module")
def ref():
    return po.load_ref()


@pytest.fixture(scope="module")
def ora():
    return po.load_oracle()


def test_tables_and_update_h(ora, ref):
    assert ora.K == ref.K
    assert np.array_equal(ora.wh, ref.wh) and np.array_equal(ora.whd, ref.whd)
    for nc in range(1, 2500):
        for h in (0.013, 0.0725091, 0.9):
            assert ora.lib.update_h(100, nc, h) == ref.lib.update_h(100, nc, h)


def rand_state(n, seed, clustered=True):
    rng = np.random.default_rng(seed)
    st = po.HostState(n)
    st.x[:] = rng.uniform(-0.5, 0.5, n)
    st.y[:] = rng.uniform(-0.5, 0.5, n)
    st.z[:] = np.clip(rng.normal(0, 0.12, n), -0.5, 0.4999) if clustered else rng.uniform(-0.5, 0.5, n)
    return st


@pytest.mark.parametrize("bucket", [64, 16, 1])
@pytest.mark.parametrize("periodic", [True, False])
def test_tree_neighbors(ora, ref, bucket, periodic):
    st = rand_state(6000, 7 + bucket)
    box = po.make_box(-0.5, 0.5, periodic)
    keys = ref.sfc_keys(st, box).copy()
    assert np.array_equal(keys, ora.sfc_keys(st, box))
    o = np.argsort(keys, kind="stable")
    for k in ("x", "y", "z"):
        st.arrays[k][:] = st.arrays[k][o]
    st.keys[:] = keys[o]
    t1, t2 = ref.octree(st.keys, bucket), ora.octree(st.keys, bucket)
    for k in t1:
        assert np.array_equal(t1[k], t2[k]), k
    st.h[:] = np.float32(0.02)
    h0 = st.h.copy()
    for it in (False, True):
        st.h[:] = h0
        n1, c1 = ref.find_neighbors(st, box, bucket=bucket, iterate_h=it)
        h1 = st.h.copy()
        st.h[:] = h0
        n2, c2 = ora.find_neighbors(st, box, bucket=bucket, iterate_h=it)
        assert np.array_equal(c1, c2) and np.array_equal(n1, n2) and np.array_equal(h1, st.h)


@pytest.mark.parametrize("ic,side,steps", [("sedov", 12, 4), ("noh", 14, 4)])
def test_full_steps(ora, ref, ic, side, steps):
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    a, b = st.copy(), st.copy()
    for _ in range(steps):
        ref.step(a, box)
        ora.step(b, box)
        for k in a.arrays:
            assert np.array_equal(a.arrays[k], b.arrays[k]), k
        assert a.minDt == b.minDt


@pytest.mark.parametrize("ic,side,steps", [("sedov", 12, 4), ("noh", 14, 4)])
def test_full_steps_av_clean(ora, ref, ic, side, steps):
    """HydroVeProp<avClean=true>: IAD writes the velocity gradient (divv_curlv_kern.hpp:113-121), momentum adds
    avRvCorrection (momentum_energy_kern.hpp:43-63, 157-161); bit-exact against the reference's template"""
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    a, b = st.copy(), st.copy()
    pr, po_ = ref.params(av_clean=True), ora.params(av_clean=True)
    for _ in range(steps):
        ref.step(a, box, params=pr)
        ora.step(b, box, params=po_)
        for k in a.arrays:
            assert np.array_equal(a.arrays[k], b.arrays[k]), k
        assert a.minDt == b.minDt
    assert np.any(b.dV11 != 0) and not np.array_equal(b.ax, _plain_steps(ora, ic, side, steps).ax)


def _plain_steps(lib, ic, side, steps):
    st, box = (po.sedov_state if ic == "sedov" else po.noh_state)(side)
    for _ in range(steps):
        lib.step(st, box)
    return st
