"""CPU checks behind the multi-rank periodic self-gravity (tests/test_gpu_distributed_pbc_gravity.py):
* the reference field of tests/pbc_gravity_ref.py (27-image softened direct sum + the oracle's Ewald correction) on the
  periodic density-wave IC approaches the analytic g_x = (4 pi G eps / k) cos(k x) as the softening shrinks;
* the near/far split's periodic distance (sx_gravity.hip cellNearKernel): per axis min(|d|, L - |d|), then the box's
  half-size subtracted, equals the smallest box-to-point distance over the 27 images the walk visits."""
import math

import numpy as np

import pbc_gravity_ref as pr
import pyoracle as po


def test_reference_field_matches_the_analytic_wave():
    eps = 0.3
    st, _ = po.pbc_wave_state(12, eps)
    k = 2 * math.pi
    amp = 4 * math.pi * eps / k
    # a quarter of the SPH h: the softening (h_i + h_j) no longer damps the mode
    a, _ = pr.periodic_field(st.x, st.y, st.z, st.m, st.h * 0.25, 1.0)
    fit = np.sum(a[:, 0] * np.cos(k * st.x)) / np.sum(np.cos(k * st.x) ** 2)
    print("fitted amplitude", fit, "analytic", amp)
    assert abs(fit / amp - 1) < 0.03
    # the transverse components vanish up to lattice noise, the x component is the cosine
    assert np.abs(a[:, 1:]).max() < 1e-2 * amp
    assert np.abs(a[:, 0] - fit * np.cos(k * st.x)).max() < 2e-2 * amp


def test_near_test_minimum_image_equals_27_images():
    rng = np.random.default_rng(5)
    L = np.array([1.0, 1.0, 1.0])
    lo = -0.5
    for _ in range(2000):
        c = rng.uniform(lo, lo + L)
        b = rng.uniform(lo, lo + L)
        s = rng.uniform(0.0, 0.2, 3)
        # the kernel's form
        a = np.abs(b - c)
        a = np.minimum(a, np.abs(L - a))
        d = np.maximum(a - s, 0.0)
        fast = float(np.sum(d * d))
        # every image of the point c
        best = np.inf
        for ix in (-1, 0, 1):
            for iy in (-1, 0, 1):
                for iz in (-1, 0, 1):
                    e = np.maximum(np.abs(b - (c + np.array([ix, iy, iz]) * L)) - s, 0.0)
                    best = min(best, float(np.sum(e * e)))
        assert abs(fast - best) <= 1e-12 * max(1.0, best)
