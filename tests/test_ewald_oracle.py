"""The Ewald periodic-gravity correction's checker (oracle/ewald.py) pinned to the reference (CPU, no GPU):
* against the committed golden vectors tests/golden/ewald_ref.npz (oracle/gen_ewald.py: ryoanji::computeGravityEwald,
  ewald.hpp:380-413, compiled from /root/reference by oracle/Makefile) -- accelerations bit-exact, energy to 1e-13
  (the reference sums it in an OpenMP reduction);
* where oracle/_ref was built here: the same on other seeds and settings, the reference run live.
The GPU's sx_gravity_ewald is checked against this restatement in tests/test_gpu_gravity.py."""
import os
import sys

import numpy as np
import pytest

import golden_util as gu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import ewald as ew  # noqa: E402
import gen_ewald as ge  # noqa: E402

REF_SO = os.path.join(os.path.dirname(ge.__file__), "_ref", "libewald_ref.so")


def _restated(x, y, z, m, M, c, lo, hi, G, s):
    ax = np.zeros(len(x), np.float32)
    ay, az = ax.copy(), ax.copy()
    e = ew.gravity_ewald(x, y, z, m, M, c, hi - lo, G, ax, ay, az, **s)
    return e, ax, ay, az


@pytest.mark.parametrize("case", list(ge.CASES))
def test_ewald_restatement_matches_golden(case):
    d = gu.load("ewald_ref.npz")
    lo, hi = d["box"]
    e, ax, ay, az = _restated(d["x"], d["y"], d["z"], d["m"], d["M"], d["center"], lo, hi, float(d["G"][0]),
                              ge.CASES[case])
    ref = d[f"{case}_acc"]
    assert np.array_equal(np.stack([ax, ay, az]), ref), np.abs(np.stack([ax, ay, az]) - ref).max()
    assert abs(e / float(d[f"{case}_egrav"][0]) - 1) < 1e-13


def test_ewald_params_table():
    """ewaldInitParameters: the k-space table holds every h with 0 < |h|^2 <= hCut^2 (hCut 2.8: 80 vectors), and the
    real-space shells are max(ceil(lCut), numReplicaShells)"""
    M = np.array([1, 0.1, 0.02, -0.03, -0.05, 0.01, -0.05, 0.3], np.float32)
    p = ew.ewald_params(M, [0, 0, 0], 1.0)
    n = sum(1 for hx in range(-3, 4) for hy in range(-3, 4) for hz in range(-3, 4)
            if 0 < hx * hx + hy * hy + hz * hz <= 2.8 * 2.8)
    assert p["hs"].shape == (n, 3) and p["numEwaldShells"] == 3
    assert ew.ewald_params(M, [0, 0, 0], 1.0, numReplicaShells=4)["numEwaldShells"] == 4
    off = ew.ewald_params(M, [0, 0, 0], 1.0, lCut=0, hCut=0, alpha_scale=0)
    assert off["numEwaldShells"] == 0 and off["numReplicaShells"] == 0


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference here)")
@pytest.mark.parametrize("seed,L,s", [(11, 1.0, dict(numReplicaShells=1)), (12, 2.5, dict(numReplicaShells=0)),
                                      (13, 1.0, dict(numReplicaShells=1, lCut=3.2, hCut=3.0, alpha_scale=2.4))])
def test_ewald_restatement_matches_reference_live(seed, L, s):
    lo, hi = -0.3 * L, 0.7 * L
    x, y, z, m = ge.cube(n=300, seed=seed, lo=lo, hi=hi)
    M, c = ge.root_moments(x, y, z, m)
    e, ax, ay, az = ge.run_ref(ge.ref_lib(), x, y, z, m, M, c, lo, hi, 0.7, s)
    e2, bx, by, bz = _restated(x, y, z, m, M, c, lo, hi, 0.7, s)
    assert np.array_equal(np.stack([ax, ay, az]), np.stack([bx, by, bz]))
    assert abs(e / e2 - 1) < 1e-13
