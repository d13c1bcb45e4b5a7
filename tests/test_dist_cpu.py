"""The multi-rank path on the CPU (no GPU): world_size 2 and 3 over gloo.

* the host-side decisions of the decomposition that the GPU path calls (sx_domain_splitters,
  sx_domain_halo_layout in libsphexa_hip.so) against a numpy restatement;
* the decomposed VE step with 2, 3 and 8 ranks (8 = one node's GPUs, seven peers per rank; oracle/dist_oracle.py: SFC assignment from the all-reduced key histogram through
  sx_domain_splitters, particle exchange, halo discovery, the five halo exchanges, global dt) against the
  single-domain oracle: after step 1 nc and h exact, floats within the full-step tolerance of
  tests/test_gpu_parity.py (neighbor sums run in another order), identical dt on every rank.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as po
import sphexa_amd as sx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["x", "y", "z", "vx", "vy", "vz", "temp", "du", "ax", "ay", "az", "alpha", "xm", "kx", "prho", "c", "divv"]


def test_splitters_equal_counts():
    rng = np.random.default_rng(3)
    bits = 12
    for P in (1, 2, 3, 8):
        hist = rng.integers(0, 50, 1 << bits).astype(np.uint32)
        split = sx.domain_splitters(hist, bits, P)
        assert split[0] == 0 and split[P] == 1 << 63 and np.all(np.diff(split.astype(np.float64)) >= 0)
        # restatement: rank q starts at the first bin b with cumsum(hist[:b]) >= q*total/P
        cum = np.concatenate([[0], np.cumsum(hist.astype(np.int64))])
        total = int(cum[-1])
        for q in range(1, P):
            b = int(np.argmax(cum >= (total * q) // P))
            assert split[q] == np.uint64(b) << np.uint64(63 - bits)
        owned = [int(cum[int(split[q + 1] >> np.uint64(63 - bits)) if q + 1 < P else -1] -
                     cum[int(split[q] >> np.uint64(63 - bits))]) for q in range(P)]
        assert sum(owned) == total and max(owned) - min(owned) <= 2 * int(hist.max())


def test_halo_layout():
    off, (first, last, total) = sx.halo_layout([3, 0, 5, 2], 1, 10)
    assert (first, last, total) == (3, 13, 20)
    assert list(off) == [0, 0, 13, 18]
    off, lay = sx.halo_layout([0], 0, 7)
    assert lay == (0, 7, 7)
    with pytest.raises(sx.SxError):
        sx.halo_layout([1, 2], 2, 5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(tmp_path, nproc, side, steps, ic="sedov", extra=()):
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_cpu_worker.py"), "--rank", str(r),
                               "--size", str(nproc), "--port", str(port), "--out", str(tmp_path), "--ic", ic,
                               "--side", str(side), "--steps", str(steps), *extra], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(nproc)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
    return [dict(np.load(os.path.join(tmp_path, f"rank{q}.npz"))) for q in range(nproc)]


def merged(ranks, s):
    out = {k: np.concatenate([d[f"s{s}_{k}"] for d in ranks]) for k in ["id", "nc", "h"] + FIELDS}
    o = np.argsort(out["id"])
    return {k: v[o] for k, v in out.items()}


@pytest.mark.parametrize("nproc,ic,side", [(2, "sedov", 16), (3, "sedov", 14), (2, "noh", 18), (8, "sedov", 24),
                                           (8, "noh", 26)])
def test_decomposed_steps_match_single_domain(tmp_path, nproc, ic, side):
    steps = 2
    ranks = run_ranks(tmp_path, nproc, side, steps, ic)
    st, obox = po.sedov_state(side) if ic == "sedov" else po.noh_state(side)
    ora = po.load_oracle()
    ref = st.copy()
    for s in range(steps):
        ora.step(ref, obox)
        got = merged(ranks, s)
        assert got["id"].size == st.n and np.array_equal(got["id"], np.arange(st.n))
        o = np.argsort(ref.id)
        if s == 0:
            assert np.array_equal(got["nc"], ref.nc[o])
            assert np.array_equal(got["h"], ref.h[o])
        for k in FIELDS:
            a = got[k].astype(np.float64)
            b = ref.arrays[k][o].astype(np.float64)
            tol = 1e-4 * np.abs(b) + 1e-5 * np.max(np.abs(b))
            assert np.all(np.abs(a - b) <= tol), (s, k, np.max(np.abs(a - b) / (np.abs(b) + 1e-300)))
        dts = {tuple(d[f"s{s}_scalars"]) for d in ranks}
        assert len(dts) == 1
        assert list(dts)[0][0] == pytest.approx(ref.minDt, rel=1e-6)
        # equal-count SFC shares, every rank holding halos
        sizes = [int(d[f"s{s}_layout"][1] - d[f"s{s}_layout"][0]) for d in ranks]
        assert max(sizes) - min(sizes) <= 0.1 * st.n / nproc + 64
        for d in ranks:
            first, last, total, _ = d[f"s{s}_layout"]
            assert last > first and total > last - first


@pytest.mark.parametrize("nproc", [2, 3])
def test_decomposed_gravity_matches_direct_sum(tmp_path, nproc):
    """the multi-rank gravity decomposition of sx_sim.cpp (level-6 cell multipoles all-gathered, far cells as
    multipoles, near cells fetched as gravity halos and traversed with the locals), restated on the CPU in
    oracle/dist_oracle.py over gloo, against a softened direct sum: within the Barnes-Hut error of theta = 0.5"""
    from test_gpu_distributed import direct_gravity

    side = 16
    ranks = run_ranks(tmp_path, nproc, side, 1, "evrard", ("--gravity",))
    st, _ = po.evrard_state(side)
    ids = np.concatenate([d["id"] for d in ranks]).astype(np.int64)
    acc = np.concatenate([d["acc"] for d in ranks])
    assert np.array_equal(np.sort(ids), np.arange(st.n))
    ad = direct_gravity(st.x, st.y, st.z, st.m.astype(np.float64), st.h)[ids]
    err = np.linalg.norm(acc - ad, axis=1) / np.linalg.norm(ad, axis=1)
    assert np.median(err) < 1e-3 and np.max(err) < 1e-2, (np.median(err), np.max(err))
    for d in ranks:
        halos, far_cells, remote_cells = d["stats"]
        assert 0 < far_cells < remote_cells and halos > 0, d["stats"]


@pytest.mark.parametrize("ic,side", [("sedov", 40), ("noh", 44)])
def test_overlapped_exchanges_classification(tmp_path, ic, side):
    """the interior/boundary cluster classification of the overlapped halo exchanges (sx_sim.cpp
    classifyClustersKernel, exchange on a comm stream while interior clusters compute): restated on the CPU over gloo
    (oracle/dist_oracle.py, overlap=True) with the halo copies of every exchanged field poisoned with NaN while the
    interior clusters run.  Two ranks, two steps: bitwise equal to the serial exchanges, both classes non-empty."""
    a = run_ranks(tmp_path / "serial", 2, side, 2, ic) if (tmp_path / "serial").mkdir() is None else None
    b = run_ranks(tmp_path / "ovl", 2, side, 2, ic, ("--overlap",)) if (tmp_path / "ovl").mkdir() is None else None
    for s in range(2):
        for q in range(2):
            inner, bound = b[q][f"s{s}_clusters"]
            assert inner > 0 and bound > 0, (s, q, inner, bound)
            for k in ["id", "nc", "h"] + FIELDS:
                x, y = a[q][f"s{s}_{k}"], b[q][f"s{s}_{k}"]
                assert np.array_equal(x, y), (s, q, k)
                assert not np.any(np.isnan(y.astype(np.float64)))
            assert np.array_equal(a[q][f"s{s}_scalars"], b[q][f"s{s}_scalars"])


def test_decomposed_gravity_matches_reference_two_ranks(tmp_path):
    """the same restatement on the IC of tests/golden/evrard20_grav_mpi.npz against the reference's own 2-rank
    gravity (Domain::syncGrav + computeGlobalMultipoles + computeGravity under MPICH, oracle/gen_grav_mpi.py): two
    Barnes-Hut trees of theta = 0.5, within the opening-angle error; the reference's 2-rank result equals its
    1-rank result bit for bit (its focus tree is independent of the decomposition; egrav to the order of its sum)"""
    import golden_util as gu

    fx = gu.load("evrard20_grav_mpi.npz")
    assert np.array_equal(fx["acc_p1"], fx["acc_p2"]) and abs(fx["egrav_p1"][0] / fx["egrav_p2"][0] - 1) < 1e-14
    ranks = run_ranks(tmp_path, 2, 20, 1, "evrard", ("--gravity", "--converge-h"))
    ids = np.concatenate([d["id"] for d in ranks]).astype(np.int64)
    acc = np.concatenate([d["acc"] for d in ranks])
    a_ref = fx["acc_p2"].astype(np.float64)[ids]
    err = np.linalg.norm(acc - a_ref, axis=1) / np.linalg.norm(a_ref, axis=1)
    assert np.median(err) < 1e-3 and np.max(err) < 1e-2, (np.median(err), np.max(err))
    eg = sum(float(d["egrav"][0]) for d in ranks)  # each rank's share of 0.5 sum G m phi
    assert abs(eg / fx["egrav_p2"][0] - 1) < 1e-3, (eg, fx["egrav_p2"][0])


@pytest.mark.parametrize("nproc,side,speed", [(2, 14, 0.04), (3, 14, 0.04), (3, 14, 0.12)])
def test_skin_premise_several_ranks(tmp_path, nproc, side, speed):
    """the argument behind multi-rank skin lists (sx_sim.cpp skinHaloRefresh; dist_oracle.skin_premise), on gloo
    ranks: halos requested with the skin radius hold every particle of every local's skin sphere, and with the
    displacement grid reduced over all ranks every cluster the filter's drift bound admits has all its current
    neighbours in its build-time skin lists -- also the particles of other ranks that were no halo at the build.
    With a rank-local grid the bound admits clusters whose new neighbours slid in from another rank (the fast case:
    the all-reduce is needed, not only sufficient)"""
    ranks = run_ranks(tmp_path, nproc, side, 6, extra=("--skin-premise", "0.08", "--premise-speed", str(speed)))
    adm = sum(int(r["global_admitted"].sum()) for r in ranks)
    loc_vio = sum(int(r["local_violations"].sum()) for r in ranks)
    print("admitted clusters (global grid)", [r["global_admitted"].tolist() for r in ranks],
          "violations with a rank-local grid", [r["local_violations"].tolist() for r in ranks])
    for r in ranks:
        assert int(r["global_mismatch"][0]) == 0
        assert int(r["global_violations"].sum()) == 0
        assert int(r["halos"][0]) > 0
    assert adm > 0
    if speed > 0.1:
        assert loc_vio > 0
