"""Multi-rank VE steps on one GPU (host-staged transport, gloo control plane) against the single-domain oracle.

The SFC decomposition, particle exchange, halo discovery and the five halo exchanges per step must not change
the physics: after step 1 (identical inputs) every particle's nc and h equal the oracle's and the float fields
agree within the full-step tolerance of test_gpu_parity.py; the global time-step is identical on all ranks.
(On the Sedov lattice the h-nc iteration does not trigger, so the reference's stale-halo-h convention does not
come into play.)  RCCL itself needs one GPU per rank; it is exercised by bench.py --gpus N on a full node.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["x", "y", "z", "vx", "vy", "vz", "temp", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "xm", "kx", "prho", "c",
          "divv", "c11", "c22", "c33", "du", "ax", "ay", "az"]


def run_ranks(tmp_path, nproc, side, steps, port, ic="sedov"):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tests", "dist_worker.py"), "--out",
           str(tmp_path), "--side", str(side), "--steps", str(steps), "--ic", ic]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [dict(np.load(os.path.join(tmp_path, f"rank{q}.npz"))) for q in range(nproc)]


def merged(ranks, s):
    out = {}
    for k in ["id", "nc", "h"] + FIELDS:
        out[k] = np.concatenate([d[f"s{s}_{k}"] for d in ranks])
    o = np.argsort(out["id"])
    return {k: v[o] for k, v in out.items()}


@pytest.mark.parametrize("nproc,port", [(2, 29641), (3, 29642)])
def test_distributed_steps_match_oracle(tmp_path, nproc, port):
    side, steps = 16, 2
    ranks = run_ranks(tmp_path, nproc, side, steps, port)
    st, obox = po.sedov_state(side)
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
        assert len(dts) == 1  # identical global time-step on every rank
        assert list(dts)[0][0] == pytest.approx(ref.minDt, rel=1e-5)
        # every rank holds halos and a non-empty local range
        for d in ranks:
            first, last, n, _ = d[f"s{s}_layout"]
            assert last > first and n > last - first


def test_distributed_device_ic_conserves(tmp_path):
    """slab IC generated on the device per rank, first sync redistributes by SFC; energy conserved"""
    ranks = run_ranks(tmp_path, 2, 20, 3, 29643, ic="sedov_dev")
    got = merged(ranks, 2)
    assert got["id"].size == 20 ** 3 and np.array_equal(got["id"], np.arange(20 ** 3))
    st, _ = po.sedov_state(20)
    e0 = po.total_energy(st)
    hs = po.HostState(st.n)
    for k in ("vx", "vy", "vz", "temp"):
        hs.arrays[k][:] = got[k]
    hs.m[:] = st.m
    assert abs(po.total_energy(hs) / e0 - 1) < 1e-6
