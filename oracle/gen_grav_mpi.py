"""Fixture: the reference's multi-rank self-gravity (TEST INFRASTRUCTURE ONLY).

Runs oracle/_ref/grav_mpi_ref (Domain::syncGrav + computeGlobalMultipoles + computeGravity of the reference, built by
oracle/Makefile) under the image's MPICH with 1 and 2 ranks on the Evrard substitute that
tests/test_gpu_distributed.py::test_distributed_gravity_matches_direct_sum decomposes (pyoracle.evrard_state(20),
h after the first search's h iteration, G = 1, theta = 0.5, global bucket 64 = max(64, N / (100 P)) as
sphexa.cpp:134-135), each rank taking an index slab of the IC, and stores the gravitational accelerations by particle
id and the total potential energy:
    tests/golden/evrard20_grav_mpi.npz: id, acc_p1 (n x 3), acc_p2 (n x 3), egrav_p1, egrav_p2, plus the IC
Run where /root/reference exists:  make -C oracle && python oracle/gen_grav_mpi.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "evrard20_grav_mpi.npz")
EXE = os.path.join(HERE, "_ref", "grav_mpi_ref")
MPIEXEC = "/opt/conda/bin/mpiexec"


def write_input(path, st, box):
    rec = np.zeros(st.n, dtype=[("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("h", "<f4"), ("m", "<f4"), ("id", "<u8")])
    for k in ("x", "y", "z", "h", "m", "id"):
        rec[k] = st.arrays[k]
    with open(path, "wb") as f:
        f.write(np.uint64(st.n).tobytes())
        f.write(np.array(list(box.lim), np.float64).tobytes())
        f.write(np.array(list(box.bnd), np.int32).tobytes())
        f.write(rec.tobytes())


def run(nranks, inp, tmp, theta=0.5, G=1.0, bucket=64):
    prefix = os.path.join(tmp, f"p{nranks}_")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    subprocess.run([MPIEXEC, "-n", str(nranks), EXE, inp, prefix, str(bucket), str(theta), str(G)], check=True,
                   env=env, timeout=600)
    ids, acc, eg = [], [], None
    for r in range(nranks):
        with open(f"{prefix}{r}.bin", "rb") as f:
            n = int(np.frombuffer(f.read(8), np.uint64)[0])
            eg = float(np.frombuffer(f.read(8), np.float64)[0])
            rec = np.frombuffer(f.read(), dtype=[("id", "<u8"), ("a", "<f4", 3)], count=n)
        ids.append(rec["id"].copy())
        acc.append(rec["a"].copy())
    ids, acc = np.concatenate(ids), np.concatenate(acc)
    o = np.argsort(ids)
    return ids[o], acc[o], eg


def main():
    if not os.path.exists(EXE):
        raise SystemExit("oracle/_ref/grav_mpi_ref missing: make -C oracle where /root/reference exists")
    st, box = po.evrard_state(20)
    po.converge_h(po.load_oracle(), st, box)
    with tempfile.TemporaryDirectory() as tmp:
        inp = os.path.join(tmp, "in.bin")
        write_input(inp, st, box)
        out = {"x": st.x.copy(), "y": st.y.copy(), "z": st.z.copy(), "h": st.h.copy(), "m": st.m.copy(),
               "box": np.array(list(box.lim) + list(box.bnd), np.float64)}
        for p in (1, 2):
            ids, acc, eg = run(p, inp, tmp)
            assert np.array_equal(ids, np.arange(st.n)), "every particle exactly once"
            out[f"acc_p{p}"] = acc
            out[f"egrav_p{p}"] = np.array([eg])
            print(f"P={p}: egrav {eg:.10g}")
        out["id"] = np.arange(st.n, dtype=np.uint64)
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
