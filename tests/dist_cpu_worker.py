"""Worker of the CPU multi-rank tests (tests/test_dist_cpu.py): gloo process group on 127.0.0.1, one rank of the
decomposed oracle (oracle/dist_oracle.py) over an index slab of a lattice IC, K steps, locals written to
DIR/rank<r>.npz.

  python tests/dist_cpu_worker.py --rank R --size P --port X --out DIR [--ic sedov|noh] [--side S] [--steps K]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sph-exa_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--ic", default="sedov")
    ap.add_argument("--side", type=int, default=16)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gravity", action="store_true", help="only the multi-rank gravity of the IC (G = 1)")
    ap.add_argument("--overlap", action="store_true", help="interior clusters before each halo exchange")
    ap.add_argument("--converge-h", action="store_true", help="h after the first search's h iteration (pyoracle)")
    args = ap.parse_args()
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{args.port}", rank=args.rank,
                            world_size=args.size)
    import dist_oracle as do
    import pyoracle as po

    ic = {"sedov": po.sedov_state, "noh": po.noh_state, "evrard": po.evrard_state}[args.ic]
    st, box = ic(args.side)
    if args.converge_h:
        po.converge_h(po.load_oracle(), st, box)
    f, l = st.n * args.rank // args.size, st.n * (args.rank + 1) // args.size
    local = po.HostState(l - f)
    for k in po.CONSERVED:
        local.arrays[k][:] = st.arrays[k][f:l]
    local.minDt, local.minDt_m1 = st.minDt, st.minDt_m1
    d = do.DistOracle(po.load_oracle(), box, local, overlap=args.overlap)
    out = {}
    if args.gravity:
        full = d._discover(d._exchange_particles(d._sort(d.local)), do.HALO_MARGIN)
        acc, eg, stats = do.distributed_gravity(d, full, 1.0, 0.5)
        np.savez(os.path.join(args.out, f"rank{args.rank}.npz"), id=full.id[d.first:d.last], acc=acc,
                 egrav=np.array([eg]), stats=np.array([stats["halos"], stats["far_cells"], stats["remote_cells"]]))
        dist.barrier()
        dist.destroy_process_group()
        return
    for s in range(args.steps):
        loc = d.step()
        for k in ("id", "nc", "h", "x", "y", "z", "vx", "vy", "vz", "temp", "du", "ax", "ay", "az", "alpha",
                  "xm", "kx", "prho", "c", "divv"):
            out[f"s{s}_{k}"] = loc.arrays[k].copy()
        out[f"s{s}_scalars"] = np.array([loc.minDt, loc.minDt_m1, loc.ttot])
        out[f"s{s}_layout"] = np.array([d.first, d.last, d.total, d.halo_retries])
        out[f"s{s}_split"] = d.split.astype(np.uint64)
        out[f"s{s}_clusters"] = np.array(d.cluster_counts)
    np.savez(os.path.join(args.out, f"rank{args.rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
