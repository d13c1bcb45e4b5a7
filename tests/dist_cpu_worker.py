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
    ap.add_argument("--skin-premise", type=float, default=0.0,
                    help="skin factor s: check the multi-rank skin argument (dist_oracle.skin_premise) over --steps "
                         "displacement steps of a sliding + sheared lattice instead of running VE steps")
    ap.add_argument("--premise-speed", type=float, default=0.04, help="slide per step in lattice spacings")
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
    if args.skin_premise > 0:
        s = args.skin_premise
        full = d._discover(d._exchange_particles(d._sort(d.local)), do.HALO_MARGIN * (1.0 + s))
        pos0 = np.stack([st.x, st.y, st.z], axis=1).astype(np.float64)  # rows by id (the IC's ids are 0 .. n-1)
        # a slab x > 0 sliding towards -x through the rest of the lattice (relative motion across rank boundaries),
        # plus a shear: --premise-speed lattice spacings per step
        V = args.premise_speed / args.side
        disps, pos = [], pos0.copy()
        for _ in range(args.steps):
            dsp = np.zeros_like(pos)
            dsp[:, 0] = -V * (pos[:, 0] > 0) + 0.3 * V * np.sin(2 * np.pi * pos[:, 1])
            dsp[:, 1] = 0.2 * V * np.cos(2 * np.pi * pos[:, 2])
            disps.append(dsp)
            pos = pos + dsp
            pos = -0.5 + np.mod(pos + 0.5, 1.0)
        for tag, glob in (("global", True), ("local", False)):
            mm, adm, vio = do.skin_premise(d, full, pos0, st.h.astype(np.float64), s, disps, global_grid=glob)
            out[f"{tag}_mismatch"] = np.array([mm])
            out[f"{tag}_admitted"] = np.array(adm)
            out[f"{tag}_violations"] = np.array(vio)
        out["halos"] = np.array([d.total - (d.last - d.first)])
        np.savez(os.path.join(args.out, f"rank{args.rank}.npz"), **out)
        dist.barrier()
        dist.destroy_process_group()
        return
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
