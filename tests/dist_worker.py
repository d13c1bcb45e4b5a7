"""Worker for the multi-rank tests (launched by torch.distributed.run with the gloo control plane).

  python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 --master-port X \
      tests/dist_worker.py --out DIR [--backend host|rccl] [--side S] [--steps K] [--ic sedov|sedov_dev]

Each rank owns an index slice of the IC, runs K distributed VE steps, and writes its local particles
(id, nc, h and the compared float fields) plus scalars to DIR/rank<r>.npz.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sph-exa_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

FIELDS = ["x", "y", "z", "vx", "vy", "vz", "temp", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "xm", "kx", "prho", "c",
          "divv", "c11", "c22", "c33", "du", "ax", "ay", "az"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", default="host")
    ap.add_argument("--side", type=int, default=16)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--ic", default="sedov",
                    help="sedov | sedov_dev | noh | evrard (self-gravity, G = 1) | pbc_wave (periodic self-gravity, G = 1)")
    ap.add_argument("--std", action="store_true", help="std propagator (HydroProp)")
    ap.add_argument("--no-overlap", action="store_true", help="serial halo exchanges (no interior/boundary split)")
    ap.add_argument("--av-clean", action="store_true", help="avClean momentum (dV halos)")
    ap.add_argument("--g", type=float, default=None, help="gravitational constant (default: 1 for evrard, else 0)")
    ap.add_argument("--bdt", action="store_true", help="ve-bdt propagator: one block time-step substep per step")
    args = ap.parse_args()

    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, size = dist.get_rank(), dist.get_world_size()
    import pyoracle as po
    import sphexa_amd as sx

    local = int(os.environ.get("LOCAL_RANK", "0"))
    ctx = sx.Context(0 if args.backend == "host" else local)
    comm = sx.Comm(args.backend)
    ic = {"evrard": po.evrard_state, "noh": po.noh_state, "pbc_wave": po.pbc_wave_state}.get(args.ic, po.sedov_state)
    st, obox = ic(args.side)
    if args.ic in ("evrard", "noh"):
        po.converge_h(po.load_oracle(), st, obox)  # these ICs' h would iterate (and may not converge) in the first search
    box = sx.make_box(list(obox.lim), list(obox.bnd))
    g = args.g if args.g is not None else (1.0 if args.ic in ("evrard", "pbc_wave") else 0.0)
    params = sx.default_params(g=g, std=args.std, av_clean=args.av_clean,
                               bdt=args.bdt)
    sim = sx.Sim(ctx, 2 * st.n // size + 4096, box, params=params)
    sim.set_comm(comm)
    sim.set_overlap(not args.no_overlap)
    if args.ic == "sedov_dev":
        sim.init_sedov(args.side, rank, size)
    else:
        f, l = st.n * rank // size, st.n * (rank + 1) // size
        sim.set_state({k: v[f:l] for k, v in st.arrays.items()}, st.minDt, st.minDt_m1)
    out = {}
    for s in range(args.steps):
        sim.step()
        got = sim.get(["id", "nc", "h", "m"] + FIELDS + (["rho", "p"] if args.std else []) +
                      (["rung"] if args.bdt else []))
        for k, v in got.items():
            out[f"s{s}_{k}"] = v
        sc = sim.scalars()
        out[f"s{s}_scalars"] = np.array([sc["minDt"], sc["minDt_m1"], sc["ttot"]])
        cq = sim.conserved()
        out[f"s{s}_conserved"] = np.array([cq[k] for k in ("ecin", "eint", "egrav", "etot", "totalNeighbors")])
        gs = sim.gravity_stats()
        out[f"s{s}_gravity"] = np.array([gs["halos"], gs["far_cells"], gs["remote_cells"]])
        if args.bdt:
            ts = sim.timestep()
            out[f"s{s}_ts"] = np.array([ts["numRungs"], ts["substep"], ts["nextDt"]])
        lay = sim.layout()
        out[f"s{s}_layout"] = np.array([lay["first"], lay["last"], lay["n"], lay["haloRetries"]])
        ov = sim.overlap_stats()
        out[f"s{s}_overlap"] = np.array([ov["interior"], ov["boundary"]])
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), **out)
    sim.close()
    comm.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
