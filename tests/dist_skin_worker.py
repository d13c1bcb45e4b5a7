"""Worker of the multi-rank skin-list test (tests/test_gpu_distributed_skin.py), launched by torch.distributed.run.

  python -m torch.distributed.run --nproc-per-node P ... tests/dist_skin_worker.py --out DIR --ic sedov|noh
      [--side S] [--steps K] [--skin 0.08] [--max-reuse 24]

Every rank runs two simulations over the host-staged transport: `a` with skin lists (filter-served steps between
full builds), `b` with the skin off (a fresh distributed sync + search every step).  Before each step b is handed a's
state of this rank, so both step from the same global state; the rank writes, per step, ids / nc / h and the compared
fields of both, and a's skin statistics, to DIR/rank<r>.npz.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sph-exa_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

STATE = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]
FIELDS = ["id", "nc", "h", "ax", "ay", "az", "du", "x", "vx"]
SKIN = ["builds", "reuse_steps", "stale_clusters", "exact_clusters", "plain_steps", "resyncs"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--ic", default="sedov")
    ap.add_argument("--side", type=int, default=20)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--skin", type=float, default=0.08)
    ap.add_argument("--max-reuse", type=int, default=24)
    ap.add_argument("--g", type=float, default=0.0, help="gravitational constant (self-gravity; evrard: 1)")
    ap.add_argument("--std", action="store_true", help="std propagator (HydroProp)")
    ap.add_argument("--av-clean", action="store_true", help="HydroVeProp<avClean=true>")
    args = ap.parse_args()

    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, size = dist.get_rank(), dist.get_world_size()
    import pyoracle as po
    import sphexa_amd as sx

    ctx = sx.Context(0)
    comm = sx.Comm("host")
    st, obox = {"noh": po.noh_state, "evrard": po.evrard_state}.get(args.ic, po.sedov_state)(args.side)
    if args.ic in ("evrard", "noh"):
        po.converge_h(po.load_oracle(), st, obox)  # the IC's h would iterate in the first search
    box = sx.make_box(list(obox.lim), list(obox.bnd))
    cap = 2 * st.n // size + 4096
    prm = sx.default_params(g=args.g, std=args.std, av_clean=args.av_clean)
    a, b = sx.Sim(ctx, cap, box, params=prm), sx.Sim(ctx, cap, box, params=prm)
    for sim, f in ((a, args.skin), (b, 0.0)):
        sim.set_comm(comm)
        sim.set_skin(f, args.max_reuse if f > 0 else 1)
    f0, l0 = st.n * rank // size, st.n * (rank + 1) // size
    a.set_state({k: v[f0:l0] for k, v in st.arrays.items()}, st.minDt, st.minDt_m1)
    out = {}
    for s in range(args.steps):
        g = a.get(STATE)
        sc = a.scalars()
        b.set_state(g, sc["minDt"], sc["minDt_m1"])
        a.step()
        b.step()
        fields = FIELDS + (["rho"] if args.std else ["xm", "kx", "divv", "alpha"])
        for tag, sim in (("a", a), ("b", b)):
            for k, v in sim.get(fields).items():
                out[f"s{s}_{tag}_{k}"] = v
            out[f"s{s}_{tag}_dt"] = np.array([sim.scalars()["minDt"]])
            out[f"s{s}_{tag}_egrav"] = np.array([sim.conserved()["egrav"]])
        ks = a.skin_stats()
        out[f"s{s}_skin"] = np.array([ks[k] for k in SKIN] + [ks["factor"], ks["next_factor"], ks["kept_clusters"],
                                                             ks["frozen_clusters"]], np.float64)
        out[f"s{s}_layout"] = np.array(list(a.layout().values()), np.int64)
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), **out)
    a.close()
    b.close()
    comm.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
