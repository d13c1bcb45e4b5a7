"""Benchmark: particle-updates/s of the VE time step (Sedov lattice) on N MI355X, one process per GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--side S] [--no-cpu-baseline]

A step is one full HydroVeProp step (ve_hydro.hpp:132-218): sync (keys, sort, reorder, tree), neighbor search with
h iteration, XMass, VeDefGradh, EOS, IAD+divv/curlv, AV switches, momentum/energy, [self-gravity], time-step,
positions, h update.  --init noh|evrard run BASELINE configs 3 and 5 (lattice substitutes for the glass block).
Inputs are generated and kept in HBM; nothing leaves the device inside the timed region except the per-step
4-byte tree-level counts and stats.  Weak scaling: side = round(200 * N^(1/3)) particles^(1/3) in total
(N=1: Sedov -n 200 = BASELINE config 2; N=8: Sedov -n 400 = config 4).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sph-exa_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector (packed) peak
MOM_OWN_BYTES = 108    # momentum kernel own record R+W
MOM_EDGE_BYTES = 4 + 88  # index + neighbor record per edge
MOM_FLOP_PER_PAIR = 150  # SURVEY.md 8(d) secondary VALU figure
# compulsory HBM bytes of one momentum launch per target, as implemented: own packed records 96 B,
# nc 4 B, outputs 20 B, u16 neighbor positions 2 B/neighbor, union index 4 B per union entry
MOM_COMPULSORY_OWN = 96 + 4 + 20
# std propagator momentum (hydro_std/momentum_energy_kern.hpp): own x,y,z,v,h,m,rho,p,c,c_ij + nc read, a,du written;
# per edge the index + x,y,z (24) v (12) h m rho p c (20) c_ij (24)
MOM_STD_OWN_BYTES = 24 + 12 + 20 + 24 + 4 + 12 + 8
MOM_STD_EDGE_BYTES = 4 + 80
# kernel-time slots of sx_sim in std mode (sx_sim.cpp: density in "xmass", IAD in "iadDivvCurlv")
STD_KERNEL_NAMES = {"findNeighbors": "findNeighbors", "xmass": "density", "iadDivvCurlv": "iad",
                    "momentumEnergy": "momentumEnergySTD", "gravity": "gravity"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_traffic(kernel_prefix, particles):
    """HBM bytes per launch of a kernel from the committed rocprofv3 --pmc summary of the same workload
    (scripts/gpu_pmc.sh + scripts/pmc_summary.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, KB units), or None
    when the summary was taken on another particle count."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("_meta", {}).get("particles_per_gpu") != particles:
        return None
    for k, v in d.items():
        if k == "_meta":
            continue
        if kernel_prefix in k and "hbm_read_bytes_est" in v and "hbm_write_bytes_est" in v:
            return v["hbm_read_bytes_est"] + v["hbm_write_bytes_est"]
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--side", type=int, default=0, help="total lattice side (default weak scaling from 200)")
    ap.add_argument("--bucket", type=int, default=64)
    ap.add_argument("--exact", action="store_true", help="use the no-FMA (bit-reproducible) kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="rccl", help="rccl (one GPU per rank) or host (staged, tests)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--init", default="sedov", choices=["sedov", "noh", "evrard"],
                    help="sedov (BASELINE metric, device IC), noh (config 3), evrard (config 5: VE + self-gravity)")
    ap.add_argument("--av-clean", action="store_true", help="HydroVeProp<avClean=true>")
    ap.add_argument("--prop", default="ve", choices=["ve", "std"],
                    help="ve (HydroVeProp, the BASELINE metric) or std (HydroProp, std_hydro.hpp)")
    return ap.parse_args()


def cpu_baseline(seconds):
    """Reference CPU path (oracle/_ref, OpenMP) timed on this host on a bounded Sedov sample."""
    import pyoracle as po

    kind = "reference"
    path = os.path.join(ROOT, "oracle", "_ref", "libsphexa_ref_fast.so")
    if not os.path.exists(path):
        path = os.path.join(ROOT, "oracle", "_ref", "libsphexa_ref.so")
    if not os.path.exists(path):
        path, kind = po.ORACLE_SO, "port"
    lib = po.Lib(path)
    side = 50
    st, box = po.sedov_state(side)
    lib.step(st, box)  # warm-up (first touch, thread pool)
    steps, t0 = 0, time.perf_counter()
    while True:
        lib.step(st, box)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 50:
            break
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return {"value": st.n * steps / el, "unit": "particle-updates/s", "cores": cores, "kind": kind,
            "sample": f"Sedov lattice -n {side} ({st.n} particles), {steps} VE steps after 1 warm-up, "
                      f"{os.path.basename(path)}, OMP threads={cores}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(args.gpus, world)
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only (gloo): rendezvous, barrier, max-reduce of timings

        dist.init_process_group("gloo")

    import numpy as np

    import sphexa_amd as sx

    default_side = {"sedov": 200, "noh": 300, "evrard": 300}[args.init]
    side = args.side or int(round(default_side * n_gpus ** (1.0 / 3.0)))
    n_total = side ** 3
    ic_arrays = None
    if args.init != "sedov":
        from sphexa_amd import ic

        ic_arrays, lim, bnd, dt0 = getattr(ic, args.init)(side)
        n_total = ic_arrays["x"].size
    device = 0
    if args.backend != "host":
        import torch  # device_count() does not initialise the GPU runtime

        device = local % max(1, torch.cuda.device_count())
    ctx = sx.Context(device, exact=args.exact)
    if ic_arrays is None:
        box = sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1])
    else:
        box = sx.make_box(lim, bnd)
    # capacity: the rank's share plus halos (surface layer of the SFC domain) with headroom
    cap = n_total if world == 1 else int(1.6 * n_total / world) + 65536
    params = sx.default_params(av_clean=args.av_clean, g=1.0 if args.init == "evrard" else 0.0,
                               std=args.prop == "std")
    sim = sx.Sim(ctx, cap, box, params=params, bucket=args.bucket)
    comm = None
    transport = args.backend
    if world > 1:
        try:
            comm = sx.Comm(args.backend)
            ok = 1
        except sx.SxError as e:  # e.g. RCCL refusing the node's topology: keep the run alive on the staged path
            print(f"rank {rank}: {e}; falling back to the host-staged transport", file=sys.stderr)
            ok = 0
        import torch

        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)  # every rank must use the same transport
        if int(flag.item()) == 0:
            if comm is not None:
                comm.close()
            comm = sx.Comm("host")
            transport = f"host (fallback: {args.backend} communicator creation failed)"
        sim.set_comm(comm)
    if ic_arrays is None:
        sim.init_sedov(side, rank, world)
    else:
        f, l = n_total * rank // world, n_total * (rank + 1) // world  # index slab; the first sync redistributes
        sim.set_state({k: v[f:l] for k, v in ic_arrays.items()}, dt0, dt0)
    for _ in range(args.warmup):
        sim.step()

    def barrier():
        if dist is not None:
            dist.barrier()

    ctx.sync()
    barrier()
    stage_sum, kern_sum = {}, {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.step()
        for k, v in sim.stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        for k, v in sim.kernel_times().items():
            kern_sum[k] = kern_sum.get(k, 0.0) + v
    ctx.sync()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    stats = sim.stats()
    n_local = sim.size()
    ms_step = el / args.steps * 1e3
    ng = stats["sumNeighbors"] / max(1, n_local)
    mom_ms = kern_sum.get("momentumEnergy", float("nan")) / args.steps
    std_prop = args.prop == "std"
    own_b, edge_b = (MOM_STD_OWN_BYTES, MOM_STD_EDGE_BYTES) if std_prop else (MOM_OWN_BYTES, MOM_EDGE_BYTES)
    mom_kernel = "momentumStdKernel" if std_prop else "momentumEnergyKernel"
    mom_bytes = n_local * (own_b + ng * edge_b)
    achieved = mom_bytes / (mom_ms * 1e-3) / 1e9
    union_pp = stats["sumUnion"] / max(1, n_local)
    comp_bytes = n_local * (MOM_COMPULSORY_OWN + 2 * ng + 4 * union_pp)
    mom_tflops = n_local * ng * MOM_FLOP_PER_PAIR / (mom_ms * 1e-3) / 1e12
    sc = sim.scalars()
    out = {
        "metric": "particle-updates/sec (whole node), Sedov -n 400, 1/2/4/8 MI355X + HBM roofline %",
        "value": n_total * args.steps / el,
        "unit": "particle-updates/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 hydro / f64 coordinates (sph::SphTypes)",
        "data": "synthetic Sedov lattice generated on device (sedov_init.hpp), no checkpoint" if ic_arrays is None
                else f"synthetic {args.init} lattice substitute for the glass block (SURVEY F6), sphexa_amd/ic.py",
        "config": {"workload": f"{args.init.capitalize()} -n {side} ({n_total} particles), "
                               f"{'std (HydroProp)' if std_prop else 'VE'} propagator"
                               f"{' + self-gravity' if args.init == 'evrard' else ''}"
                               f"{' + AV cleaning' if args.av_clean else ''}, {args.steps} steps",
                   "particles_per_gpu": n_local, "bucket": args.bucket, "ngmax": 150, "ng0": 100,
                   "parallelism": "1 GPU" if world == 1 else
                   f"{world} GPUs: SFC domain decomposition, halo + particle exchange over {transport}",
                   "halos_per_gpu": sim.layout()["n"] - n_local,
                   **({"gravity_halos_per_gpu": sim.gravity_stats()["halos"],
                       "gravity_far_cells": sim.gravity_stats()["far_cells"]} if world > 1 and args.init == "evrard"
                      else {}),
                   "kernels": "exact (no FMA)" if args.exact else "fast (FMA)"},
        "roofline": {"bound": "hbm", "kernel": mom_kernel, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(mom_kernel, n_local),
                     "algorithmic_bytes_per_launch": mom_bytes, "avg_launch_ms": mom_ms,
                     "model": f"edge model (SURVEY.md 8(d)): {own_b} B own + {ng:.1f} neighbors x "
                              f"{edge_b} B; effective bandwidth, neighbor records come from LDS",
                     "compulsory_bytes_per_launch": comp_bytes,
                     "compulsory_frac": comp_bytes / (mom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "valu": {"flop_per_pair": MOM_FLOP_PER_PAIR, "achieved_tflops": mom_tflops,
                              "peak_tflops": FP32_PEAK_TFLOPS, "frac": mom_tflops / FP32_PEAK_TFLOPS},
                     "traffic_source": os.path.relpath(PMC_FILE, ROOT)},
        "kernels_ms": {(STD_KERNEL_NAMES.get(k) if std_prop else k): v / args.steps for k, v in kern_sum.items()
                       if not std_prop or k in STD_KERNEL_NAMES},
        "stages_ms": {k: v / args.steps for k, v in stage_sum.items()},
        "neighbors_per_particle": ng,
        "candidates_per_particle": stats["sumCandidates"] / max(1, n_local),
        "union_per_particle": stats["sumUnion"] / max(1, n_local),
        "minDt": sc["minDt"],
    }
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    sim.close()
    if comm is not None:
        comm.close()
    ctx.close()
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
