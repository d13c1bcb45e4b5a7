"""Benchmark: particle-updates/s of the VE time step (Sedov lattice) on N MI355X, one process per GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--side S] [--no-cpu-baseline]

A step is one full HydroVeProp step (ve_hydro.hpp:132-218): sync (keys, sort, reorder, tree), neighbor search with
h iteration, XMass, VeDefGradh, EOS, IAD+divv/curlv, AV switches, momentum/energy, [self-gravity], time-step,
positions, h update.  --init noh|evrard run BASELINE configs 3 and 5 (lattice substitutes for the glass block).
Inputs are generated and kept in HBM; nothing leaves the device inside the timed region except the per-step
4-byte tree-level counts and stats.  The workload is the metric's own: Sedov -n 400 (64M particles) in total at every
N (strong scaling: N=1 holds all 64M particles on one MI355X, N=8 holds 8M + halos per GPU); --side 200 gives
BASELINE config 2.
With skin lists (one rank, the default) the timed window starts with a forced full sync + skin build, so the headline
carries the builds' cost (1 per K steps; the steady state has 1 per max_reuse = 24, reported as amortized_*).
Rank 0 prints ONE JSON line.  Its "roofline" is the dominant kernel's (largest share of the step): HBM bytes per
launch from the committed rocprofv3 PMC passes of the same workload (profiles/pmc_<init>_n<side>.json) over the kernel's
average launch time measured here with HIP events on its stream.
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
NUM_CU = 256
CLOCK_HZ = 2.4e9
# wave64 VALU instructions per second the chip can issue: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 op
# (measured: VeDefGradh issues faster than one op per 4 cycles per SIMD)
VALU_ISSUE_PEAK = NUM_CU * 4 * CLOCK_HZ / 2
MOM_FLOP_PER_PAIR = 150  # SURVEY.md 8(d) secondary VALU figure
# SURVEY.md 8(d) flop per neighbor pair of each pair kernel (the reference's J-loops: XMass 17, VeDefGradh 29,
# IAD+divv/curlv 95, AV switches 57, momentum 150); valu_frac = pairs x flop / time / FP32 peak (157.3 TF = 2.4 GHz x
# 256 CUs x 128 lanes x 2 flop per FMA x 2 packed lanes -- the clock is the peak's 2.4 GHz, the kernels run at
# 1.83-2.34 GHz, profiles/r3b_pmc_clock_waits_sedov_n400.txt)
FLOP_PER_PAIR = {"xmass": 17, "veDefGradh": 29, "iadDivvCurlv": 95, "avSwitches": 57, "momentumEnergy": 150}
# self-gravity flop per interaction: the reference's own accounting (nbody/traversal.cuh:632: 20 per P2P, 2 P^3 = 16
# per quadrupole M2P) and this kernel's (sx_gravity.hip: P2P 23 flop -- as ryoanji/test/demo_mpi.cpp:118 --, M2P 54)
GRAV_FLOP_REF = (20, 16)
GRAV_FLOP_IMPL = (23, 54)
# SURVEY.md 8(d) edge model per kernel: own record R+W, and index + neighbor record per edge.  Reads of neighbor
# records come from LDS/L2, so edge-model bytes / time is an EFFECTIVE bandwidth, reported as effective_gbs only.
EDGE_MODEL = {"findNeighbors": (32, 28), "xmass": (44, 32), "veDefGradh": (48, 36), "iadDivvCurlv": (80, 48),
              "avSwitches": (88, 52), "momentumEnergy": (108, 92)}
# compulsory (unique-field) HBM bytes per target as implemented: packed own records + outputs, plus
# 2 B per stored neighbor (u16 union positions) and 4 B per union entry; the search reads x,y,z,h (28 B) and the
# tree, writes h, nc, the lists and the targets' 32-B RecX records (NsArgs::rxOut)
COMPULSORY_OWN = {"findNeighbors": 28 + 8 + 32, "xmass": 32 + 4 + 4, "veDefGradh": 48 + 4 + 8,
                  "iadDivvCurlv": 80 + 4 + 28, "avSwitches": 96 + 4 + 4, "momentumEnergy": 96 + 4 + 20}
# kernel-time slot -> rocprofv3 kernel-name fragments it launches (sx_sim.cpp kev slots)
PMC_KERNELS = {"findNeighbors": ("findNeighborsKernel", "leafFrameKernel", "skinFilterKernel", "dispGridKernel",
                                  "leafBoxKernel", "innerBoxKernel"), "xmass": ("xmassKernel",),
               "veDefGradh": ("veDefGradhKernel",), "iadDivvCurlv": ("iadDivvCurlv",),
               "avSwitches": ("avSwitchesKernel",), "momentumEnergy": ("momentumEnergyKernel",),
               "gravity": ("gravityTraverseKernel",)}
# std propagator momentum (hydro_std/momentum_energy_kern.hpp): own x,y,z,v,h,m,rho,p,c,c_ij + nc read, a,du written;
# per edge the index + x,y,z (24) v (12) h m rho p c (20) c_ij (24)
MOM_STD_OWN_BYTES = 24 + 12 + 20 + 24 + 4 + 12 + 8
MOM_STD_EDGE_BYTES = 4 + 80
# kernel-time slots of sx_sim in std mode (sx_sim.cpp: density in "xmass", IAD in "iadDivvCurlv")
STD_KERNEL_NAMES = {"findNeighbors": "findNeighbors", "xmass": "density", "iadDivvCurlv": "iad",
                    "momentumEnergy": "momentumEnergySTD", "gravity": "gravity"}


def pmc_file(key):
    """the committed rocprofv3 --pmc summary of one workload: profiles/pmc_<init>_n<side>[_<variant>].json"""
    return os.path.join(ROOT, "profiles", f"pmc_{key}.json")


def load_pmc(key, particles, workload):
    """per-kernel rocprofv3 --pmc summary of the same workload (scripts/gpu_pmc.sh + scripts/pmc_summary.py, KB
    units), or None when absent or taken on another workload"""
    try:
        with open(pmc_file(key)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    meta = d.get("_meta", {})
    if meta.get("particles_per_gpu") != particles or meta.get("workload", "").split(",")[0] != workload.split(",")[0]:
        return None
    return d


# kernels of a full search build: not part of a step the skin filter served (sx_skin.hpp)
SEARCH_BUILD_KERNELS = ("findNeighborsKernel", "leafFrameKernel")


def pmc_slot(pmc, slot, exclude=()):
    """counters of one kernel-time slot, summed over the kernels it launches, per launch of the slot (kernels whose
    name contains an `exclude` fragment left out)"""
    if pmc is None:
        return None
    frags = PMC_KERNELS.get(slot, ())
    tot, hit = {}, False
    for k, v in pmc.items():
        if k == "_meta" or not any(f in k for f in frags) or any(f in k for f in exclude):
            continue
        hit = True
        calls = v.get("calls_per_step", 1.0)
        for c in ("hbm_read_bytes_est", "hbm_write_bytes_est", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT",
                  "profiled_ms"):
            if c in v:
                tot[c] = tot.get(c, 0.0) + v[c] * calls
    return tot if hit else None


CALIB_FILE = os.path.join(ROOT, "profiles", "r3_fetch_calib.json")


def step_traffic(pmc, reuse_only=False):
    """HBM bytes of one whole step from the PMC summary: every kernel's (FETCH_SIZE x2 + WRITE_SIZE) x its launches
    per step.  reuse_only: the timed steps were all served by the skin filter, so the kernels the PMC run launched
    less than once per step (its initial sync and full build) are left out"""
    if pmc is None:
        return None
    tot = 0.0
    for k, v in pmc.items():
        if k == "_meta" or (reuse_only and v.get("calls_per_step", 1.0) < 0.99):
            continue
        tot += (v.get("hbm_read_bytes_est", 0.0) + v.get("hbm_write_bytes_est", 0.0)) * v.get("calls_per_step", 1.0)
    return tot


def calibration():
    """FETCH_SIZE / WRITE_SIZE factors measured on this library's access shapes (scripts/fetch_calib.hip)"""
    try:
        with open(CALIB_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return {k: round(v["factor"], 3) for k, v in d.items() if v.get("factor")}


def kernel_roofline(slot, ms, n_local, ng, union_pp, pmc, exclude=()):
    """roofline entry of one kernel-time slot: HBM counter bytes / measured time vs the 8 TB/s peak, VALU issue and
    LDS conflict shares from the same counters, edge-model effective bandwidth"""
    own, edge = EDGE_MODEL.get(slot, (0, 0))
    r = {"avg_launch_ms": ms}
    if own:
        r["effective_gbs"] = n_local * (own + ng * edge) / (ms * 1e-3) / 1e9
    if slot in COMPULSORY_OWN:
        r["algorithmic_bytes_per_launch"] = n_local * (COMPULSORY_OWN[slot] + 2 * ng + 4 * union_pp)
        r["algorithmic_frac"] = r["algorithmic_bytes_per_launch"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    c = pmc_slot(pmc, slot, exclude)
    if c and "hbm_read_bytes_est" in c and "hbm_write_bytes_est" in c:
        traffic = c["hbm_read_bytes_est"] + c["hbm_write_bytes_est"]
        r["traffic"] = traffic
        r["achieved"] = traffic / (ms * 1e-3) / 1e9
        r["frac"] = r["achieved"] / HBM_PEAK_GBS
    else:
        r["traffic"] = r["achieved"] = r["frac"] = None
    if c and "SQ_INSTS_VALU" in c:
        r["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (ms * 1e-3 * VALU_ISSUE_PEAK)
        if slot in FLOP_PER_PAIR:  # lane-instructions per neighbor pair (wave64 instructions x 64 / pairs)
            r["valu_lane_ops_per_pair"] = c["SQ_INSTS_VALU"] * 64 / max(1.0, n_local * ng)
    if c and "SQ_LDS_BANK_CONFLICT" in c:
        r["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / NUM_CU / (ms * 1e-3 * CLOCK_HZ)
    if c and "profiled_ms" in c:
        r["pmc_profiled_ms"] = c["profiled_ms"]
    if slot in FLOP_PER_PAIR:
        r["tflops"] = n_local * ng * FLOP_PER_PAIR[slot] / (ms * 1e-3) / 1e12
        r["valu_frac"] = r["tflops"] / FP32_PEAK_TFLOPS
    return r


def gravity_roofline(ms, n_local, inter, pmc):
    """self-gravity traversal: FLOP roofline (FP32 VALU) from the per-target interaction counts of one step right
    after the timed ones (sx_sim_set_gravity_counting + sx_sim_gravity_interactions, the reference's BhStats; the
    timed steps run the non-counting traversal) -- the kernel is compute/latency bound, its HBM traffic is a few % of
    the peak"""
    p2p, m2p = inter["p2p"], inter["m2p"]
    flop_impl = GRAV_FLOP_IMPL[0] * p2p + GRAV_FLOP_IMPL[1] * m2p
    flop_ref = GRAV_FLOP_REF[0] * p2p + GRAV_FLOP_REF[1] * m2p
    r = {"avg_launch_ms": ms, "p2p_per_target": p2p / max(1, n_local), "m2p_per_target": m2p / max(1, n_local),
         "tflops": flop_impl / (ms * 1e-3) / 1e12, "tflops_reference_model": flop_ref / (ms * 1e-3) / 1e12}
    # headline: the reference's own flop accounting (traversal.cuh:632); the implementation's count is secondary
    r["flop_frac"] = r["tflops_reference_model"] / FP32_PEAK_TFLOPS
    r["flop_frac_impl_model"] = r["tflops"] / FP32_PEAK_TFLOPS
    c = pmc_slot(pmc, "gravity")
    if c and "SQ_INSTS_VALU" in c:
        r["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (ms * 1e-3 * VALU_ISSUE_PEAK)
    if c and "hbm_read_bytes_est" in c and "hbm_write_bytes_est" in c:
        r["traffic"] = c["hbm_read_bytes_est"] + c["hbm_write_bytes_est"]
        r["hbm_frac"] = r["traffic"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    return r


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24, help="timed steps (default: one skin cycle, max_reuse)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--side", type=int, default=0,
                    help="total lattice side (default: the metric's Sedov -n 400 at every N; noh/evrard 300)")
    ap.add_argument("--bucket", type=int, default=64)
    ap.add_argument("--exact", action="store_true", help="use the no-FMA (bit-reproducible) kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-build-step", action="store_true",
                    help="do not force a full sync + skin build at the start of the timed window (profiling runs of "
                         "filter-served steps only: the PMC summary normalises its counters by steps + warmup)")
    ap.add_argument("--backend", default="rccl", help="rccl (one GPU per rank) or host (staged, tests)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--cpu-side", type=int, default=200, help="Sedov lattice side of the CPU baseline sample")
    ap.add_argument("--init", default="sedov", choices=["sedov", "noh", "evrard"],
                    help="sedov (BASELINE metric, device IC), noh (config 3), evrard (config 5: VE + self-gravity)")
    ap.add_argument("--av-clean", action="store_true", help="HydroVeProp<avClean=true>")
    ap.add_argument("--prop", default="ve", choices=["ve", "std"],
                    help="ve (HydroVeProp, the BASELINE metric) or std (HydroProp, std_hydro.hpp)")
    ap.add_argument("--skin", type=float, default=0.05,
                    help="neighbor lists behind a skin 2h(1+s) between full builds (sx_sim_set_skin; 0: sync + "
                         "search every step, the reference's flow)")
    ap.add_argument("--skin-reuse", type=int, default=24, help="steps between full builds at most")
    ap.add_argument("--seam", action="store_true",
                    help="the drop-in path instead: whole VE steps through the C++ mirror of the reference seam "
                         "(sph-exa_amd/lib/ve_seam_bench, every call synchronous, sync + search every step), "
                         "default Sedov -n 200; prints that program's JSON line")
    return ap.parse_args()


def seam_bench(args):
    """the reference propagator's view of this library: ve_seam_bench (host/examples/ve_seam_bench.cpp) as a child
    process on one GPU, its JSON line passed through with the sx_sim figure of the same workload for comparison"""
    import subprocess

    exe = os.path.join(ROOT, "sph-exa_amd", "lib", "ve_seam_bench")
    if not os.path.exists(exe):
        raise SystemExit("sph-exa_amd/lib/ve_seam_bench missing: make -C sph-exa_amd")
    side = args.side or 200
    r = subprocess.run([exe, str(side), str(args.steps), str(args.warmup)], capture_output=True, text=True,
                       timeout=1200)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-2000:] + r.stderr[-2000:])
        raise SystemExit(r.returncode)
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds, side):
    """Reference CPU path (oracle/_ref, OpenMP) timed on this host on a bounded sample of the same Sedov workload:
    the lattice of side `side` (n=200: 8M particles, one step ~4 s on 16 cores), one warm-up step, then whole steps
    until `seconds` have passed (at least one)."""
    import pyoracle as po

    kind = "reference"
    path = os.path.join(ROOT, "oracle", "_ref", "libsphexa_ref_fast.so")
    if not os.path.exists(path):
        path = os.path.join(ROOT, "oracle", "_ref", "libsphexa_ref.so")
    if not os.path.exists(path):
        path, kind = po.ORACLE_SO, "port"
    lib = po.Lib(path)
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
            "cpu_model": cpu_model(),
            "sample": f"Sedov lattice -n {side} ({st.n} particles, the metric's Sedov IC at 1/8 the particles), "
                      f"{steps} VE steps after 1 warm-up, {os.path.basename(path)} (the reference's own CPU "
                      f"loops, -O3 -march=x86-64-v3), OMP threads={cores}, "
                      f"OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND', 'unset')}, "
                      f"OMP_PLACES={os.environ.get('OMP_PLACES', 'unset')}"}


def main():
    args = parse()
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_cpu_baseline:
        # the reference CPU baseline's OpenMP threads pinned to cores, close together; set before any
        # OpenMP runtime is loaded (the reference library is loaded only by cpu_baseline)
        os.environ.setdefault("OMP_PROC_BIND", "close")
        os.environ.setdefault("OMP_PLACES", "cores")
    if args.seam:
        print(json.dumps(seam_bench(args)))
        return
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

    side = args.side or {"sedov": 400, "noh": 300, "evrard": 300}[args.init]
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
    sim.set_skin(args.skin, args.skin_reuse)
    comm = None
    transport = args.backend
    if world > 1:
        # no silent fallback: a scaling run that cannot create its RCCL communicator fails (a host-staged run would
        # time PCIe + gloo instead of xGMI)
        try:
            comm = sx.Comm(args.backend)
            ok = 1
        except sx.SxError as e:
            print(f"rank {rank}: {e}", file=sys.stderr)
            ok = 0
        import torch

        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)  # every rank learns whether some rank failed
        if int(flag.item()) == 0:
            print(f"rank {rank}: {args.backend} communicator creation failed on some rank; no bench line",
                  file=sys.stderr)
            dist.destroy_process_group()
            sys.exit(3)
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

    # skin lists: the timed window starts with a full sync + build of every cluster's skin (on every rank: the build
    # decisions are collective), so `value` and `ms_per_step` carry at least their share of the builds that come every
    # max_reuse steps at the latest (a window shorter than max_reuse carries more than its share: 1 build in K steps,
    # against 1 in max_reuse)
    skin_window = args.skin > 0 and not args.no_build_step
    if skin_window:
        sim.rebuild_lists()
    ctx.sync()
    barrier()
    skin0 = sim.skin_stats()
    stage_sum, kern_sum, kern_steps = {}, {}, {}
    step_s = []  # host time of every timed step (sx_sim_step returns after its stream synchronisation)
    search_ms, kept_steps = [], []  # per step: the search slot's kernel time, clusters whose exact lists were kept
    # (of them frozen)
    kept0, frz0 = skin0.get("kept_clusters", 0), skin0.get("frozen_clusters", 0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        sim.step()
        step_s.append(time.perf_counter() - ts)
        for k, v in sim.stage_times().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
        kt = sim.kernel_times()
        for k, v in kt.items():
            kern_sum[k] = kern_sum.get(k, 0.0) + v
            if v > 0.0:
                kern_steps.setdefault(k, []).append(round(v, 2))
        search_ms.append(round(kt.get("findNeighbors", 0.0), 3))
        if args.skin > 0:
            ks = sim.skin_stats()
            kept_steps.append((int(ks["kept_clusters"] - kept0), int(ks["frozen_clusters"] - frz0)))
            kept0, frz0 = ks["kept_clusters"], ks["frozen_clusters"]
    ctx.sync()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    stats = sim.stats()
    skin = {k: (v - skin0[k] if k in ("builds", "reuse_steps", "stale_clusters", "exact_clusters", "plain_steps",
                                      "kept_clusters", "frozen_clusters", "early_exact") else v)
            for k, v in sim.skin_stats().items()}  # the timed steps'
    if args.skin > 0:
        skin["search_ms_per_step"] = search_ms
        skin["kept_frozen_clusters_per_step"] = kept_steps
    n_local = sim.size()
    ms_step = el / args.steps * 1e3
    if dist is not None:  # per-step times: the slowest rank's
        import torch

        t = torch.tensor(step_s, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_s = [float(v) for v in t]
    if skin_window and args.steps > 1 and skin.get("builds", 0) >= 1:
        # the window's first step was the full sync + build, the others (up to max_reuse) filter-served
        R = max(1, int(args.skin_reuse))
        build_ms = step_s[0] * 1e3
        filt_ms = sum(step_s[1:]) / (len(step_s) - 1) * 1e3
        skin["build_step_ms"] = build_ms
        skin["filter_step_ms"] = filt_ms
        skin["filter_step_value"] = n_total / (filt_ms * 1e-3)
        skin["amortized_ms_per_step"] = (filt_ms * (R - 1) + build_ms) / R
        skin["amortized_value"] = n_total / (skin["amortized_ms_per_step"] * 1e-3)
        skin["amortized_note"] = (f"value/ms_per_step: the timed window starts with a full sync + skin build "
                                  f"({skin['builds']} build(s) in {args.steps} steps); amortized: one build every {R} "
                                  "steps (max_reuse), the other steps filter-served; both from the same window's "
                                  "per-step host times")
    inter = None
    if args.init == "evrard":  # self-gravity on (g = 1); the same decision on every rank: the extra step is collective
        # the interaction counts (BhStats) of one more step after the timed region: counting is a separate, slower
        # instantiation of the traversal, so the timed steps run without it
        sim.set_gravity_counting(True)
        sim.step()
        inter = sim.gravity_interactions()
        sim.set_gravity_counting(False)
    ng = stats["sumNeighbors"] / max(1, n_local)
    union_pp = stats["sumUnion"] / max(1, n_local)
    std_prop = args.prop == "std"
    kern_ms = {k: v / args.steps for k, v in kern_sum.items()}
    workload = (f"{args.init.capitalize()} -n {side} ({n_total} particles), "
                f"{'std (HydroProp)' if std_prop else 'VE'} propagator"
                f"{' + self-gravity' if args.init == 'evrard' else ''}"
                f"{' + AV cleaning' if args.av_clean else ''}, {args.steps} steps")
    pmc_key = f"{args.init}_n{side}" + ("_avclean" if args.av_clean else "") + ("_std" if std_prop else "")
    pmc = load_pmc(pmc_key, n_local, workload) if not std_prop else None
    per_kernel = {}
    for k, ms in kern_ms.items():
        if ms > 0.01 and k in EDGE_MODEL:
            # every timed step served by the skin filter: the search slot's counters are the filter's alone (the
            # PMC run's first step is a full build, whose kernels would be averaged in)
            ex = SEARCH_BUILD_KERNELS if (k == "findNeighbors" and skin.get("builds", 1) == 0 and
                                          skin.get("plain_steps", 1) == 0 and skin.get("reuse_steps", 0) > 0) else ()
            per_kernel[k] = kernel_roofline(k, ms, n_local, ng, union_pp, pmc, ex)
        elif ms > 0.01 and k == "gravity" and inter is not None:  # (without self-gravity the slot times no kernel)
            per_kernel[k] = gravity_roofline(ms, n_local, inter, pmc)
    dominant = max(per_kernel, key=lambda k: per_kernel[k]["avg_launch_ms"]) if per_kernel else "momentumEnergy"
    dom = per_kernel.get(dominant, {})
    grav_dom = dominant == "gravity"
    roofline = {"bound": "valu" if grav_dom else "hbm", "kernel": dominant,
                "achieved": dom.get("tflops_reference_model") if grav_dom else dom.get("achieved"),
                "peak": FP32_PEAK_TFLOPS if grav_dom else HBM_PEAK_GBS,
                "unit": "TFLOP/s" if grav_dom else "GB/s",
                "frac": dom.get("flop_frac") if grav_dom else dom.get("frac"), "traffic": dom.get("traffic"),
                "avg_launch_ms": dom.get("avg_launch_ms"),
                "share_of_step": dom.get("avg_launch_ms", 0.0) / ms_step,
                "binding": ("FP32 VALU / latency: flop roofline from the per-target P2P/M2P counts (see "
                            "tflops (this kernel's own count), valu_issue_frac, hbm_frac)" if grav_dom else
                            "valu-issue/latency (HBM frac < 0.5; see valu_issue_frac, lds_conflict_frac)"
                            if (dom.get("frac") or 0) < 0.5 else "hbm"),
                "traffic_source": os.path.relpath(pmc_file(pmc_key), ROOT) if pmc else None,
                "definition": "achieved = rocprofv3 PMC HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, same "
                              "workload; FETCH_SIZE x2 equals the bytes read for coalesced 4/8/16-B streams and "
                              "leaf-run record gathers, profiles/r3_fetch_calib.json; for random 16-B/4-B gathers "
                              "the calibration only shows FETCH_SIZE x2 at 3.3x/8.2x the useful bytes, i.e. whole "
                              "lines, so the x2 reading is inferred there, not measured) / avg launch time measured "
                              "live with HIP events; frac = achieved / 8 TB/s; "
                              "valu_issue_frac = SQ_INSTS_VALU / (time x 1.23e12 wave64 ops/s: 2 cycles per "
                              "instruction per SIMD-32 at 2.4 GHz, the chip's rate; one wave alone issues at most "
                              "half of it, profiles/r4_issue_calib.jsonl); valu_frac = SURVEY 8(d) flop "
                              "per pair x pairs / time / 157.3 TF (FP32 peak at 2.4 GHz); gravity: achieved and "
                              "flop_frac = the reference's accounting (traversal.cuh:632: 20 per P2P + 16 per M2P) / "
                              "time / 157.3 TF, flop_frac_impl_model = this kernel's (23 P2P + 54 M2P); "
                              "lds_conflict_frac = "
                              "SQ_LDS_BANK_CONFLICT / 256 CUs / (time x 2.4 GHz); effective_gbs = SURVEY 8(d) edge "
                              "model (neighbor records served from LDS/L2, not a roofline)",
                **{k: dom[k] for k in ("valu_issue_frac", "lds_conflict_frac", "effective_gbs",
                                       "algorithmic_bytes_per_launch", "algorithmic_frac", "hbm_frac",
                                       "tflops", "flop_frac_impl_model", "p2p_per_target", "m2p_per_target",
                                       "valu_lane_ops_per_pair") if k in dom},
                "per_kernel": per_kernel}
    st_bytes = step_traffic(pmc, skin.get("builds", 1) == 0 and skin.get("plain_steps", 1) == 0 and
                            skin.get("reuse_steps", 0) > 0)
    if st_bytes:
        roofline["step_traffic"] = st_bytes
        roofline["step_hbm_gbs"] = st_bytes / (ms_step * 1e-3) / 1e9
        roofline["step_hbm_frac"] = roofline["step_hbm_gbs"] / HBM_PEAK_GBS
    cal = calibration()
    if cal:
        roofline["counter_calibration"] = {"source": os.path.relpath(CALIB_FILE, ROOT),
                                           "known_bytes_per_counter_byte": cal}
    mom = per_kernel.get("momentumEnergy")
    if mom and not std_prop:
        roofline["momentum_valu"] = {"flop_per_pair": MOM_FLOP_PER_PAIR,
                                     "achieved_tflops": n_local * ng * MOM_FLOP_PER_PAIR /
                                     (mom["avg_launch_ms"] * 1e-3) / 1e12, "peak_tflops": FP32_PEAK_TFLOPS}
    if std_prop:
        mom_ms = kern_ms.get("momentumEnergy", float("nan"))
        roofline["effective_gbs_momentumStd"] = n_local * (MOM_STD_OWN_BYTES + ng * MOM_STD_EDGE_BYTES) / \
            (mom_ms * 1e-3) / 1e9
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
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 hydro / f64 coordinates (sph::SphTypes)",
        "data": "synthetic Sedov lattice generated on device (sedov_init.hpp), no checkpoint" if ic_arrays is None
                else f"synthetic {args.init} lattice substitute for the glass block (SURVEY F6), sphexa_amd/ic.py",
        "config": {"workload": workload,
                   "particles_per_gpu": n_local, "bucket": args.bucket, "ngmax": 150, "ng0": 100,
                   "parallelism": "1 GPU" if world == 1 else
                   f"{world} GPUs: SFC domain decomposition, halo + particle exchange over {transport}",
                   "halos_per_gpu": sim.layout()["n"] - n_local,
                   **({"gravity_halos_per_gpu": sim.gravity_stats()["halos"],
                       "gravity_far_cells": sim.gravity_stats()["far_cells"]} if world > 1 and args.init == "evrard"
                      else {}),
                   "kernels": "exact (no FMA)" if args.exact else "fast (FMA)",
                   "neighbor_skin": {"initial_factor": args.skin, "max_reuse": args.skin_reuse,
                                     "note": "steps between full builds filter the last build's lists within "
                                             "2h(1+s) (sx_skin.hpp; several ranks: halos of the build refreshed, "
                                             "displacement grid all-reduced); same neighbor sets, nc, h",
                                     **skin}},
        "roofline": roofline,
        "kernels_ms": {(STD_KERNEL_NAMES.get(k) if std_prop else k): v for k, v in kern_ms.items()
                       if not std_prop or k in STD_KERNEL_NAMES},
        "stages_ms": {k: v / args.steps for k, v in stage_sum.items()},
        # per timed step (the lattice's h moves across a shell every other step: 92- and 122-neighbor steps differ)
        "kernels_ms_per_step": {(STD_KERNEL_NAMES.get(k) if std_prop else k): v for k, v in kern_steps.items()
                                if not std_prop or k in STD_KERNEL_NAMES},
        "neighbors_per_particle": ng,
        "candidates_per_particle": stats["sumCandidates"] / max(1, n_local),
        "union_per_particle": union_pp,
        "minDt": sc["minDt"],
    }
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.cpu_side)
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
