"""Block time-steps at scale: HydroVeBdtProp (sphexa_amd.ve_bdt) vs the VE propagator (sx_sim) on the same Sedov
lattice generated on the device, one GPU.  Prints one JSON line: per substep the active particles and wall time,
and for both propagators the simulated time advanced per wall second over the same number of hierarchies.

  python scripts/bdt_bench.py --side 200 --hierarchies 2
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sph-exa_amd", "python"))

import numpy as np  # noqa: E402

import sphexa_amd as sx  # noqa: E402
from sphexa_amd.ve_bdt import HydroVeBdtProp  # noqa: E402

CONS = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", type=int, default=200)
    ap.add_argument("--hierarchies", type=int, default=2)
    ap.add_argument("--warmup-steps", type=int, default=1, help="VE steps before both runs (converged h)")
    args = ap.parse_args()
    n = args.side ** 3
    ctx = sx.Context(0)
    box = sx.make_box([-0.5, 0.5] * 3, [1, 1, 1])
    sim = sx.Sim(ctx, n, box)
    sim.init_sedov(args.side)
    for _ in range(args.warmup_steps):
        sim.step()
    host = sim.get(CONS)
    sc = sim.scalars()
    t_start = sc["ttot"]

    prop = HydroVeBdtProp(ctx, host, box, sc["minDt"], min_dt_m1=sc["minDt_m1"])
    subs = []
    ctx.sync()
    t0 = time.perf_counter()
    hier = 0
    while hier < args.hierarchies:
        a = time.perf_counter()
        prop.step()
        subs.append(dict(ms=1e3 * (time.perf_counter() - a), numRungs=prop.ts.numRungs,
                         rungRanges=list(prop.ts.rungRanges), dt=float(prop.ts.nextDt)))
        hier += prop.is_synced()
    bdt_wall = time.perf_counter() - t0
    bdt_sim = prop.ttot

    # the VE propagator over the same simulated time
    t0 = time.perf_counter()
    steps = 0
    while sim.scalars()["ttot"] - t_start < bdt_sim and steps < 10 * len(subs):
        sim.step()
        steps += 1
    ve_wall = time.perf_counter() - t0
    ve_sim = sim.scalars()["ttot"] - t_start
    print(json.dumps(dict(workload=f"Sedov -n {args.side} ({n} particles)", substeps=len(subs),
                          bdt=dict(wall_s=bdt_wall, sim_time=bdt_sim, sim_time_per_s=bdt_sim / bdt_wall,
                                   ms_per_substep=[round(s["ms"], 2) for s in subs],
                                   numRungs=[s["numRungs"] for s in subs], rungRanges=subs[0]["rungRanges"]),
                          ve=dict(wall_s=ve_wall, steps=steps, sim_time=ve_sim, sim_time_per_s=ve_sim / ve_wall,
                                  ms_per_step=1e3 * ve_wall / max(1, steps)))))
    sim.close()
    ctx.close()


if __name__ == "__main__":
    main()
