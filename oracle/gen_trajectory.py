"""Trajectory fixtures: whole runs of the reference's CPU path at the configured step counts.

TEST INFRASTRUCTURE ONLY. Run in the build container, where /root/reference exists:
    make -C oracle && OMP_NUM_THREADS=8 python oracle/gen_trajectory.py [--fast] [case ...]   (trajectory.CASES)

For each case of trajectory.CASES the reference's own VE step (oracle/_ref, ref_step: Domain::sync + computeForces +
integrate of ve_hydro.hpp:132-218, F2-corrected) runs from the IC for the configured number of steps, un-reseeded,
and the fixture records
  * per step: ttot, minDt, total energy, |linear momentum|;
  * at the profile steps: the binned radial profiles of trajectory.profiles (rho, p, |v|, u) and the bin counts;
  * Sedov only: the reference's analytic solution (oracle/_ref/sedov_solution, built from
    main/src/analytical_solutions/sedov_solution) at the final time, its r/rho/p/vel columns, and the density L1 of
    the reference run against it by compare_solutions.py's formula (the number the reference CI asserts:
    0.138 -0.015/+0.01 at Sedov -n 50 -s 200, .jenkins/reframe_ci.py:286,350-351).
The fixtures are data (outputs of the reference), committed under tests/golden/traj_*.npz.
"""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402
import trajectory as tj  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
SOLVER = os.path.join(HERE, "_ref", "sedov_solution")


def sedov_solution(t):
    """run the reference's solver at time t; returns the (r, rho, u, p, vel, cs) columns"""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sol.dat")
        subprocess.run([SOLVER, "--time", repr(float(t)), "--out", out], check=True, capture_output=True, cwd=d)
        return np.loadtxt(out)


def run_case(ref, name):
    fname, init, side, steps, prof_steps, rmax, nbins = tj.CASES[name]
    kw = tj.CASE_PARAMS.get(name, {})
    std = bool(kw.get("std", False))
    params = ref.params(**kw)
    st, box = getattr(po, init + "_state")(side)
    out = {"box": np.array(list(box.lim) + list(box.bnd), np.float64), "side": np.array([side]),
           "steps": np.array([steps]), "prof_steps": np.array(prof_steps), "rmax": np.array([rmax]),
           "nbins": np.array([nbins])}
    e0, p0 = tj.energies(st.arrays)
    ser = {"ttot": [0.0], "minDt": [st.minDt], "etot": [e0], "mom": [p0]}
    if params.g != 0.0:
        ser["egrav"] = [float("nan")]  # the potential of a state is computed inside its step (of the state before)
    t0 = time.time()
    for s in range(1, steps + 1):
        ref.step(st, box, params=params)
        e, p = tj.energies(st.arrays)
        if params.g != 0.0:
            ser["egrav"].append(st.egrav)
        ser["ttot"].append(st.ttot)
        ser["minDt"].append(st.minDt)
        ser["etot"].append(e)
        ser["mom"].append(p)
        if s in prof_steps:
            _, prof, cnt = tj.profiles(st.arrays, rmax, nbins, std=std)
            for k, v in prof.items():
                out[f"s{s}_{k}"] = v
            out[f"s{s}_count"] = cnt
            print(f"{name} step {s}: t={st.ttot:.6g} dt={st.minDt:.3g} etot={e:.10g} ({time.time() - t0:.0f} s)",
                  flush=True)
        elif st.n > 1_000_000 and s % 5 == 0:
            print(f"{name} step {s} ({time.time() - t0:.0f} s)", flush=True)
    for k, v in ser.items():
        out["series_" + k] = np.array(v, np.float64)
    if init == "sedov":
        sol = sedov_solution(st.ttot)
        r = tj.radii(st.arrays)
        rho, p = tj.eos_rho_p(st.arrays, std=std)
        vel = np.sqrt(sum(st.arrays[k].astype(np.float64) ** 2 for k in ("vx", "vy", "vz")))
        l1 = tj.analytic_l1(r, rho.astype(np.float64), sol[:, 0], sol[:, 1])
        # compare_solutions.py:115,126 compare p and |v| against the solution's rho column; both printed
        out["ref_l1_density"] = np.array([l1])
        out["ref_l1_pressure_vs_rho_col"] = np.array([tj.analytic_l1(r, p.astype(np.float64), sol[:, 0], sol[:, 1])])
        out["ref_l1_velocity_vs_rho_col"] = np.array([tj.analytic_l1(r, vel, sol[:, 0], sol[:, 1])])
        # the solution columns on every 10th row of the solver's 1e5-row grid plus the two shock-front rows
        shock = np.nonzero(np.diff(sol[:, 1]) != 0)[0]
        rows = np.union1d(np.arange(0, sol.shape[0], 10), np.concatenate([shock, shock + 1]))
        rows = rows[rows < sol.shape[0]]
        out["sol_time"] = np.array([st.ttot])
        out["sol"] = sol[rows][:, [0, 1, 3, 4]]  # r, rho, p, vel
        out["ref_l1_density_subsampled"] = np.array([tj.analytic_l1(r, rho.astype(np.float64), out["sol"][:, 0],
                                                                    out["sol"][:, 1])])
        print(f"{name}: density L1 vs analytic = {l1:.4f} (subsampled solution {out['ref_l1_density_subsampled'][0]:.4f})"
              f" at t = {st.ttot:.6g}")
    if init == "noh":
        out["final_time"] = np.array([st.ttot])
        out["ref_l1_noh_density_attr"] = np.array([tj.noh_l1(st.arrays, st.ttot, tj.NOH_RHO0_ATTR)])
        out["ref_l1_noh_density_ic"] = np.array([tj.noh_l1(st.arrays, st.ttot, tj.NOH_RHO0_IC)])
        print(f"{name}: density L1 vs nohRho at t = {st.ttot:.6g}: {out['ref_l1_noh_density_attr'][0]:.4f} "
              f"(rho0 = 1, compare_noh.py), {out['ref_l1_noh_density_ic'][0]:.4f} (rho0 of the IC)")
    np.savez_compressed(os.path.join(OUT, fname), **out)
    print(fname, os.path.getsize(os.path.join(OUT, fname)), "bytes;",
          f"energy drift {ser['etot'][-1] / ser['etot'][0] - 1:.3g}")


def main():
    args = sys.argv[1:]
    fast = "--fast" in args  # the -O3 build of the same reference templates (full-size cases)
    args = [a for a in args if a != "--fast"]
    ref = po.Lib(os.path.join(HERE, "_ref", "libsphexa_ref_fast.so")) if fast else po.load_ref()
    if ref is None:
        raise SystemExit("oracle/_ref/libsphexa_ref.so missing: run `make -C oracle` where /root/reference exists")
    names = args or [c for c in tj.CASES if not c.endswith(("300", "400"))]  # the full-size ones: by name
    for n in names:
        run_case(ref, n)


if __name__ == "__main__":
    main()
