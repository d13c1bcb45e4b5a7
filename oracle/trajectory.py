"""Whole-run observables for trajectory parity (TEST INFRASTRUCTURE ONLY: the checker, never the product path).

A run of several hundred steps is not comparable particle by particle: two float32 trajectories that differ in
summation order separate like any two runs of a shock problem.  What the reference itself checks over a whole run is
the radial profile against the analytic solution (main/src/analytical_solutions/compare_solutions.py:85-89, CI
references .jenkins/reframe_ci.py:349-359), and the energy budget (main/src/observables/conserved_quantities.hpp).
So a trajectory is summarised here by
  * binned radial profiles of rho, p, |v| and u (mean per spherical shell),
  * the total energy, linear momentum and time of every step,
computed by the same numpy code for the reference's run (oracle/_ref, fixtures under tests/golden/traj_*.npz, made
by oracle/gen_trajectory.py) and for the GPU's run (tests/test_gpu_trajectory.py).

rho and p of the VE propagator are EOS outputs (hydro_ve/eos.hpp:52-72): rho = kx m / xm, p = rho cv T (gamma - 1),
recomputed here from the stored kx, xm, m, temp in float32 exactly as computeEOS_Impl rounds them.
"""
import numpy as np

import pyoracle as po


def eos_rho_p(f, mui=np.float32(10.0), gamma=5.0 / 3.0, std=False):
    """rho = kx*m/xm (float), p = rho * (cv*T*(gamma-1)) (idealGasEOS, sph/eos.hpp:31-40: double since T is double).
    std: the std propagator's own density field (computeDensity, hydro_std/density.hpp:41-60) instead of kx m / xm"""
    if std:
        rho = np.asarray(f["rho"], np.float32)
    else:
        kx = np.asarray(f["kx"], np.float32)
        m = np.asarray(f["m"], np.float32)
        xm = np.asarray(f["xm"], np.float32)
        rho = (kx * m / xm).astype(np.float32)
    cv = np.float64(po.ideal_gas_cv(mui, gamma))
    tmp = cv * np.asarray(f["temp"], np.float64) * (gamma - 1.0)
    return rho, (rho.astype(np.float64) * tmp).astype(np.float32)


def radii(f):
    x, y, z = (np.asarray(f[k], np.float64) for k in ("x", "y", "z"))
    return np.sqrt(x * x + y * y + z * z)


def profiles(f, rmax, nbins, std=False):
    """mean rho, p, |v|, u per radial shell [r_b, r_b+1) of width rmax/nbins; particles beyond rmax are ignored.
    Returns (edges, {name: mean per bin}, count per bin)."""
    r = radii(f)
    rho, p = eos_rho_p(f, std=std)
    v = np.sqrt(sum(np.asarray(f[k], np.float64) ** 2 for k in ("vx", "vy", "vz")))
    u = np.float64(po.ideal_gas_cv()) * np.asarray(f["temp"], np.float64)
    edges = np.linspace(0.0, rmax, nbins + 1)
    b = np.clip(np.searchsorted(edges, r, side="right") - 1, 0, nbins)
    keep = r < rmax
    cnt = np.bincount(b[keep], minlength=nbins)[:nbins].astype(np.float64)
    out = {}
    for name, q in (("rho", rho), ("p", p), ("vel", v), ("u", u)):
        s = np.bincount(b[keep], weights=np.asarray(q, np.float64)[keep], minlength=nbins)[:nbins]
        out[name] = np.where(cnt > 0, s / np.maximum(cnt, 1), 0.0)
    return edges, out, cnt


def profile_l1(got, ref, cnt):
    """particle-weighted relative L1 distance of two binned profiles: sum_b n_b |g_b - r_b| / sum_b n_b |r_b|"""
    g, r = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    den = float(np.sum(cnt * np.abs(r)))
    return float(np.sum(cnt * np.abs(g - r))) / den if den > 0 else 0.0


def analytic_l1(r_sim, y_sim, r_sol, y_sol):
    """computeL1Error (compare_solutions.py:85-89): mean |interp(r_sim; solution) - y_sim| over the particles"""
    order = np.argsort(r_sol)
    ys = np.interp(r_sim, np.asarray(r_sol)[order], np.asarray(y_sol)[order])
    return float(np.sum(np.abs(ys - y_sim)) / len(r_sim))


def energies(f, mui=np.float32(10.0), gamma=5.0 / 3.0):
    """(ekin + eint, |linear momentum|) in float64 (conserved_quantities.hpp:49-101)"""
    m = np.asarray(f["m"], np.float64)
    v = [np.asarray(f[k], np.float64) for k in ("vx", "vy", "vz")]
    ekin = 0.5 * float(np.sum(m * (v[0] ** 2 + v[1] ** 2 + v[2] ** 2)))
    eint = float(np.sum(np.float64(po.ideal_gas_cv(mui, gamma)) * np.asarray(f["temp"], np.float64) * m))
    mom = np.sqrt(sum(float(np.sum(m * vv)) ** 2 for vv in v))
    return ekin + eint, mom


def noh_rho(r, t, gamma=5.0 / 3.0, rho0=1.0, vel0=-1.0, xgeom=3):
    """analytic Noh density (compare_noh.py:49-60, nohShockFront + nohRho, vectorised): behind the shock front
    r2 = (gamma - 1)/2 |vel0| t the density is rho0 ((gamma + 1)/(gamma - 1))^xgeom, ahead of it
    rho0 (1 - vel0 t / r)^(xgeom - 1)"""
    r = np.asarray(r, np.float64)
    r2 = 0.5 * (gamma - 1) * abs(vel0) * t
    with np.errstate(divide="ignore"):
        pre = rho0 * (1.0 - vel0 * t / np.maximum(r, 1e-300)) ** (xgeom - 1)
    return np.where(r > r2, pre, rho0 * ((gamma + 1) / (gamma - 1)) ** xgeom)


# the reference's Noh attributes (noh_init.hpp:46-56): r1 = 0.5, mTotal = 1, rho0 = 1.  compare_noh.py evaluates the
# solution with the rho0 attribute, although mTotal = 1 in a sphere of radius 0.5 is a density of 1/(pi/6) = 1.91;
# both are reported: NOH_RHO0_ATTR (the reference's number) and NOH_RHO0_IC (the IC's own density)
NOH_RHO0_ATTR = 1.0
NOH_RHO0_IC = 1.0 / (4.0 / 3.0 * np.pi * 0.5 ** 3)


def noh_l1(f, t, rho0, std=False):
    """createDensityPlot's L1 (compare_noh.py:141-148): mean |nohRho(r_i, t) - rho_i| over the particles"""
    rho, _ = eos_rho_p(f, std=std)
    return float(np.sum(np.abs(noh_rho(radii(f), t, rho0=rho0) - rho.astype(np.float64))) / rho.size)


def energies_grav(f, egrav, mui=np.float32(10.0), gamma=5.0 / 3.0):
    """ekin + eint + egrav (conserved_quantities.hpp with self-gravity: etot includes the potential energy)"""
    return energies(f, mui, gamma)[0] + egrav


FIELDS = ["x", "y", "z", "vx", "vy", "vz", "temp", "m", "kx", "xm"]
FIELDS_STD = ["x", "y", "z", "vx", "vy", "vz", "temp", "m", "rho"]

# the trajectory cases: (fixture name, IC, side, steps, profile steps, profile radius, bins)
CASES = {
    "sedov": ("traj_sedov50.npz", "sedov", 50, 200, (50, 100, 200), 0.5, 25),
    "noh": ("traj_noh30.npz", "noh", 30, 100, (25, 50, 100), 0.5, 15),
    # the std propagator (HydroProp, std_hydro.hpp:124-184) on the CI's Sedov case: its analytic L1 next to VE's
    "sedov_std": ("traj_sedov50_std.npz", "sedov", 50, 200, (50, 100, 200), 0.5, 25),
    # Evrard with self-gravity (G = 1): the energy budget including egrav of the reference's run
    "evrard": ("traj_evrard30.npz", "evrard", 30, 100, (50, 100), 1.0, 20),
    # BASELINE configs 3 and 5 at full size (14.1M particles each), the reference's run at the configured length
    # (made with the -O3 build of the reference, libsphexa_ref_fast.so: ~1 h each on 8 cores)
    "noh300": ("traj_noh300.npz", "noh", 300, 100, (25, 50, 100), 0.5, 50),
    "evrard300": ("traj_evrard300.npz", "evrard", 300, 100, (50, 100), 1.0, 50),
    # the metric's own workload (BASELINE config 4, Sedov -n 400, 64M particles): the reference's run for 30 steps,
    # long enough that the GPU's skin lists go through a forced full rebuild (max_reuse 24) inside the compared window
    "sedov400": ("traj_sedov400.npz", "sedov", 400, 30, (10, 20, 30), 0.5, 50),
}
# propagator / physics options of a case (pyoracle.default_params keywords; both the reference run and the GPU run)
CASE_PARAMS = {"sedov_std": {"std": True}, "evrard": {"g": 1.0}, "evrard300": {"g": 1.0}}
