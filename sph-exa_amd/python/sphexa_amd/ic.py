"""Initial conditions of the BASELINE configurations other than the device-generated Sedov lattice
(sx_sim_init_sedov): host numpy arrays in the layout sx_sim_set_state takes.

The reference builds Noh and Evrard from a glass block (main/src/init/{noh,evrard}_init.hpp, --glass) that is not
available offline; both use a cell-centred lattice instead, with the reference's field values.
"""
import math

import numpy as np

R_GAS = np.float32(8.317e7)


def ideal_gas_cv(mui=np.float32(10.0), gamma=5.0 / 3.0):
    """idealGasCv<float, double> (sph/eos.hpp:13-18)"""
    return np.float32(np.float64(R_GAS / np.float32(mui)) / (gamma - 1.0))


def _lattice(side, r):
    step = (2.0 * r) / side
    c = -r + 0.5 * step + np.arange(side, dtype=np.float64) * step
    zz, yy, xx = np.meshgrid(c, c, c, indexing="ij")
    return xx.ravel(), yy.ravel(), zz.ravel()


def _fields(n):
    f = {k: np.zeros(n, np.float32) for k in ("h", "m", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha")}
    f["alpha"][:] = np.float32(0.05)  # alphamin
    f["id"] = np.arange(n, dtype=np.uint64)
    return f


def noh(side):
    """Noh implosion (noh_init.hpp:46-100 field values): lattice cut to r <= 0.5, v = -r_hat, x_m1 = v dt0,
    T = 1e-20/cv, dt0 = 1e-4,
    open box.  Returns (arrays, box limits, boundary, dt0)."""
    r = 0.5
    x, y, z = _lattice(side, r)
    rad = np.sqrt(x * x + y * y + z * z)
    keep = rad <= r
    x, y, z, rad = x[keep], y[keep], z[keep], rad[keep]
    n = x.size
    f = _fields(n)
    f["x"], f["y"], f["z"] = x, y, z
    vol = 4.0 / 3.0 * math.pi * r ** 3
    f["h"][:] = np.float32(np.cbrt(3.0 / (4 * math.pi) * 100 * vol / n) * 0.5)
    f["m"][:] = np.float32(1.0 / n)
    inv = np.where(rad > 0, 1.0 / np.maximum(rad, 1e-300), 0.0)
    f["vx"][:], f["vy"][:], f["vz"][:] = -x * inv, -y * inv, -z * inv
    # the integrator's previous displacement x_m1 = v * minDt (noh_init.hpp:96-98): the first positionUpdate takes
    # the velocity from dX_n / dt_m1 (positions.hpp:77-88), so x_m1 = 0 would stop the inflow
    for d in ("x", "y", "z"):
        f[d + "_m1"][:] = (f["v" + d].astype(np.float64) * 1e-4).astype(np.float32)
    f["temp"] = np.full(n, 1e-20 / np.float64(ideal_gas_cv()))
    lo, hi = -0.5 - 1e-3, 0.5 + 1e-3
    return f, [lo, hi, lo, hi, lo, hi], [0, 0, 0], 1e-4


def evrard(side):
    """Evrard collapse (evrard_init.hpp:50-108 field values): lattice in [-1,1]^3 cut to 0 < r <= 1 and contracted by
    sqrt(r) to a 1/r density profile; m = 1/N, u0 = 0.05, h from the 1/r concentration, G = 1, dt0 = 1e-4; open box
    [-1.25, 1.25]^3 (the reference re-fits open boxes to the particles every sync)."""
    r = 1.0
    x, y, z = _lattice(side, r)
    rad0 = np.sqrt(x * x + y * y + z * z)
    keep = (rad0 <= r) & (rad0 > 1e-9 * r)
    x, y, z, rad0 = x[keep], y[keep], z[keep], rad0[keep]
    con = np.sqrt(rad0)
    x, y, z = x * con, y * con, z * con
    n = x.size
    f = _fields(n)
    f["x"], f["y"], f["z"] = x, y, z
    f["m"][:] = np.float32(1.0 / n)
    f["temp"] = np.full(n, 0.05 / np.float64(ideal_gas_cv()))
    c0 = 2.0 / 3.0 * n / (4.0 * math.pi / 3.0 * r ** 3)
    radius = np.sqrt(x * x + y * y + z * z)
    f["h"][:] = (np.cbrt(3.0 / (4.0 * math.pi) * 100 / (c0 / np.maximum(radius, 1e-12))) * 0.5).astype(np.float32)
    lo, hi = -1.25 * r, 1.25 * r
    return f, [lo, hi, lo, hi, lo, hi], [0, 0, 0], 1e-4
