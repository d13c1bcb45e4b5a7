"""Known-answer data of the reference's own SPH kernel tests (sph/test/ve.cpp:52-233).

The input file tests/golden/ve_example_data.txt is the reference's data file sph/test/example_data.txt
(99 particles x 31 columns, column order of ve.cpp:75-76). Expected values and tolerances below are the
numbers ve.cpp asserts (T=double); they are data, restated here with their line numbers.
"""
import os

import numpy as np

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ve_example_data.txt")
COLS = ["x", "y", "z", "vx", "vy", "vz", "h", "c", "c11", "c12", "c13", "c22", "c23", "c33", "p", "gradh", "rho0",
        "sumwhrho0", "sumwh", "dvxdx", "dvxdy", "dvxdz", "dvydx", "dvydy", "dvydz", "dvzdx", "dvzdy", "dvzdz",
        "alpha", "u", "divv"]
MPART = 3.781038064465603e26      # ve.cpp:94
DT = 0.3                          # ve.cpp:95 (AV switches)

# (name, expected, abs tolerance) -- ve.cpp line numbers in comments
EXPECTED = {
    "alpha": (0.93941905320351171, 2e-9),          # :119
    "divv": (3.3760353440920682e-2, 2e-9),         # :131
    "curlv": (3.7836647734377962e-2, 2e-9),        # :132
    "c11": (1.9296619855715329e-18, 1e-10),        # :152
    "c12": (-1.7838691836843698e-20, 1e-10),
    "c13": (-1.2892885646884301e-20, 1e-10),
    "c22": (1.9482845913025683e-18, 1e-10),
    "c23": (1.635410357476855e-20, 1e-10),
    "c33": (1.9246939006338132e-18, 1e-10),        # :157
    "ax": (-521261.07791667967, 0.022),            # :211 (no AV cleaning)
    "ay": (-74471.016515749841, 0.064),
    "az": (-1730426.827721074, 0.042),
    "du": (7.1838438980436924e12, 3.1e5),          # :214
    "maxvsignal": (26490876.319252387, 1e-6),      # :215
    "rho": (3.4662283566584293e1, 8e-7),           # :227 VeDefGradh density
    "gradh": (0.98699067585409861, 5e-7),          # :228
    "kx": (1.0042661134076782, 3e-7),              # :229
    "rho0": (34.515038498081417, 7.33e-7),         # :239 XMass
}


def load():
    a = np.loadtxt(PATH)
    assert a.shape == (99, 31)
    return {c: a[:, k].copy() for k, c in enumerate(COLS)}


def sphynx_3d_k(n):
    """sph_kernel_tables.hpp:62-75 (KAT uses this K, ve.cpp:90)."""
    b0, b1, b2, b3 = 2.7012593e-2, 2.0410827e-2, 3.7451957e-3, 4.7013839e-2
    return b0 + b1 * np.sqrt(n) + b2 * n + b3 * np.sqrt(n * n * n)
