"""Reference field of periodic self-gravity for the multi-rank tests (test infrastructure, CPU, float64): the walk's
part as a softened direct sum over the box and its 26 images (P2P of kernel.hpp:514-535, R^2 >= (h_i + h_j)^2, the
target's own image in the central box left out -- computeGravity with numShells = 1, gravity_wrapper.hpp:135-140),
plus the Ewald correction of the oracle restatement (oracle/ewald.py, pinned bit for bit to the reference's
computeGravityEwald by tests/test_ewald_oracle.py) from the root expansion of all particles."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import ewald as ew  # noqa: E402
import gen_ewald as ge  # noqa: E402


def direct_images(x, y, z, m, h, L, G=1.0, chunk=256):
    """(acc (n, 3), phi (n,)) of the 27-image softened direct sum"""
    n = x.size
    P = np.stack([x, y, z], 1).astype(np.float64)
    mj = m.astype(np.float64)
    hj = h.astype(np.float64)
    acc = np.zeros((n, 3))
    phi = np.zeros(n)
    for i0 in range(0, n, chunk):
        i1 = min(n, i0 + chunk)
        hij = hj[i0:i1, None] + hj[None, :]
        for ix in (-1, 0, 1):
            for iy in (-1, 0, 1):
                for iz in (-1, 0, 1):
                    d = P[None, :, :] + np.array([ix, iy, iz], np.float64) * L - P[i0:i1, None, :]
                    R2 = np.sum(d * d, axis=2)
                    R2e = np.maximum(R2, hij * hij)
                    w = mj[None, :] / (R2e * np.sqrt(R2e))
                    if ix == iy == iz == 0:
                        w[np.arange(i1 - i0), np.arange(i0, i1)] = 0.0
                    acc[i0:i1] += np.einsum("ij,ijk->ik", w, d)
                    phi[i0:i1] -= np.sum(w * R2, axis=1)
    return G * acc, phi


def periodic_field(x, y, z, m, h, L, G=1.0):
    """(acc (n, 3), egrav) of the image walk + Ewald correction, exact to the BH error the GPU's walk adds"""
    acc, phi = direct_images(x, y, z, m, h, L, G)
    M, c = ge.root_moments(x, y, z, m)
    ex = np.zeros(x.size, np.float32)
    ey = np.zeros(x.size, np.float32)
    ez = np.zeros(x.size, np.float32)
    e_ewald = ew.gravity_ewald(x, y, z, m, M, c, L, G, ex, ey, ez)
    acc = acc + np.stack([ex, ey, ez], 1).astype(np.float64)
    egrav = 0.5 * G * float(np.sum(m.astype(np.float64) * phi)) + e_ewald
    return acc, egrav
