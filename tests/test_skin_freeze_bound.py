"""The argument behind frozen clusters (sph-exa_amd/csrc/sx_skin.hpp, SkinArgs::frz; sx_skin.hip step 1b), restated
on the CPU in float64.  A walk leaves, per target, g = min((min |t| - tol) / (R + 2h), R - 2h) with t = |r|^2 - 4h^2
over the target's skin entries (here tol = 0: exact arithmetic); a later step whose targets satisfy both the skin's
validity 2h + d_i + A <= R and the freeze condition (d_i + A) - (d_i + A)_ref + 2 |h - h_ref| < g keeps every hit and
every miss -- also of particles that were outside the skin at the build.  Random and adversarial moves (the entry
nearest to the sphere pushed straight across it by the whole allowance) over Sedov-like lattices and random clouds."""
import numpy as np
import pytest


def _margin(dist, h, R):
    """g of one target: a lower bound of every skin entry's distance to the 2h sphere"""
    t = np.abs(dist**2 - 4.0 * h * h)
    return min(np.min(t) / (R + 2.0 * h), R - 2.0 * h) if dist.size else R - 2.0 * h


def _hits(x, i, h):
    d = np.linalg.norm(x - x[i], axis=1)
    d[i] = np.inf
    return d < 2.0 * h


def _cloud(rng, kind):
    if kind == "lattice":
        g = np.arange(-6, 7, dtype=np.float64)
        x = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
        return x + rng.uniform(-1e-3, 1e-3, x.shape)  # the lattice's shells, slightly broken ties
    return rng.uniform(-6.0, 6.0, (4000, 3))


@pytest.mark.parametrize("kind", ["lattice", "cloud"])
def test_frozen_hits_unchanged(kind):
    rng = np.random.default_rng(7 if kind == "lattice" else 11)
    x0 = _cloud(rng, kind)
    i = int(np.argmin(np.linalg.norm(x0, axis=1)))  # the target: the particle nearest the centre
    checked = adversarial = 0
    for trial in range(600):
        s = rng.choice([0.02, 0.05, 0.08])
        h_b = rng.uniform(1.35, 1.6) if kind == "lattice" else rng.uniform(1.0, 1.6)  # 2h around 2.8 .. 3.2 spacings
        R = 2.0 * h_b * (1.0 + s)
        dist0 = np.linalg.norm(x0 - x0[i], axis=1)
        skin = (dist0 < R) & (np.arange(len(x0)) != i)
        # the reference walk: at the build, or after an earlier drift (d_ref, A_ref) within the skin
        d_ref = rng.uniform(0.0, 0.2) * (R - 2.0 * h_b)
        A_ref = rng.uniform(0.0, 0.3) * (R - 2.0 * h_b - d_ref)
        h_ref = h_b * rng.uniform(0.99, 1.01)
        if 2.0 * h_ref + d_ref + A_ref > R:
            continue
        # positions at the reference: every particle moved by at most A_ref, the target by d_ref (relative motion)
        x_ref = x0 + rng.normal(size=x0.shape) * (A_ref / 3.0 / np.sqrt(3.0))
        x_ref = x0 + np.clip(x_ref - x0, -A_ref / np.sqrt(3.0), A_ref / np.sqrt(3.0))
        v = rng.normal(size=3)
        x_ref[i] = x0[i] + v / np.linalg.norm(v) * d_ref * rng.uniform()
        g = _margin(np.linalg.norm(x_ref[skin] - x_ref[i], axis=1), h_ref, R)
        if g <= 0.0:
            continue
        K = g + d_ref + A_ref
        # this step: a further move within the freeze condition and the skin's validity
        budget = (K - d_ref - A_ref) * rng.uniform(0.0, 0.999)
        share = rng.uniform(0.0, 1.0, 3)
        share /= share.sum()
        dd, dA, dh = budget * share[0], budget * share[1], budget * share[2] / 2.0
        h_new = h_ref + rng.choice([-1.0, 1.0]) * dh
        if 2.0 * h_new + d_ref + dd + A_ref + dA > R:
            continue
        x_new = x_ref.copy()
        move = rng.normal(size=x0.shape)
        move /= np.linalg.norm(move, axis=1, keepdims=True)
        x_new += move * rng.uniform(0.0, dA, (len(x0), 1))
        if trial % 3 == 0:
            # adversarial: the entry nearest the sphere moves straight across it by the whole allowance
            de = np.linalg.norm(x_ref[skin] - x_ref[i], axis=1)
            k = np.flatnonzero(skin)[int(np.argmin(np.abs(de - 2.0 * h_ref)))]
            u = (x_ref[k] - x_ref[i]) / np.linalg.norm(x_ref[k] - x_ref[i])
            inward = 1.0 if np.linalg.norm(x_ref[k] - x_ref[i]) > 2.0 * h_ref else -1.0
            x_new[k] = x_ref[k] - inward * u * dA
            x_new[i] = x_ref[i] + inward * u * dd
            h_new = h_ref + inward * dh
            adversarial += 1
        else:
            v = rng.normal(size=3)
            x_new[i] = x_ref[i] + v / np.linalg.norm(v) * dd
        assert np.array_equal(_hits(x_new, i, h_new), _hits(x_ref, i, h_ref)), (kind, trial, g, dd, dA, dh)
        checked += 1
    assert checked > 300 and adversarial > 100, (checked, adversarial)


def test_margin_is_needed():
    """without the condition the hits do change: a move of the allowance plus a little takes the nearest entry
    across the sphere (the bound is tight, not vacuous)"""
    rng = np.random.default_rng(3)
    x = _cloud(rng, "lattice")
    i = int(np.argmin(np.linalg.norm(x, axis=1)))
    h, R = 1.45, 2.0 * 1.45 * 1.05
    d = np.linalg.norm(x - x[i], axis=1)
    skin = (d < R) & (np.arange(len(x)) != i)
    g = _margin(d[skin], h, R)
    k = np.flatnonzero(skin)[int(np.argmin(np.abs(d[skin] - 2.0 * h)))]
    u = (x[k] - x[i]) / d[k]
    inward = 1.0 if d[k] > 2.0 * h else -1.0
    x2 = x.copy()
    x2[k] = x[k] - inward * u * (np.abs(d[k] - 2.0 * h) * 1.001 + 1e-9)
    assert g <= np.abs(d[k] - 2.0 * h) + 1e-12
    assert not np.array_equal(_hits(x2, i, h), _hits(x, i, h))
