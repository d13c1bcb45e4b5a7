"""The fast gravity traversal's float MAC prefilter (sx_gravity.hip, gravityTraverseKernel<FAST>: `violates`) decides
in float only outside an error bound and leaves the rest to the double test of the reference (`evaluateMacs`-style
box distance vs mac^2, traversal_cpu.hpp).  This restates the float evaluation and its bound in numpy (same
operation order, float32 throughout) and checks, on cases concentrated at the MAC boundary (mac^2 within 1e-9 .. 1e-3
relative of the box distance), that every decision the float path takes equals the double decision."""
import numpy as np

f32 = np.float32


def _decide(tc, ts, c, mac2):
    d = np.abs(tc - c) - ts
    d = 0.5 * (d + np.abs(d))
    exact = (d[:, 0] ** 2 + (d[:, 1] ** 2 + d[:, 2] ** 2)) < mac2
    tcf, tsf, cf, m2f = tc.astype(f32), ts.astype(f32), c.astype(f32), mac2.astype(f32)
    df = np.abs(tcf - cf) - tsf
    df = f32(0.5) * (df + np.abs(df))
    D = df[:, 0] * df[:, 0] + (df[:, 1] * df[:, 1] + df[:, 2] * df[:, 2])
    E = f32(2.0 ** -22) * (np.abs(tcf).sum(1) + np.abs(cf).sum(1) + tsf.sum(1))
    tol = f32(2.5) * np.sqrt(m2f) * E + f32(6) * E * E + f32(2.0 ** -20) * m2f
    fast = D < m2f - tol
    amb = ~fast & ~(D > m2f + tol)
    return exact, fast, amb


def test_float_mac_prefilter_never_contradicts_double():
    rng = np.random.default_rng(7)
    n = 1_000_000
    tc = rng.uniform(-1.25, 1.25, (n, 3))  # the Evrard box
    ts = rng.uniform(1e-5, 0.05, (n, 3))
    c = tc + rng.normal(0, 0.2, (n, 3))
    d = np.abs(tc - c) - ts
    d = 0.5 * (d + np.abs(d))
    D = d[:, 0] ** 2 + (d[:, 1] ** 2 + d[:, 2] ** 2)
    mac2 = np.where(D > 0, D * (1 + rng.choice([-1, 1], n) * 10 ** rng.uniform(-9, -3, n)), 1e-8)
    exact, fast, amb = _decide(tc, ts, c, mac2)
    decided = ~amb
    assert np.array_equal(fast[decided], exact[decided])
    assert decided.sum() > 0.2 * n  # the bound is not vacuous even this close to the boundary


def test_float_mac_prefilter_decides_typical_nodes():
    """away from the boundary (typical traversal tests) the float path decides almost everything"""
    rng = np.random.default_rng(8)
    n = 200_000
    tc = rng.uniform(-1.0, 1.0, (n, 3))
    ts = rng.uniform(1e-4, 0.01, (n, 3))
    c = tc + rng.normal(0, 0.1, (n, 3))
    mac2 = rng.uniform(1e-6, 0.05, n)
    exact, fast, amb = _decide(tc, ts, c, mac2)
    assert amb.mean() < 1e-3
    assert np.array_equal(fast[~amb], exact[~amb])
