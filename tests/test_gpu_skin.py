"""Skin-list reuse of the neighbor search (sph-exa_amd/csrc/sx_skin.hpp) against a fresh search and the oracle.

Between full builds a one-rank step filters the last build's lists within 2h(1 + s) instead of syncing and
searching.  What must not change is the step's neighbor search result (cstone::findNeighbors + findNeighborsSph,
findneighbors.hpp:95-188, find_neighbors.hpp:10-44):
  * the neighbor SETS, nc and h of a filtered step equal those of a fresh sync + search of the same state (a second
    Sim with the skin off, handed the state before every step), particle by particle by id, over runs that rebuild
    stale clusters (Sedov's blast, Noh's infall, an Evrard-like collapse IC) and run the exact-search fallback;
  * every filtered step checked per particle against the CPU oracle (gpu_util.shadow_steps: nc and h exact, rates
    within the fast-variant tolerance);
  * the skin does its job: most steps are served by the filter on a quiescent state.
"""
import numpy as np
import pytest

import gpu_util as gutil
import pyoracle as po
import sphexa_amd as sx

pytestmark = pytest.mark.gpu

STATE = ["x", "y", "z", "h", "m", "temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha", "id"]


def _ic(kind, side):
    if kind == "sedov":
        return po.sedov_state(side)
    if kind == "noh":
        return po.noh_state(side)
    return po.evrard_state(side)


@pytest.fixture(scope="module")
def ctx():
    c = sx.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("kind,side,steps,factor", [("sedov", 24, 14, 0.08), ("noh", 24, 12, 0.08),
                                                    ("evrard", 22, 10, 0.08), ("sedov", 20, 10, 0.02),
                                                    ("noh", 20, 12, 0.004), ("noh", 24, 6, 0.25),
                                                    ("sedov", 20, 6, 0.25)])
def test_skin_sets_equal_fresh_search(ctx, kind, side, steps, factor):
    """each filtered step's neighbor sets, nc and h equal a fresh search's from the same state"""
    st, obox = _ic(kind, side)
    box = gutil.box_to_sx(obox)
    a = sx.Sim(ctx, st.n, box)
    a.set_skin(factor, 24)
    b = sx.Sim(ctx, st.n, box)
    b.set_skin(0.0, 1)
    a.set_state(st.arrays, st.minDt, st.minDt_m1)
    try:
        for s in range(steps):
            g = a.get(STATE)
            sc = a.scalars()
            b.set_state(g, sc["minDt"], sc["minDt_m1"])
            a.step()
            b.step()
            ga, gb = a.get(["id", "nc", "h"]), b.get(["id", "nc", "h"])
            oa, ob = np.argsort(ga["id"]), np.argsort(gb["id"])
            bad_nc = np.nonzero(ga["nc"][oa] != gb["nc"][ob])[0]
            assert bad_nc.size == 0, (kind, s, bad_nc.size, ga["nc"][oa][bad_nc[:8]], gb["nc"][ob][bad_nc[:8]],
                                      np.sort(oa[bad_nc] // 256)[:16], a.skin_stats())
            assert np.array_equal(ga["h"][oa], gb["h"][ob]), (kind, s)
            na, nb = a.neighbor_sets(), b.neighbor_sets()
            bad = [k for k in na if not np.array_equal(na[k], nb[k])]
            assert not bad, (kind, s, len(bad), bad[:3])
        ks = a.skin_stats()
        print(kind, side, factor, ks)
        assert ks["reuse_steps"] > 0, ks
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("kind,side,steps,factor", [("sedov", 16, 6, 0.08), ("noh", 24, 6, 0.3)])
def test_skin_steps_vs_oracle(ctx, kind, side, steps, factor):
    """filtered steps, each checked per particle against an oracle step from the same state (Noh's infall outruns a
    thin skin at this resolution: a wide one keeps it for several steps)"""
    ora = po.load_oracle()
    st, obox = _ic(kind, side)
    sim = sx.Sim(ctx, st.n, gutil.box_to_sx(obox))
    sim.set_skin(factor, 24)
    sim.set_state(st.arrays, st.minDt, st.minDt_m1)
    try:
        gutil.shadow_steps(ctx, ora, sim, obox, steps, ora.params(), ["x", "y", "z", "vx", "vy", "vz", "temp", "du",
                                                                     "ax", "ay", "az", "alpha", "xm", "kx"])
        ks = sim.skin_stats()
        print(kind, factor, ks)
        assert ks["reuse_steps"] >= steps // 2, ks
    finally:
        sim.close()


def test_skin_quiescent_lattice_reuses(ctx):
    """a lattice at rest (Sedov outside the blast): after the first full build every step is served by the filter,
    without stale clusters, until maxReuse forces the next full build"""
    st, obox = po.sedov_state(20)
    st.temp[:] = st.temp.min()  # no blast: nothing moves
    sim = sx.Sim(ctx, st.n, gutil.box_to_sx(obox))
    sim.set_skin(0.08, 5)
    sim.set_state(st.arrays, st.minDt, st.minDt_m1)
    try:
        for _ in range(11):
            sim.step()
            assert sim.stats()["numFailed"] == 0
        ks = sim.skin_stats()
        assert ks["builds"] == 2 and ks["reuse_steps"] == 9 and ks["stale_clusters"] == 0, ks
        # nothing moves: reuse steps whose hits equal the last step's keep the exact lists in place
        assert ks["kept_clusters"] > 0, ks
    finally:
        sim.close()


def _sorted_rows(sim):
    """the last step's neighbor lists as one array: a row per particle in id order, its neighbor ids sorted and padded
    with 2^32 - 1 (the vectorized form of Sim.neighbor_sets, for runs of a few 100k particles)"""
    n, ngmax = sim.size(), int(sim.params.ngmax)
    buf = sim.ctx.alloc(n * ngmax, np.uint32)
    try:
        sim.ctx.check(sim.L.sx_sim_export_neighbors(sim.h, buf.ptr), "export_neighbors")
        rows = buf.get()[: n * ngmax].reshape(n, ngmax)
    finally:
        sim.ctx.free(buf)
    g = sim.get(["id", "nc"])
    ids = g["id"].astype(np.uint32)
    cnt = np.minimum(g["nc"].astype(np.int64) - 1, ngmax)
    out = np.where(np.arange(ngmax)[None, :] < cnt[:, None], ids[rows], np.uint32(0xFFFFFFFF))
    out.sort(axis=1)
    return out[np.argsort(ids)]


def test_skin_early_exact_search_equals_fresh_search(ctx):
    """Noh's infall at 80^3 (268k particles): from step 6 on some clusters are stale on the step after their rebuild
    and take the exact search on the auxiliary stream, concurrently with the rebuild + filter of the other stale
    clusters (sx_sim.cpp skinSearch).  Every step's nc and h equal a fresh sync + search's; on each step with such
    clusters the neighbor sets of all particles do too"""
    st, obox = po.noh_state(80)
    box = gutil.box_to_sx(obox)
    a = sx.Sim(ctx, st.n, box)
    a.set_skin(0.05, 24)
    b = sx.Sim(ctx, st.n, box)
    b.set_skin(0.0, 1)
    a.set_state(st.arrays, st.minDt, st.minDt_m1)
    checked = 0
    try:
        early0 = 0
        for s in range(16):
            g = a.get(STATE)
            sc = a.scalars()
            b.set_state(g, sc["minDt"], sc["minDt_m1"])
            a.step()
            b.step()
            ga, gb = a.get(["id", "nc", "h"]), b.get(["id", "nc", "h"])
            oa, ob = np.argsort(ga["id"]), np.argsort(gb["id"])
            assert np.array_equal(ga["nc"][oa], gb["nc"][ob]), s
            assert np.array_equal(ga["h"][oa], gb["h"][ob]), s
            ks = a.skin_stats()
            if ks["early_exact"] > early0:
                assert np.array_equal(_sorted_rows(a), _sorted_rows(b)), s
                checked += 1
            early0 = ks["early_exact"]
        print("noh 80", checked, "steps with early exact searches", a.skin_stats())
        assert checked >= 2, a.skin_stats()
    finally:
        a.close()
        b.close()


def test_skin_frozen_steps_equal_fresh_search(ctx):
    """a lattice at rest: its h follows nc from shell to shell, so the hit sets change together on some steps and stand
    still on others; on those the filter proves from the last walk's margins that no entry can have crossed its 2h
    sphere and keeps the exact lists without walking the skin lists (frozen clusters, sx_skin.hpp SkinArgs::frz).
    Every step's nc, h and neighbor sets equal a fresh sync + search of the same state, and xm (the frozen path's
    XMass over the exact lists) agrees with the fresh step's to float rounding"""
    st, obox = po.sedov_state(20)
    st.temp[:] = st.temp.min()
    box = gutil.box_to_sx(obox)
    a = sx.Sim(ctx, st.n, box)
    a.set_skin(0.05, 24)
    b = sx.Sim(ctx, st.n, box)
    b.set_skin(0.0, 1)
    a.set_state(st.arrays, st.minDt, st.minDt_m1)
    try:
        for s in range(12):
            g = a.get(STATE)
            sc = a.scalars()
            b.set_state(g, sc["minDt"], sc["minDt_m1"])
            a.step()
            b.step()
            ga, gb = a.get(["id", "nc", "h", "xm"]), b.get(["id", "nc", "h", "xm"])
            oa, ob = np.argsort(ga["id"]), np.argsort(gb["id"])
            assert np.array_equal(ga["nc"][oa], gb["nc"][ob]) and np.array_equal(ga["h"][oa], gb["h"][ob]), s
            np.testing.assert_allclose(ga["xm"][oa], gb["xm"][ob], rtol=2e-6, err_msg=str(s))
            na, nb = a.neighbor_sets(), b.neighbor_sets()
            assert all(np.array_equal(na[k], nb[k]) for k in na), s
        ks = a.skin_stats()
        print(ks)
        assert ks["frozen_clusters"] > 0 and ks["kept_clusters"] >= ks["frozen_clusters"], ks
    finally:
        a.close()
        b.close()


def test_skin_with_gravity_matches_fresh_tree(ctx):
    """self-gravity on filter-served steps (sx_sim.cpp: the last sync's tree, multipoles from the current positions,
    MAC boxes refreshed to hold each node's cell and its particles): each step's accelerations and potential energy
    against a fresh sync + search + tree of the same state, within the Barnes-Hut approximation (theta = 0.5: the two
    trees accept different nodes, so the fields may differ at the level of the multipole truncation, not bit for bit;
    measured: 1.2e-6 of the rms acceleration at worst)"""
    st, obox = po.evrard_state(22)
    box = gutil.box_to_sx(obox)
    prm = sx.default_params(g=1.0)
    a = sx.Sim(ctx, st.n, box, params=prm)
    a.set_skin(0.08, 24)
    b = sx.Sim(ctx, st.n, box, params=prm)
    b.set_skin(0.0, 1)
    a.set_state(st.arrays, st.minDt, st.minDt_m1)
    worst = 0.0
    try:
        for s in range(8):
            g = a.get(STATE)
            sc = a.scalars()
            b.set_state(g, sc["minDt"], sc["minDt_m1"])
            a.step()
            b.step()
            ga, gb = a.get(["id", "ax", "ay", "az"]), b.get(["id", "ax", "ay", "az"])
            oa, ob = np.argsort(ga["id"]), np.argsort(gb["id"])
            acc_a = np.stack([ga[k][oa] for k in ("ax", "ay", "az")]).astype(np.float64)
            acc_b = np.stack([gb[k][ob] for k in ("ax", "ay", "az")]).astype(np.float64)
            rms = np.sqrt(np.mean(np.sum(acc_b * acc_b, axis=0)))
            err = np.sqrt(np.sum((acc_a - acc_b) ** 2, axis=0)) / rms
            worst = max(worst, float(err.max()))
            assert err.max() < 1e-4 and np.median(err) < 1e-5, (s, float(err.max()), float(np.median(err)))
            ea, eb = a.conserved()["egrav"], b.conserved()["egrav"]
            assert abs(ea / eb - 1) < 1e-5, (s, ea, eb)
        ks = a.skin_stats()
        print("gravity on filter-served steps: worst |da| / rms(a)", f"{worst:.2e}", ks)
        assert ks["reuse_steps"] >= 4, ks
    finally:
        a.close()
        b.close()

