"""Generate the golden fixtures under tests/golden/ from the reference's own CPU path (oracle/_ref).

TEST INFRASTRUCTURE ONLY. Run in the build container, where /root/reference exists:
    make -C oracle && python oracle/gen_golden.py
The fixtures are data (inputs + the reference's outputs); they travel with the repo so the parity tests
run on the GPU box, which has no /root/reference.

Fixtures
  sedov10.npz    Sedov lattice n=10 (1000 particles): IC, and full state after steps 1..3 (ref_step)
  noh10.npz      Noh lattice-sphere n=12 (open box): IC and state after steps 1..3
  kernels.npz    one Sedov n=12 state after 2 steps + the reference neighbor list (CPU layout) and every
                 per-kernel output computed by the reference *Impl loops on it
  tree_rand.npz  2000 seeded random points: Hilbert keys, cornerstone leaves (bucket 16), linked octree
                 arrays, node centers/sizes, neighbor lists + counts with and without h iteration
  evrard14.npz   Evrard substitute n=14 (1472 particles, key-sorted): gravity alone (expansion centers + MAC
                 radii, quadrupoles, accelerations, egrav; G = 1, theta = 0.5) and 2 full VE steps with gravity

  std_sedov10.npz, std_noh12.npz  std propagator (HydroProp, std_hydro.hpp:124-184): IC and states after 3 steps
  std_kernels.npz  Sedov n=12 after 2 std steps + neighbor list and the outputs of density, EOS_HydroStd, IAD,
                   momentumEnergySTD (the reference's std *Impl loops)

    python oracle/gen_golden.py [--only gravity|std]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def snapshot(st, prefix):
    d = {f"{prefix}{k}": v.copy() for k, v in st.arrays.items()}
    d[f"{prefix}scalars"] = np.array([st.minDt, st.minDt_m1, st.ttot, st.minDtCourant, st.minDtRho])
    return d


def box_arr(box):
    return np.array(list(box.lim) + list(box.bnd), dtype=np.float64)


def run_steps(ref, st, box, nsteps, name):
    out = {"box": box_arr(box)}
    out.update(snapshot(st, "s0_"))
    for s in range(1, nsteps + 1):
        ref.step(st, box)
        out.update(snapshot(st, f"s{s}_"))
    np.savez_compressed(os.path.join(OUT, name), **out)


def gravity_fixture(ref):
    st, box = po.evrard_state(14)
    keys = ref.sfc_keys(st, box).copy()
    order = np.argsort(keys, kind="stable")
    for k in po.CONSERVED:
        st.arrays[k][:] = st.arrays[k][order]
    st.keys[:] = keys[order]
    p = ref.params(g=1.0, theta=0.5)
    out = {"box": box_arr(box)}
    out.update(snapshot(st, "s0_"))
    g = st.copy()
    egrav, cen, mp = ref.gravity(g, box, p)
    out.update({"grav_centers": cen, "grav_multipoles": mp, "grav_ax": g.ax.copy(), "grav_ay": g.ay.copy(),
                "grav_az": g.az.copy(), "grav_egrav": np.array([egrav])})
    for s in range(1, 3):
        ref.step(st, box, params=p)
        out.update(snapshot(st, f"s{s}_"))
        out[f"s{s}_egrav"] = np.array([st.egrav])
    np.savez_compressed(os.path.join(OUT, "evrard14.npz"), **out)


def std_fixture(ref):
    """std propagator (HydroProp): 3 steps of Sedov n=10 and Noh n=12, and each std kernel on a Sedov n=12 state"""
    p = ref.params(std=True)
    for ic, side, name in [(po.sedov_state, 10, "sedov"), (po.noh_state, 12, "noh")]:
        st, box = ic(side)
        out = {"box": box_arr(box)}
        out.update(snapshot(st, "s0_"))
        for s in range(1, 4):
            ref.step(st, box, params=p)
            out.update(snapshot(st, f"s{s}_"))
        out_name = f"std_{name}{side}.npz"
        np.savez_compressed(os.path.join(OUT, out_name), **out)
    st, box = po.sedov_state(12)
    ref.step(st, box, params=p)
    ref.step(st, box, params=p)
    ref.sfc_keys(st, box)
    order = np.argsort(st.keys, kind="stable")
    for k in po.CONSERVED + ["keys"]:
        st.arrays[k][:] = st.arrays[k][order]
    pre = st.copy()
    nbr, nc = ref.find_neighbors(st, box, iterate_h=True)
    st.nc[:] = nc
    out = {"box": box_arr(box), "nbr": nbr, "nc": nc}
    out.update(snapshot(pre, "in_"))
    ref.density(st, box, nbr, params=p)
    out["rho"] = st.rho.copy()
    ref.eos_std(st, params=p)
    out["p"], out["c"] = st.p.copy(), st.c.copy()
    ref.iad_std(st, box, nbr, params=p)
    for k in ["c11", "c12", "c13", "c22", "c23", "c33"]:
        out[k] = st.arrays[k].copy()
    out["minDtCourant"] = np.array([ref.momentum_energy_std(st, box, nbr, params=p)])
    for k in ["du", "ax", "ay", "az"]:
        out[k] = st.arrays[k].copy()
    np.savez_compressed(os.path.join(OUT, "std_kernels.npz"), **out)


def main():
    ref = po.load_ref()
    if ref is None:
        raise SystemExit("oracle/_ref/libsphexa_ref.so missing: run `make -C oracle` where /root/reference exists")
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if only in (None, "std"):
        std_fixture(ref)
    if only in (None, "gravity"):
        gravity_fixture(ref)
    if only is not None:
        return

    st, box = po.sedov_state(10)
    run_steps(ref, st, box, 3, "sedov10.npz")

    st, box = po.noh_state(12)
    run_steps(ref, st, box, 3, "noh10.npz")

    # per-kernel fixture: state after two steps, then each kernel on the reference's own neighbor list
    st, box = po.sedov_state(12)
    ref.step(st, box)
    ref.step(st, box)
    ref.sfc_keys(st, box)
    order = np.argsort(st.keys, kind="stable")
    for k in po.CONSERVED + ["keys"]:
        st.arrays[k][:] = st.arrays[k][order]
    pre = st.copy()
    nbr, nc = ref.find_neighbors(st, box, iterate_h=True)
    st.nc[:] = nc
    out = {"box": box_arr(box), "nbr": nbr, "nc": nc, "h_after_iter": st.h.copy()}
    out.update(snapshot(pre, "in_"))
    ref.xmass(st, box, nbr)
    out["xm"] = st.xm.copy()
    ref.ve_def_gradh(st, box, nbr)
    out["kx"], out["gradh"] = st.kx.copy(), st.gradh.copy()
    ref.eos(st)
    out["prho"], out["c"] = st.prho.copy(), st.c.copy()
    ref.iad_divv_curlv(st, box, nbr)
    for k in ["c11", "c12", "c13", "c22", "c23", "c33", "divv", "curlv"]:
        out[k] = st.arrays[k].copy()
    ref.av_switches(st, box, nbr)
    out["alpha"] = st.alpha.copy()
    out["minDtCourant"] = np.array([ref.momentum_energy(st, box, nbr)])
    for k in ["du", "ax", "ay", "az"]:
        out[k] = st.arrays[k].copy()
    np.savez_compressed(os.path.join(OUT, "kernels.npz"), **out)

    # tree + neighbor search on seeded random points (cstone findneighbors test style, random.hpp seed 42)
    rng = np.random.default_rng(42)
    n = 2000
    st = po.HostState(n)
    st.x[:] = rng.uniform(-0.5, 0.5, n)
    st.y[:] = rng.uniform(-0.5, 0.5, n)
    st.z[:] = np.clip(rng.normal(0.0, 0.15, n), -0.5, 0.4999)
    box = po.make_box(-0.5, 0.5, True)
    keys = ref.sfc_keys(st, box).copy()
    order = np.argsort(keys, kind="stable")
    for k in ["x", "y", "z"]:
        st.arrays[k][:] = st.arrays[k][order]
    st.keys[:] = keys[order]
    tree = ref.octree(st.keys, 16)
    cen, siz = ref.node_centers(tree["prefixes"], box)
    st.h[:] = np.float32(0.06)
    out = {"x": st.x.copy(), "y": st.y.copy(), "z": st.z.copy(), "keys_unsorted": keys, "order": order,
           "box": box_arr(box), "centers": cen, "sizes": siz}
    out.update({f"tree_{k}": v for k, v in tree.items()})
    nbr, nc = ref.find_neighbors(st, box, bucket=16, iterate_h=False)
    out["nbr_noiter"], out["nc_noiter"] = nbr, nc
    h0 = st.h.copy()
    nbr, nc = ref.find_neighbors(st, box, bucket=16, iterate_h=True)
    out["nbr_iter"], out["nc_iter"], out["h_iter"], out["h0"] = nbr, nc, st.h.copy(), h0
    np.savez_compressed(os.path.join(OUT, "tree_rand.npz"), **out)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
