"""Phase split of the neighbor search from a probe build (SX_NS_PROBE=1, e.g. sph-exa_amd/lib_probe):
    SPHEXA_AMD_LIB=$PWD/sph-exa_amd/lib_probe/libsphexa_hip.so python scripts/search_probe.py [side] [steps]
Runs a Sedov state for `steps` steps and prints the kcycles per wave of each phase of the compact search kernel
(the device counters g_nsProbe, read through the probe build's sx_debug_ns_probe_* functions)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, "sph-exa_amd/python")
import sphexa_amd as sx  # noqa: E402

PHASES = ["regions", "tree walk", "scan+reach", "stream+test", "h-vote", "union", "rewrite+expand", "tail"]

side = int(sys.argv[1]) if len(sys.argv) > 1 else 400
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lib = ctypes.CDLL(os.environ["SPHEXA_AMD_LIB"])
FNS = {"compact": lib.sx_debug_ns_probe_small, "large": lib.sx_debug_ns_probe_large}
for f in FNS.values():
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]


ctx = sx.Context(0)
n = side ** 3
sim = sx.Sim(ctx, n, sx.make_box([-0.5, 0.5, -0.5, 0.5, -0.5, 0.5], [1, 1, 1]))
sim.init_sedov(side)
sim.step()  # warm-up (includes the first h iteration from the initial guess)
for f in FNS.values():
    z = np.zeros(16, np.uint64)
    assert f(z.ctypes.data, 1) == 0
for s in range(steps):
    sim.step()
for name, f in FNS.items():
    v = np.zeros(16, np.uint64)
    assert f(v.ctypes.data, 0) == 0
    waves = int(v[8]) or 1
    tot = float(v[:8].sum()) / waves / 1e3
    print(f"{name}: {steps} steps, {waves} waves (persistent), kcycles per persistent wave:")
    for k, p in enumerate(PHASES):
        print(f"  {p:15s} {float(v[k]) / waves / 1e3:10.1f}  ({float(v[k]) / max(1.0, float(v[:8].sum())):.3f})")
    print(f"  {'total':15s} {tot:10.1f}")
    for k, c in enumerate(["blocks", "streamed", "staged", "chunks", "exact chunks", "test kcycles"]):
        print(f"  per wave: {c:13s} {float(v[9 + k]) / waves / (1e3 if k == 5 else 1):10.1f}")
sim.close()
ctx.close()
