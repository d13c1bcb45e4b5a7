"""Per-kernel register / scratch / LDS / occupancy table of the library's HIP sources (compile-time remarks).

  python scripts/kernel_resources.py [source-substring ...]

Compiles each source of sph-exa_amd/Makefile's rules device-only with -Rpass-analysis=kernel-resource-usage and
prints one line per kernel; spills and scratch are what to look for first.
"""
import re
import subprocess
import sys
import os

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sph-exa_amd")
BASE = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-I../include",
        "-Rpass-analysis=kernel-resource-usage", "--offload-device-only", "-c", "-o", "/dev/null"]
SOURCES = {
    "sx_neighbors (large)": ("csrc/sx_neighbors.hip", ["-ffp-contract=off"]),
    "sx_neighbors (small)": ("csrc/sx_neighbors.hip", ["-ffp-contract=off", "-DSX_NS_SMALL", "-DSX_NS_CCAP=1024",
                                                       "-DSX_NS_CAND_LOG2=14", "-DSX_NS_BATCH=24", "-DSX_NS_WAVES_PER_EU=4"]),
    "sx_hydro_cluster": ("csrc/sx_hydro_cluster.hip", ["-ffp-contract=fast", "-fno-slp-vectorize",
                                                       "-fgpu-flush-denormals-to-zero"]),
    "sx_hydro (fast)": ("csrc/sx_hydro.hip", ["-ffp-contract=fast", "-DSX_VARIANT=fast"]),
    "sx_gravity": ("csrc/sx_gravity.hip", ["-ffp-contract=off", "-fno-slp-vectorize"]),
    "sx_tree": ("csrc/sx_tree.hip", ["-ffp-contract=off"]),
    "sx_timestep": ("csrc/sx_timestep.hip", ["-ffp-contract=off"]),
    "sx_skin": ("csrc/sx_skin.hip", ["-ffp-contract=off"]),
}
KEYS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ",
        "SGPRs Spill": "sspill", "VGPRs Spill": "vspill", "LDS Size [bytes/block]": "lds"}


def run(name, src, flags, extra):
    out = subprocess.run(BASE + flags + extra + [src], cwd=ROOT, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?): (\S+) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2)
        if k == "Function Name":
            cur = {"kernel": v}
            rows.append(cur)
        elif cur is not None and k in KEYS:
            cur[KEYS[k]] = v
    print(f"== {name}")
    for r in rows:
        flag = " <-- spills" if r.get("vspill", "0") != "0" or r.get("scratch", "0") != "0" else ""
        print(f"  {r['kernel'][:78]:78s} vgpr {r.get('vgpr', '?'):>3} occ {r.get('occ', '?'):>2} "
              f"scratch {r.get('scratch', '?'):>4} vspill {r.get('vspill', '?'):>3} lds {r.get('lds', '?'):>6}{flag}")


if __name__ == "__main__":
    sel = sys.argv[1:]
    extra = os.environ.get("EXTRA", "").split()
    for name, (src, flags) in SOURCES.items():
        if not sel or any(s in name for s in sel):
            run(name, src, flags, extra)
