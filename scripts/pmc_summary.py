"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/pmc_counter_collection.csv) per kernel: average counter
value per dispatch, with FETCH_SIZE doubled per the gfx950 note (MI355X_MICROARCH.md, HBM) and duration."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] in ("FETCH_SIZE",):
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
out = {}
for k, cs in acc.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    d["dispatches"] = max(len(v) for v in cs.values())  # per pass: each counter is collected in one pass
    if "FETCH_SIZE" in d:
        d["hbm_read_bytes_est"] = 2 * d["FETCH_SIZE"] * 1024  # KB units, x2 gfx950 correction
    if "WRITE_SIZE" in d:
        d["hbm_write_bytes_est"] = d["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
        d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
    if dur.get(k):
        d["profiled_ms"] = sum(dur[k]) / len(dur[k])
    out[k] = d
keys = sorted((k for k in out if k != "_meta"), key=lambda k: -out[k].get("profiled_ms", 0))
for k in keys[:10]:
    d = out[k]
    print(f"{k[:40]:40s} ms={d.get('profiled_ms', 0):7.3f} rd={d.get('hbm_read_bytes_est', 0)/1e9:7.3f}GB "
          f"wr={d.get('hbm_write_bytes_est', 0)/1e9:6.3f}GB L2hit={d.get('l2_hit_rate', 0):.3f} "
          f"vmem_rd={d.get('SQ_INSTS_VMEM_RD', 0):.3g} valu={d.get('SQ_INSTS_VALU', 0):.3g}")
if len(sys.argv) > 2:
    # the workload the passes ran (bench.py's JSON line of the last pass), so bench.py only reuses matching traffic
    meta = {}
    for lf in sorted(glob.glob(os.path.join(root, "p*.log")))[-1:]:
        for line in open(lf):
            if line.startswith("{"):
                try:
                    d = json.loads(line)
                    meta = {"particles_per_gpu": d["config"]["particles_per_gpu"], "workload": d["config"]["workload"],
                            "steps_per_pass": d["steps"] + d["warmup"]}
                except (ValueError, KeyError):
                    pass
    for k, d in out.items():
        if meta.get("steps_per_pass"):
            d["calls_per_step"] = d["dispatches"] / meta["steps_per_pass"]
    out["_meta"] = meta
    json.dump(out, open(sys.argv[2], "w"), indent=1)
