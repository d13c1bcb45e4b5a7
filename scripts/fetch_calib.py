"""FETCH_SIZE / WRITE_SIZE calibration factors from scripts/fetch_calib.hip's rocprofv3 passes.

  python scripts/fetch_calib.py <dir> [out.json]

<dir> holds known.json (the program's JSON line), f/ (the --pmc FETCH_SIZE pass) and w/ (the --pmc WRITE_SIZE pass).
For each access shape: the counter bytes of its last dispatch (KB units x 1024) and factor = known bytes / counter
bytes, i.e. what a counter reading of that shape must be multiplied by to give bytes.
"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
known = json.load(open(os.path.join(root, "known.json")))
last = {}
for sub, counter in (("f", "FETCH_SIZE"), ("w", "WRITE_SIZE")):
    for f in glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].strip()
            name = name.replace("void ", "").split("<")[0]
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            last[(name, counter)] = (float(r["Counter_Value"]) * 1024.0, ms)
out = {}
for shape, kb in known.items():
    counter = "WRITE_SIZE" if shape.startswith("wr") else "FETCH_SIZE"
    v = last.get((shape, counter))
    if v is None:
        continue
    out[shape] = {"counter": counter, "known_bytes": kb, "counter_bytes": v[0], "factor": kb / v[0] if v[0] else None,
                  "ms": v[1], "known_gbs": kb / (v[1] * 1e-3) / 1e9}
    print(f"{shape:9s} {counter:10s} known {kb / 2**20:8.1f} MiB  counter {v[0] / 2**20:8.1f} MiB  "
          f"factor {out[shape]['factor']:.3f}  {v[1]:.3f} ms  {out[shape]['known_gbs']:.0f} GB/s")
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
