#!/usr/bin/env python3
"""Per-(kernel, grid) durations from a rocprofv3 kernel trace (gpurun_out/prof_kt).

    python scripts/trace_summary.py --round r02

rocprofv3 --stats averages every dispatch of a kernel; a bench run also
launches k_rsa_pow / k_rsa_final / k_grant_prep for the producer signer's
public-key check (workload generation, smaller grids), so the headline
launches are separated here by grid size.  Writes
profiles/<round>_kernel_trace_summary.json.
"""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ap = argparse.ArgumentParser()
ap.add_argument("--round", default="r02")
ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out", "prof_kt"))
a = ap.parse_args()
f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("mochi::", "").replace("void ", "")
    d[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {}
for (k, g), v in sorted(d.items(), key=lambda x: -sum(x[1])):
    if not k.startswith("k_"):
        continue
    v = sorted(v)
    e = {"calls": len(v), "avg_ms": round(sum(v) / len(v), 4), "min_ms": round(v[0], 4),
         "median_ms": round(v[len(v) // 2], 4), "max_ms": round(v[-1], 4)}
    # persistent kernels keep one grid for every batch size: the headline
    # launches are those at least half as long as the longest (only for them:
    # a kernel stretched once by running beside k_rsa_pow would pick its outlier)
    h = [x for x in v if x >= 0.5 * v[-1]]
    if k in ("k_rsa_pow", "k_rsa_final", "k_bucket_count", "k_bucket_scan", "k_bucket_scatter") and len(h) < len(v):
        e["headline"] = {"calls": len(h), "avg_ms": round(sum(h) / len(h), 4), "median_ms": round(h[len(h) // 2], 4)}
    out[f"{k} grid={g}"] = e
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
dst = os.path.join(ROOT, "profiles", f"{a.round}_kernel_trace_summary.json")
json.dump({"source": os.path.relpath(f, ROOT), "kernels": out}, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
