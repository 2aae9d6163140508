#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (gpurun_out/) into committed files under profiles/.

    python scripts/pmc_summary.py --round r01

Reads gpurun_out/pmc/<pass>/run_counter_collection.csv (scripts/pmc.sh) and
gpurun_out/prof_kt/run_kernel_stats.csv (`scripts/gpu.sh kt`), writes
profiles/<round>_pmc_summary.json, profiles/<round>_kernel_stats.csv and
profiles/pmc_rsa_pow.json (read by bench.py for roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reads 1/2 of the bytes of a 16-B-per-lane stream, so the
read side is doubled (our kernels read 16 B per lane, gathered by grant).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_pass(name):
    files = glob.glob(os.path.join(ROOT, "gpurun_out", "pmc", name, "*counter_collection.csv"))
    if not files:
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    rows = list(csv.DictReader(open(files[0])))
    # only the headline dispatches: per kernel, the largest grid (bench.py also
    # runs host-path chunks and the wire path, which launch smaller grids)
    big = collections.defaultdict(int)
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("mochi::", "").replace("void ", "")
        big[k] = max(big[k], int(r["Grid_Size"]))
    # persistent kernels (k_rsa_pow / k_rsa_final) launch one grid for every
    # size: keep, per kernel, the dispatches whose duration is at least half the
    # longest (the headline; the producer's public-key checks are ~4x shorter)
    dur = collections.defaultdict(dict)
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("mochi::", "").replace("void ", "")
        dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("mochi::", "").replace("void ", "")
        if int(r["Grid_Size"]) != big[k] or dur[k][r["Dispatch_Id"]] < 0.5 * max(dur[k].values()):
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--grants", type=int, default=15980098)
    ap.add_argument("--what", default="bench.py --headline-only --steps 2 --warmup 1 (C4: 16M grants, R=4)")
    a = ap.parse_args()
    per = collections.defaultdict(dict)
    for p in ("sq1", "sq2", "sq3", "fetch", "write"):
        for k, d in load_pass(p).items():
            per[k].update(d)
    out = {"source": f"rocprofv3 --pmc, scripts/pmc.sh ({a.what}); values are per dispatch of the largest grid "
                     "(the headline launch), averaged over those dispatches", "kernels": {}}
    for k, d in per.items():
        e = dict(d)
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            e["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
            e["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]
        if "GRBM_GUI_ACTIVE" in d:
            e["gui_active_cycles_per_xcd"] = d["GRBM_GUI_ACTIVE"] / 8
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            w = d["SQ_WAVE_CYCLES"]
            e["frac_active"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
            e["frac_wait_inst"] = d.get("SQ_WAIT_INST_ANY", 0) / w
            e["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / w
        if "SQC_ICACHE_HITS" in d:
            tot = d["SQC_ICACHE_HITS"] + d.get("SQC_ICACHE_MISSES", 0) + d.get("SQC_ICACHE_MISSES_DUPLICATE", 0)
            e["icache_miss_rate"] = (d.get("SQC_ICACHE_MISSES", 0) + d.get("SQC_ICACHE_MISSES_DUPLICATE", 0)) / tot
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            # MFMA busy cycles summed over the 1,024 SIMDs vs the kernel's GPU cycles
            e["mfma_busy_frac"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (d["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_INSTS_VALU" in d and "SQ_INSTS_VALU_INT64" in d:
            e["valu_int64_share"] = d["SQ_INSTS_VALU_INT64"] / d["SQ_INSTS_VALU"]
        out["kernels"][k] = e
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{a.round}_pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    pow_ = out["kernels"].get("k_rsa_pow", {})
    if "hbm_bytes_per_launch" in pow_:
        algo = a.grants * (256 + 4 + 2 + 74 * 4)
        with open(os.path.join(ROOT, "profiles", "pmc_rsa_pow.json"), "w") as f:
            json.dump({"kernel": "k_rsa_pow", "round": a.round, "grants_per_launch": a.grants,
                       "hbm_bytes_per_launch": round(pow_["hbm_bytes_per_launch"]),
                       "algorithmic_bytes_per_launch": algo,
                       "note": "FETCH_SIZE*2 (gfx950 16-B/lane correction) + WRITE_SIZE, KiB->B"}, f, indent=1)
    ks = os.path.join(ROOT, "gpurun_out", "prof_kt", "run_kernel_stats.csv")
    found = glob.glob(os.path.join(ROOT, "gpurun_out", "prof_kt", "**", "*kernel_stats.csv"), recursive=True)
    ks = found[0] if found else ks
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(ROOT, "profiles", f"{a.round}_kernel_stats.csv"))
    print(json.dumps({k: {kk: v for kk, v in e.items() if not kk.startswith("SQ")} for k, e in out["kernels"].items()},
                     indent=1))


if __name__ == "__main__":
    main()
