#!/usr/bin/env python3
"""Turns the rocprofv3 --pmc passes of tools/gpu_pmc.sh into the per-launch traffic
summary bench.py reports as roofline.traffic.

Counters (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are KiB per
dispatch from the L2's memory-side request counters (Infinity-Cache hits included);
on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it is doubled.  The
rollout-cost stage is the fused k_rollout kernel (one launch per iteration).

Usage: python tools/pmc_traffic.py <pmc dir> <out.json>
"""
import csv
import collections
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    src, out = sys.argv[1], sys.argv[2]
    merged = collections.defaultdict(dict)
    for f in sorted(os.listdir(src)):
        if f.endswith("counter_collection.csv"):
            for k, d in per_kernel(os.path.join(src, f)).items():
                merged[k].update(d)
    kernels = {}
    for k, d in merged.items():
        if "stomp::" not in k:
            continue
        e = {c: round(v, 3) for c, v in d.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            e["fetch_bytes_corrected"] = 2.0 * d["FETCH_SIZE"] * 1024
            e["fetch_bytes_uncorrected"] = d["FETCH_SIZE"] * 1024
            e["write_bytes"] = d["WRITE_SIZE"] * 1024
            e["hbm_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
            e["hbm_bytes_uncorrected"] = e["fetch_bytes_uncorrected"] + e["write_bytes"]
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            e["l2_hit_rate"] = round(d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1.0), 4)
        kernels[k] = e
    stage = [k for k in kernels if k.startswith("stomp::k_rollout")]
    res = {
        "source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE TCC_HIT_sum TCC_MISS_sum | SQ_* (separate passes), "
                  "bench.py --steps 40 --warmup 5 --no-timing; per-dispatch means",
        "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B, MI355X_MICROARCH.md:298, calibrated "
                      "for wide coalesced reads); the SDF gathers are 4-B lane loads, for which the factor is "
                      "uncalibrated, so the uncorrected figure (x1) is reported beside it: the true bytes lie "
                      "between the two.  KiB -> B; Infinity-Cache hits are counted (memory side of L2), so this is "
                      "L2-miss traffic, an upper bound on HBM bytes",
        "stage": "rollout_cost = k_rollout",
        "hbm_bytes_per_launch": sum(kernels[k].get("hbm_bytes", 0.0) for k in stage),
        "hbm_bytes_per_launch_uncorrected": sum(kernels[k].get("hbm_bytes_uncorrected", 0.0) for k in stage),
        "kernels": kernels,
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v.get("hbm_bytes") for k, v in kernels.items()}, indent=1))
    print("stage bytes per launch", res["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
