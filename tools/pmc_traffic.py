#!/usr/bin/env python3
"""Turns the rocprofv3 --pmc passes of `tools/gpu.sh pmc` into the per-launch traffic
summary bench.py reports as roofline.traffic.

Counters (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are KiB per
dispatch from the L2's memory-side request counters (Infinity-Cache hits included);
on gfx950 FETCH_SIZE tallies every 128-B L2 line request at 64 B, so it is doubled (calibrated
for the SDF gathers by tools/micro/gather_fetch.hip).  The
rollout-cost stage is the fused k_rollout kernel (one launch per iteration).

SQ_INSTS_VALU (VALU instructions issued, summed over the launch's waves) gives the VALU issue
fraction: SQ_INSTS_VALU x 4 cycles (a wave64 instruction on a 16-lane SIMD) / (CUs x 4 SIMDs) /
(kernel duration x 2.4 GHz), with the duration from the kernel-trace stats of the same build
(bench.py divides by its own event-measured duration).

The summary records the engine's source hash (_build.source_hash): bench.py reports these
numbers only while the sources are the ones profiled.

Usage: python tools/pmc_traffic.py <pmc dir> <out.json> [kernel_stats.csv [workload]]
(workload: the bench.py --workload the passes ran, cfg2 by default; bench.py reports a summary for
the workload it runs only)
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
    out = {}
    for k, d in agg.items():
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        out[k]["dispatches"] = max(len(v) for v in d.values())
    return out


def main():
    src, out = sys.argv[1], sys.argv[2]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from stomp_motion_planner_icra2011_amd import _build
    durations = {}
    if len(sys.argv) > 3:
        for r in csv.DictReader(open(sys.argv[3])):
            durations[r["Name"].split("(")[0].replace("void ", "").strip()] = float(r["AverageNs"])
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
        if "SQ_INSTS_VALU" in d and k in durations:
            e["avg_ns"] = durations[k]
            e["valu_issue_frac"] = round(d["SQ_INSTS_VALU"] * 4.0 / (256 * 4) / (durations[k] * 1e-9 * 2.4e9), 4)
        kernels[k] = e
    workload = sys.argv[4] if len(sys.argv) > 4 else "cfg2"
    # the iteration's rollout launch: the k_rollout instantiation with the most dispatches (the
    # deferred noiseless flush at the end of a run is a different, rare launch)
    ro = [k for k in kernels if k.startswith("stomp::k_rollout")]
    stage = [max(ro, key=lambda k: kernels[k].get("dispatches", 0))] if ro else []
    res = {
        "source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE TCC_HIT_sum TCC_MISS_sum | SQ_* (separate passes), "
                  "bench.py --workload " + workload + " --no-timing (tools/gpu.sh pmc); per-dispatch means",
        "workload": workload,
        "correction": "FETCH_SIZE x2: gfx950 tallies every L2 miss (one 128-B line request) at 64 B, for wide "
                      "coalesced reads (MI355X_MICROARCH.md:298) and for the SDF's 2-byte scattered gathers alike "
                      "(tools/micro/gather_fetch.hip, profiles/r6_gather_fetch.txt: one 2-B load per distinct line "
                      "and four per line both read 64.0 B per line touched, two or four far-apart loads per line "
                      "128 / 256 B); the x1 figure is kept beside it for comparison with earlier rounds.  KiB -> B; "
                      "Infinity-Cache hits are counted (memory side of L2), so this is L2-miss traffic, an upper "
                      "bound on HBM bytes",
        "stage": stage[0] if stage else None,
        "source_hash": _build.embedded_hash(_build.LIB),   # the library the PMC passes ran
        "hbm_bytes_per_launch": sum(kernels[k].get("hbm_bytes", 0.0) for k in stage),
        "valu_insts_per_launch": sum(kernels[k].get("SQ_INSTS_VALU", 0.0) for k in stage),
        "valu_issue_frac": kernels[stage[0]].get("valu_issue_frac") if stage else None,
        "hbm_bytes_per_launch_uncorrected": sum(kernels[k].get("hbm_bytes_uncorrected", 0.0) for k in stage),
        "kernels": kernels,
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v.get("hbm_bytes") for k, v in kernels.items()}, indent=1))
    print("stage bytes per launch", res["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
