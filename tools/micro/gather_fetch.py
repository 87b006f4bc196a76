#!/usr/bin/env python3
"""Reads the rocprofv3 --pmc passes of tools/micro/gather_fetch (tools/gpu.sh micro) and reports,
per kernel and cache state, the bytes FETCH_SIZE tallies per 128-B line touched and per load
request, against the bytes the kernel asked for (known.json, written by the binary).

Usage: python3 tools/micro/gather_fetch.py DIR [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def dispatches(path):
    """[(kernel, {counter: value})] in dispatch order."""
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows))
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        rows.setdefault(did, (name, {}))[1][r["Counter_Name"]] = float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def main():
    d = sys.argv[1]
    known = json.load(open(os.path.join(d, "known.json")))
    per_pass = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        names = {k["kernel"] for k in known}
        per_pass.append([x for x in dispatches(f) if x[0] in names])
    res = []
    for i, k in enumerate(known):
        e = dict(k)
        for p in per_pass:
            if i < len(p):
                name, cnt = p[i]
                assert name == k["kernel"], (name, k["kernel"])
                e.update(cnt)
        if "FETCH_SIZE" in e:
            b = e["FETCH_SIZE"] * 1024.0
            e["fetch_bytes"] = b
            e["fetch_bytes_per_line"] = round(b / k["lines"], 2)
            e["fetch_bytes_per_request"] = round(b / k["requests"], 2)
            e["fetch_over_bytes_loaded"] = round(b / k["bytes_loaded"], 4)
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            e["l2_hit_rate"] = round(e["TCC_HIT_sum"] / max(e["TCC_HIT_sum"] + e["TCC_MISS_sum"], 1.0), 4)
        res.append(e)
    for e in res:
        print(f"{e['kernel']:10s} {e['cache']:4s} lines {e['lines']:>9.0f} requests {e['requests']:>9.0f} "
              f"FETCH/line {e.get('fetch_bytes_per_line')} FETCH/request {e.get('fetch_bytes_per_request')} "
              f"L2 hit {e.get('l2_hit_rate')}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump({"source": "tools/micro/gather_fetch.hip under rocprofv3 --pmc (one pass per counter set)",
                       "rows": res}, f, indent=1)


if __name__ == "__main__":
    main()
