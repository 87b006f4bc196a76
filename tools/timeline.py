"""Kernel timeline of a rocprofv3 kernel trace (rocprofv3 --kernel-trace): the last `n` iterations,
each dispatch's start relative to the first and its duration, in microseconds."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = list(csv.DictReader(open(path)))
rows = [r for r in rows if "k_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# take the tail: the last n rollout launches onward
idx = [i for i, r in enumerate(rows) if "k_rollout" in r["Kernel_Name"]]
sel = rows[idx[-n - 1]:idx[-1]] if len(idx) > n else rows
t0 = int(sel[0]["Start_Timestamp"])
prev_end = None
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void stomp::", "")[:28]
    gap = "" if prev_end is None else f"gap {(s - prev_end) / 1000:7.2f}"
    print(f"{name:28s} q{r.get('Queue_Id', '?'):>3s} start {(s - t0) / 1000:8.2f} dur {(e - s) / 1000:7.2f} {gap}")
    prev_end = e if prev_end is None else max(prev_end, e)
span = (int(sel[-1]["End_Timestamp"]) - t0) / 1000
print(f"span {span:.2f} us over {n} iterations: {span / n:.2f} us/iteration")
