#!/usr/bin/env python3
"""Per-launch durations of the BP kernels from a rocprofv3 kernel trace
(diagnostic): the monolithic k_bp launches and, per tail iteration, the
variable / check kernel durations and the gap between iterations.
Usage: bp_tail_trace.py DIR"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
bp = [r for r in rows if "k_bp" in r["Kernel_Name"]]
runs, cur = [], []
for r in bp:
    if "k_bp<" in r["Kernel_Name"] or "k_bpILi" in r["Kernel_Name"] or r["Kernel_Name"].split("(")[0].endswith("k_bp"):
        if cur:
            runs.append(cur)
        cur = [r]
    else:
        cur.append(r)
if cur:
    runs.append(cur)
for i, run in enumerate(runs[-6:]):
    t0, t1 = int(run[0]["Start_Timestamp"]), int(run[-1]["End_Timestamp"])
    mono = (int(run[0]["End_Timestamp"]) - t0) / 1e3
    chk = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in run if "tail_chk" in r["Kernel_Name"]]
    var = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in run if "tail_var" in r["Kernel_Name"]]
    print(f"run {i}: total {(t1 - t0) / 1e3:9.1f} us  k_bp {mono:8.1f} us  tail iterations {len(chk)}")
    if chk:
        q = [chk[j] for j in (0, len(chk) // 4, len(chk) // 2, 3 * len(chk) // 4, len(chk) - 1)]
        print("   chk us (first, q1, median, q3, last):", [round(x, 1) for x in q], " sum", round(sum(chk), 1))
        print("   var us median", round(sorted(var)[len(var) // 2], 1), " sum", round(sum(var), 1),
              " gaps (total - k_bp - kernels)", round((t1 - t0) / 1e3 - mono - sum(chk) - sum(var), 1))
