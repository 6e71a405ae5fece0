#!/usr/bin/env python3
"""Summarise scripts/pmc_calib.hip under rocprofv3: per access pattern, the
bytes FETCH_SIZE / WRITE_SIZE report over the bytes the kernel touched
(1 GiB each).  Usage: pmc_calib.py DIR (holding the f/ and w/ passes)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

BYTES = 1 << 30


def load(d, cname):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = defaultdict(list)
    for path in f:
        for row in csv.DictReader(open(path)):
            if row.get("Counter_Name") == cname:
                out[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return out


def short(name):
    m = re.search(r"(rd_dma|rd|wr)(?:<(\d+), (true|false)>)?", name)
    if not m:
        return name[:40]
    if m.group(1) == "rd_dma":
        return "read LDS-DMA 16B/lane"
    kind = "read" if m.group(1) == "rd" else "write"
    return f"{kind} {m.group(2)}B/lane{' nontemporal' if m.group(3) == 'true' else ''}"


def main():
    d = sys.argv[1]
    res = {}
    for sub, cname, kind in (("f", "FETCH_SIZE", "read"), ("w", "WRITE_SIZE", "write")):
        for k, v in load(os.path.join(d, sub), cname).items():
            s = short(k)
            if not s.startswith(kind):
                continue
            res[s] = round(sum(v) / len(v) * 1024 / BYTES, 4)
    print(json.dumps(dict(sorted(res.items())), indent=1))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump({"what": "counter bytes / touched bytes per access pattern (1 GiB each, scripts/pmc_calib.hip)",
                       "ratios": dict(sorted(res.items()))}, fh, indent=1)


if __name__ == "__main__":
    main()
