#!/usr/bin/env python3
"""Summarise scripts/profile.sh output into profiles/<round>_<tag>_*.

HBM bytes per dispatch from the TCC counters (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts
exactly half of a wide (16 B/lane) coalesced streaming read, so the read side
is reported both raw and doubled; WRITE_SIZE is exact for 16-B stores.
Our kernels mix 8- and 16-B loads, so the corrected read figure is an upper
bound and the raw one a lower bound; `hbm_bytes_per_launch` uses the
corrected (x2) read side.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    if "k_gemm_i8<3>" in name:
        return "k_gemm_i8_Az"   # three digit planes of z
    if "k_gemm_i8<4>" in name:
        return "k_gemm_i8_Ab"   # four digit planes of beta
    if "k_gemm_f<" in name:  # caller-matrix GEMMs: <real, 0> A^T z, <real, 1> A beta
        return "k_gemm_f_Ab" if ", 1>" in name else "k_gemm_f_Az"
    for k in ("k_secb", "k_sec2", "k_sec43", "k_sec4", "k_sec8", "k_sec", "k_row2", "k_rowv", "k_rowc", "k_row", "k_dense_az", "k_dense_ab", "k_dense_den", "k_decide",
              "k_gemm_i8", "k_i8_quant", "k_i8_build",
              "k_bp_tail_chk", "k_bp_tail_var", "k_bp_tail_end", "k_bp", "k_llr", "k_bp2sp", "k_sp_norm", "k_colsum"):
        if any(p in name for p in (f"::{k}<", f" {k}<", f" {k}(", f"::{k}(")) or name.startswith((f"{k}<", f"{k}(")):
            return k
    return name.split("(")[0][-40:]


def counters(path, cname):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    acc = defaultdict(list)
    with open(f[0]) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") == cname:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag, rnd, key = sys.argv[1], sys.argv[2], sys.argv[3]
    out = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, f"{rnd}_{tag}_kernel_stats.csv"))
    fetch = counters(os.path.join(out, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(out, "write"), "WRITE_SIZE")
    res = {}
    bt = os.path.join(out, "build.txt")
    src = open(bt).read().strip() if os.path.exists(bt) else None
    for k in sorted(set(fetch) | set(write)):
        fk, wk = fetch.get(k, 0.0), write.get(k, 0.0)
        res[k] = {"fetch_kib_raw": fk, "write_kib": wk,
                  "hbm_bytes_per_launch": int((2 * fk + wk) * 1024),
                  "hbm_bytes_per_launch_raw": int((fk + wk) * 1024), "sources": src, "round": rnd}
    with open(os.path.join(dst, f"{rnd}_{tag}_pmc.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    p = os.path.join(dst, "pmc_traffic.json")
    allp = json.load(open(p)) if os.path.exists(p) else {}
    allp[key] = res
    with open(p, "w") as fh:
        json.dump(allp, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
