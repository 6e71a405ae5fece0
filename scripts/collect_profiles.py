#!/usr/bin/env python3
"""Copy the round's profile summaries from gpurun_out/ (scripts/profile_set.sh)
into profiles/<round>_*: kernel stats, PMC traffic per launch (also merged
into profiles/pmc_traffic.json under the bench's workload key), the
graph-replayed kernel durations, SQ counters and phase stamps."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RND = sys.argv[1] if len(sys.argv) > 1 else "r04"
# tag -> bench.py load_pmc key (workload_backend_precision_B)
KEYS = {"c2": "c2_hadamard_fp32_B1", "c4b1": "c4_hadamard_fp32_B1", "c3": "c3_hadamard_fp32_B256",
        "c4": "c4_hadamard_fp32_B256", "c2f64": "c2_hadamard_fp64_B1", "c3f64": "c3_hadamard_fp64_B256",
        "c4f64": "c4_hadamard_fp64_B256", "joint": "c5_hadamard_fp64_B256",
        "dense_l768": "c4_dense_fp32_B1", "c3dense": "c3_dense_fp32_B256",
        "c2matrix": "c2_matrix_fp32_B1", "c3matrix": "c3_matrix_fp32_B256"}


def main():
    out = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    for tag, key in KEYS.items():
        if not os.path.isdir(os.path.join(out, f"prof_{tag}")):
            print("missing", tag)
            continue
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), tag, RND, key], check=True,
                       stdout=subprocess.DEVNULL)
        tr = None
        for dp, _, fs in os.walk(os.path.join(out, f"prof_{tag}", "trace")):
            for f in fs:
                if f.endswith("kernel_trace.csv"):
                    tr = os.path.join(dp, f)
        bt = os.path.join(out, f"prof_{tag}", "build.txt")
        src = open(bt).read().strip() if os.path.exists(bt) else "unknown"
        if tr:
            subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "graph_trace.py"), tr,
                            os.path.join(dst, f"{RND}_{tag}_graph_trace.txt"), src], check=False,
                           stdout=subprocess.DEVNULL)
    for tag in ("c2", "c3", "c4", "c3f64", "c3dense", "bp"):
        p = os.path.join(out, f"sq_{tag}.txt")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{RND}_{tag}_sq_counters.txt"))
    for tag, kern in (("c2", "k_sec4"), ("c4b1", "k_sec43"), ("c3", "k_secb")):
        p = os.path.join(out, f"stamps_{tag}.txt")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{RND}_{tag}_{kern}_stamps.txt"))
    cal = os.path.join(out, "pmc_calib.json")
    if os.path.exists(cal):
        shutil.copy(cal, os.path.join(dst, f"{RND}_pmc_calib.json"))
    print(sorted(f for f in os.listdir(dst) if f.startswith(RND)))


if __name__ == "__main__":
    main()
