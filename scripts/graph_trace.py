#!/usr/bin/env python3
"""Per-kernel durations inside the timed, graph-replayed region of a bench run
from a rocprofv3 --kernel-trace CSV (diagnostic).

The bench issues warmup + K graph replays, then eager profiling decodes; the
rocprofv3 --stats summary averages all of them.  This prints, per kernel, the
median / mean duration and the median gap to the next dispatch over the
dispatches of the graph-replayed decodes of the timed steps, plus the
per-decode wall time.

Two durations per kernel:
  * "duration": End - Start of the dispatch.  Inside a replayed graph the
    profiler's Start precedes the wait on the predecessor's completion, so
    these overlap: their sum over a decode exceeds the decode's wall time.
  * "exclusive": End - End of the preceding kernel of the decode (the first
    kernel: End - Start), i.e. the kernel plus the same-stream boundary in
    front of it; these add up to the decode's wall time exactly, and are what
    bench.py's back-to-back HIP-event timing measures.

Usage: graph_trace.py <kernel_trace.csv> [out.txt] [source-hash]
"""
import csv
import statistics as st
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402

LOOP = ("k_sec4", "k_sec43", "k_sec2", "k_sec", "k_secb", "k_row2", "k_rowv", "k_rowc", "k_row", "k_gemm_i8_Az", "k_gemm_i8_Ab", "k_gemm_f_Az", "k_gemm_f_Ab",
        "k_dense_az", "k_dense_ab", "k_dense_den", "k_i8_quant")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
           for r in rows]
    # one decode = k_fill32 (iteration counters) ... k_iters_final; the graph
    # replays are the decodes whose dispatches follow each other with no host
    # gap (median gap < 1 us), the eager profiling decodes have launch gaps
    runs, cur = [], None
    for k in seq:
        if "k_fill32" in k[3]:
            cur = []
        elif "k_iters_final" in k[3]:
            if cur:
                runs.append(cur)
            cur = None
        elif cur is not None and k[0] in LOOP:
            cur.append(k[:3])
    def med_gap(r):
        return st.median([r[i + 1][1] - r[i][2] for i in range(len(r) - 1)]) if len(r) > 1 else 1e9
    timed = [r for r in runs if len(r) > 2 and med_gap(r) < 1000]
    if not timed:
        sys.exit("no graph-replayed decode found")
    n0 = st.mode([len(r) for r in timed])
    timed = [r for r in timed if len(r) == n0]
    out = []
    if len(sys.argv) > 3:
        out.append(f"sources sha256 {sys.argv[3]}")
    out.append(f"{len(timed)} graph-replayed decodes of {n0} loop kernels each")
    per = {}
    for r in timed:
        for i, (k, s, e) in enumerate(r):
            d = per.setdefault(k, {"dur": [], "gap": [], "exc": []})
            d["dur"].append(e - s)
            d["exc"].append(e - (r[i - 1][2] if i > 0 else s))
            if i + 1 < len(r):
                d["gap"].append(r[i + 1][1] - e)
    for k, d in per.items():
        out.append(f"{k:14s} n={len(d['dur']):5d}  duration median {st.median(d['dur']):8.0f} ns  mean "
                   f"{st.mean(d['dur']):8.0f} ns  min {min(d['dur']):7d}  gap to next median "
                   f"{st.median(d['gap']) if d['gap'] else 0:6.0f} ns  exclusive median {st.median(d['exc']):8.0f} ns"
                   f"  mean {st.mean(d['exc']):8.0f} ns")
    walls = [r[-1][2] - r[0][1] for r in timed]
    sums = [sum(e - s for _, s, e in r) for r in timed]
    out.append(f"replay wall (first start -> last end): median {st.median(walls) / 1e3:.1f} us; "
               f"sum of durations median {st.median(sums) / 1e3:.1f} us")
    txt = "\n".join(out)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
