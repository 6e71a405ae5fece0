#!/usr/bin/env python3
"""Timeline of the pipelined joint step from a rocprofv3 --kernel-trace CSV
(diagnostic): over the window of the last N AMP/BP kernels, how much wall time
has AMP kernels running, BP kernels running, both, or neither, per stream.

Usage: joint_timeline.py <kernel_trace.csv> [window_start_fraction]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = []
    for r in rows:
        k = r["Kernel_Name"]
        kind = "bp" if "k_bp" in k else ("amp" if any(s in k for s in ("k_secb", "k_rowc", "k_row", "k_sec")) else "glue")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r["Stream_Id"], k.split("::", 1)[-1].split("(")[0][:40]))
    ev.sort()
    # the timed step of `bench_joint.py --no-ref --warmup 0 --steps 1`: from the
    # first section kernel to the last kernel of the last slice's streams (the
    # eager profiling decodes after it run on the first slice's streams only)
    streams = sorted({e[3] for e in ev}, key=int)
    last_streams = set(streams[-2:]) if len(streams) > 2 else set(streams)
    ws = min(e[0] for e in ev if "k_secb" in e[4])
    we = max(e[1] for e in ev if e[3] in last_streams and e[2] != "glue") if len(streams) > 2 else None
    if we is None:  # one slice: up to the last BP kernel of the step (before the profiling decodes)
        bps = [e for e in ev if e[2] == "bp"]
        we = bps[-1][1] if bps else max(e[1] for e in ev)
        # the profiling run's own BP launch is the last one: the step's BP ends before the profile's AMP
        prof = [e[0] for e in ev if e[2] == "amp" and e[0] > ws]
    ev = [e for e in ev if e[0] >= ws and e[1] <= we]
    t0 = ws
    # sweep
    pts = []
    for s, e, kind, st, _ in ev:
        pts.append((s, 1, kind))
        pts.append((e, -1, kind))
    pts.sort()
    cnt = {"amp": 0, "bp": 0, "glue": 0}
    acc = {}
    last = pts[0][0]
    for t, d, kind in pts:
        key = ("amp" if cnt["amp"] else "") + ("+bp" if cnt["bp"] else "") + ("+glue" if cnt["glue"] and not cnt["amp"] and not cnt["bp"] else "")
        acc[key or "idle"] = acc.get(key or "idle", 0) + (t - last)
        cnt[kind] += d
        last = t
    tot = sum(acc.values())
    phases(ev, t0)
    print(f"window {tot / 1e6:.2f} ms")
    for k, v in sorted(acc.items(), key=lambda x: -x[1]):
        print(f"  {k:12s} {v / 1e6:9.3f} ms  {100 * v / tot:5.1f} %")
    # per stream busy
    per = {}
    for s, e, kind, st, _ in ev:
        per.setdefault((st, kind), 0)
        per[(st, kind)] += e - s
    for k, v in sorted(per.items()):
        print(f"  stream {k[0]} {k[1]:5s} busy(sum of durations) {v / 1e6:9.3f} ms")
    # bp tail kernel durations alone vs overlapped
    import statistics as stt
    for name in ("k_bp_tail_chk", "k_bp_tail_var", "k_secb", "k_rowc"):
        d = [e - s for s, e, kind, st, nm in ev if name in nm]
        if d:
            print(f"  {name:14s} n={len(d):6d} median {stt.median(d) / 1e3:8.2f} us  mean {stt.mean(d) / 1e3:8.2f} us")


def phases(ev, t0, gap=200_000):
    """Per stream: runs of same-kind kernels (gaps < `gap` ns merged)."""
    out = {}
    for s, e, kind, st, nm in sorted(ev):
        if kind == "glue":
            continue
        lst = out.setdefault(st, [])
        if lst and lst[-1][2] == kind and s - lst[-1][1] < gap:
            lst[-1][1] = max(lst[-1][1], e)
            lst[-1][3] += 1
        else:
            lst.append([s, e, kind, 1])
    for st, lst in sorted(out.items(), key=lambda x: int(x[0])):
        print(f"  stream {st}: " + "  ".join(f"{k}[{(a - t0) / 1e6:.1f}-{(b - t0) / 1e6:.1f}]" for a, b, k, _ in lst))


if __name__ == "__main__":
    main()
