#!/usr/bin/env python3
"""Benchmark: decoded codewords/s of the MI355X SPARC AMP decoder.

Metric (BASELINE.json): "decoded codewords/sec (T AMP iters) at L=512,M=512;
achieved HBM GB/s vs roofline".  Default workload = BASELINE configs[1]:
L=512 M=512 R=1 P=4 (n=4608), T=64 iterations, one codeword per step, on the
matrix-free Hadamard backend in fp32.  A "step" is one full AMP decode of the
batch (T iterations, the early stop disabled so every step does T
iterations), with y already resident in HBM.

Contract: ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the
driver launches one rank per GPU with torch.distributed.run; reps are
sharded (weak scaling: each rank decodes its own batch, no data-path
collective); the only exchange is the final max-of-times / counter
all-reduce over RCCL.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
I8_PEAK_TOPS = 5000.0  # dense int8 MFMA: 2x the ~2.5 PF bf16 rate per clock (MI355X_MICROARCH.md, Matrix cores)
NP_Z, NP_B = 3, 4      # int8 digit planes of z and beta on the dense GEMM path (csrc/dense_i8.hip)
PROFILE_REP = 16       # back-to-back launches per event pair (roofline timing)

WORKLOADS = {
    # name: (L, M, R, P, snr_dB or sigma, T, B)
    "c2": dict(L=512, M=512, R=1.0, P=4.0, sigma=float(np.sqrt(4.0 / 10 ** (10 / 20))), T=64, B=1,
               desc="BASELINE configs[1]: L=512 M=512 R=1 P=4, T=64, single codeword"),
    "c3": dict(L=512, M=512, R=1.0, P=4.0, sigma=float(np.sqrt(4.0 / 10 ** (10 / 20))), T=64, B=256,
               desc="BASELINE configs[2]: L=512 M=512 R=1 P=4, T=64, batch of 256 codewords"),
    "c4": dict(L=768, M=512, R=5 / 6, P=1.8, sigma=0.6, T=64, B=256,
               desc="BASELINE configs[3]: L=768 M=512 R=5/6 P=1.8, T=64, 256 reps per GPU per step"),
}


def n_of(w):
    return int(w["L"] * np.log2(w["M"]) / w["R"])


def synth_y(op, Pl, sigma, seeds):
    """Synthetic reps: RandomState(seed) -> L indices in [0, M),
    then N(0, σ²) noise; x = A β₀ on the device."""
    L, M, n = op.L, op.M, op.n
    c = np.sqrt(n * Pl)
    B = len(seeds)
    beta0 = np.zeros((B, L * M))
    noise = np.empty((B, n))
    for i, s in enumerate(seeds):
        rs = np.random.RandomState(s)
        idx = rs.randint(0, M, L)
        beta0[i, np.arange(L) * M + idx] = c
        noise[i] = rs.randn(n) * sigma
    return op.Ab_batch(beta0) + noise


def sec_bytes(L, M, n, w, B, G, s, kernel="k_sec4"):
    """Algorithmic bytes of one k_sec launch: the bucket and Ab
    tables once (uint16 per slot and per section-row; k_sec43 packs a section
    triple's Ab entries into one uint32 per row), z once per codeword, β read
    + write, Ab partials written.  k_sec4i / k_sec43i (bucket tables built in
    LDS from the ordering values) read n ordering values per section instead
    of the w-entry bucket tables and the Ab table."""
    if kernel in ("k_sec4i", "k_sec43i"):
        # bucket tables built in LDS: only the ordering values are read (pairs
        # one uint32 per row and pair, triples 8 bytes per row and triple)
        tables = (8 if kernel == "k_sec43i" else 4) * n * G
    else:
        tables = 2 * L * w + (4 * n * G if kernel == "k_sec43" else 2 * L * n)
    return tables + B * (n * s + 2 * L * M * s + G * n * s)


def row_bytes(n, B, G, s):
    """k_row: Ab partials read, y read, z read + write."""
    return B * (G * n * s + 3 * n * s)


def gemv_bytes(L, M, n):
    """4·n·L·M + 4·(n + L·M) per fp32 GEMV."""
    return 4 * n * L * M + 4 * (n + L * M)


def i8_gemm_ops(L, M, n, B, planes):
    """Algorithmic int8 multiply-adds x 2 of one dense GEMM on the matrix cores:
    `planes` digit planes of B codewords against the n x L·M ±1 matrix (the
    fp32-equivalent GEMM of SURVEY §8d is 2·n·L·M·B flops: this counts each
    digit plane's product, the work the int8 MFMA actually does)."""
    return 2 * planes * B * n * L * M


def _cpu_worker(args, barrier, q):
    """One host process: build the oracle operator (untimed), wait at the
    barrier for every other process, then time Tsample AMP iterations of one
    codeword; puts its (start, end) wall-clock span."""
    L, M, n, P, sigma, Tsample, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import amp_oracle as orc
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    Pl = P / L * np.ones(L)
    _, y = orc.rep_inputs(L, M, n, Pl, sigma, Ab, seed)
    barrier.wait()  # every process starts its timed loop together: no spawn / import stagger in the span
    t0 = time.time()
    orc._amp_core(y, Pl, L, M, Tsample, Ab, Az, None, early_stop=False)  # exactly Tsample iterations
    q.put((t0, time.time()))


def host_cpus():
    """(usable cores, description): every core of sched_getaffinity, bounded by
    the cgroup CPU quota when one is set (the cores this process may really
    use), and the CPU model from /proc/cpuinfo."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    use = aff if quota is None else min(aff, quota)
    return use, f"{model}; sched_getaffinity {aff} cores, cgroup quota {quota or 'none'}"


def cpu_baseline(w, procs=None, Tsample=None):
    """The oracle (the reference's algorithm in fp64 NumPy, vectorised FWHT) on
    the host: `procs` independent single-threaded processes (default: every
    usable core), each timing Tsample AMP iterations of its own codeword after
    a barrier (set-up untimed); the rate is all iterations over the wall-clock
    span from the common start to the last finish, scaled to T iterations per
    codeword."""
    import multiprocessing as mp
    L, M, P, sigma, T = w["L"], w["M"], w["P"], w["sigma"], w["T"]
    n = n_of(w)
    use, desc = host_cpus()
    procs = procs or use
    Tsample = Tsample or T  # a whole decode per process: no extrapolation
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(procs), ctx.Queue()
    ps = [ctx.Process(target=_cpu_worker, args=((L, M, n, P, sigma, Tsample, 1000 + i), barrier, q))
          for i in range(procs)]
    for p in ps:
        p.start()
    spans = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    wall = max(e for _, e in spans) - min(s for s, _ in spans)
    per_core = float(np.mean([e - s for s, e in spans])) / Tsample
    return {
        "value": procs * Tsample / wall / T, "unit": "codewords/s", "cores": procs, "kind": "port",
        "cpu": desc,
        "sample": f"oracle amp() fp64 NumPy (the reference algorithm), {procs} single-threaded processes x "
                  f"1 codeword x {Tsample} iterations (L={L} M={M} n={n}) in {wall:.1f} s wall, "
                  f"scaled to T={T} iterations/codeword; {per_core * 1e3:.1f} ms/iteration/process",
    }


def dense_gemv_probe(device):
    """North-star GEMV at L=768 M=512 R=5/6 (n=8294) on the dense backend:
    fp32 A (13.05 GB) streamed once per product; per-kernel event timing."""
    import sparc_ldpc_amd as sp
    L, M, R, P = 768, 512, 5 / 6, 1.8
    n = int(L * np.log2(M) / R)
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense", precision="fp32", device=device)
    Pl = P / L * np.ones(L)
    y = synth_y(op, Pl, 0.6, [7])
    op.reserve(1, 4)
    op.stage(y, Pl)
    op.profile(1, 2, early_stop=False)  # warm
    kinds, _ = op.profile(1, 2, early_stop=False, rep=4)
    gb = gemv_bytes(L, M, n) / 1e9
    out = {"workload": "L=768 M=512 R=5/6 single codeword, dense fp32 A", "bytes_per_gemv": gemv_bytes(L, M, n)}
    for k in ("k_dense_az", "k_dense_ab"):
        ms = kinds[k][0]
        out[k] = {"ms": ms, "achieved_GBs": gb / (ms * 1e-3), "frac": gb / (ms * 1e-3) / HBM_PEAK_GBS}
    del op
    return out


def load_sq(tag, kernel):
    """SQ counters (mean per launch) of `kernel` from the newest committed
    profiles/<round>_<tag>_sq_counters.txt (scripts/pmc_sq.sh), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{tag}_sq_counters.txt")))
    if not files:
        return None
    out, cur = {}, None
    for line in open(files[-1]):
        if not line.startswith(" "):
            cur = line.split(" ")[0]
        elif cur == kernel:
            k, v = line.split()
            out[k] = float(v)
    return (out, os.path.relpath(files[-1], ROOT)) if out else None


def valu_bound(tag, kernel, kernel_ms, cus, clock_ghz=2.4):
    """VALU busy and issue fractions of the SIMDs over the batched section
    kernel's duration from its SQ counters (SQ_ACTIVE_INST_VALU in
    quad-cycles; a wave64 VALU instruction issues over 2 cycles on a SIMD-32,
    MI355X_MICROARCH.md).  Busy well above issue: the kernel waits on
    dependent chains, not on VALU issue (a quarter fewer VALU
    instructions measured neutral, the gather without its table loads 10 %
    faster)."""
    got = load_sq(tag, kernel)
    if got is None:
        return None
    sq, src = got
    simd_cycles = 4 * cus * kernel_ms * 1e-3 * clock_ghz * 1e9
    return {"valu_busy_frac": round(4 * sq["SQ_ACTIVE_INST_VALU"] / simd_cycles, 3),
            "valu_issue_frac": round(2 * sq["SQ_INSTS_VALU"] / simd_cycles, 3),
            "valu_instructions_per_launch": int(sq["SQ_INSTS_VALU"]),
            "lds_bank_conflict_cycles_frac": round(sq["SQ_LDS_BANK_CONFLICT"] / max(1.0, sq["SQ_LDS_IDX_ACTIVE"]), 3),
            "source": src, "clock_ghz_assumed": clock_ghz}


PROFILE_TAGS = {  # (workload, codewords, backend) -> scripts/profile_r*.sh tag (binary32)
    ("c2", 1, "hadamard"): "c2", ("c4", 1, "hadamard"): "c4b1", ("c3", 256, "hadamard"): "c3",
    ("c4", 256, "hadamard"): "c4", ("c3", 256, "dense"): "c3dense", ("c4", 1, "dense"): "dense_l768",
}


def load_graph_median(tag, kernel):
    """In-graph launch duration of `kernel` (ns): the median over the
    graph-replayed decodes of the newest committed
    profiles/<round>_<tag>_graph_trace.txt (rocprofv3 kernel trace of the same
    bench command, scripts/graph_trace.py), with that file's name; or None."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{tag}_graph_trace.txt")))
    if not files:
        return None
    for line in open(files[-1]):
        m = re.match(r"(\S+)\s+n=\s*(\d+)\s+duration median\s+(\d+) ns", line)
        if m and m.group(1) == kernel:
            return float(m.group(3)), int(m.group(2)), os.path.relpath(files[-1], ROOT)
    return None


def load_pmc(workload, kernel):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        return d.get(workload, {}).get(kernel)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--backend", default="hadamard", choices=["hadamard", "dense"])
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--batch", type=int, default=0, help="override codewords per step")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0)
    ap.add_argument("--no-fp64", action="store_true", help="skip the binary64 leg of an fp32 run")
    args = ap.parse_args()

    from sparc_ldpc_amd import dist

    rank, world, local = dist.env_rank()
    if args.gpus != world:
        # a launch without torchrun (or with another rank count) would print an
        # honest n_gpus = WORLD_SIZE line for a job nobody asked for: refuse it
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N > 1 as "
              f"python -m torch.distributed.run --nproc-per-node N bench.py --gpus N", file=sys.stderr)
        sys.exit(2)
    import sparc_ldpc_amd as sp
    # one rank per GPU over RCCL (librccl through ctypes, no PyTorch); the
    # rehearsal mode SPARC_DIST_BACKEND=socket puts several ranks on one GPU
    # (device LOCAL_RANK % device count) with the CPU all-reduce instead
    ndev = sp.load_library().sa_device_count()
    device = local % max(1, ndev) if os.environ.get("SPARC_DIST_BACKEND") == "socket" else local
    if world > 1:
        dist.init(device=device)

    w = dict(WORKLOADS[args.workload])
    if args.batch and args.batch != w["B"]:
        w["B"] = args.batch
        w["desc"] = w["desc"].split(", T=")[0] + f", T={w['T']}, batch of {args.batch} codeword(s) (--batch)"
    L, M, P, T, B, sigma = w["L"], w["M"], w["P"], w["T"], w["B"], w["sigma"]
    n = n_of(w)
    Pl = P / L * np.ones(L)
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend=args.backend,
                          precision=args.precision, device=device)
    # per-rank synthetic reps: seeds 1000 + rank*B + i (sharded, no overlap)
    seeds = [1000 + rank * B + i for i in range(B)]
    y = synth_y(op, Pl, sigma, seeds)
    op.reserve(B, T)
    op.stage(y, Pl)

    def sync_all():
        op.wait()
        dist.barrier()

    for _ in range(args.warmup):
        op.run(B, T, early_stop=False)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        op.run(B, T, early_stop=False)
    sync_all()
    elapsed = time.perf_counter() - t0
    elapsed = float(dist.allreduce_max(np.array([elapsed]))[0])  # the slowest rank's time

    # per-kernel device times over one eager decode (HIP events on the
    # library's stream), for the roofline of the dominant kernel
    kinds, total_ms = op.profile(B, T, early_stop=False)
    # the roofline's launch duration: each launch of a short eager decode
    # issued REP times back to back between two HIP events on the library's
    # stream (mean = elapsed / REP: kernel + same-stream boundary, without the
    # event packets' own dispatch overhead that a per-launch bracket adds)
    kinds_rep, _ = op.profile(B, min(T, 4), early_stop=False, rep=PROFILE_REP)
    s = 8 if args.precision == "fp64" else 4
    plan = op.plan(B)
    if args.backend == "hadamard":
        G = plan["partials"]  # Ab partials per codeword of the section kernel this batch runs
        wv = op.w
        sk = plan["section_kernel"]
        per = {
            "k_sec": sec_bytes(L, M, n, wv, B, G, s, sk.rstrip("f")),
            "k_row": row_bytes(n, B, G, s),
        }
        if sk.endswith("f"):  # the fused kernel also does the row step (k_row: the last one only)
            per["k_sec"] += per["k_row"]
    elif plan["section_kernel"] == "dense_mfma":
        per = {"k_dense_az": i8_gemm_ops(L, M, n, B, NP_Z), "k_dense_ab": i8_gemm_ops(L, M, n, B, NP_B)}
    else:
        per = {"k_dense_az": gemv_bytes(L, M, n) * B, "k_dense_ab": gemv_bytes(L, M, n) * B,
               "k_dense_den": B * (8 * 4 * L * M + 8 * L * M), "k_row": row_bytes(n, B, 8, s)}
    share = {k: kinds[k][0] * kinds[k][1] for k in per}
    dom = max(share, key=share.get)
    dom_ms = kinds_rep[dom][0]
    mfma = plan["section_kernel"] == "dense_mfma"
    achieved = per[dom] / (dom_ms * 1e-3) / (1e12 if mfma else 1e9)
    peak = I8_PEAK_TOPS if mfma else HBM_PEAK_GBS
    kname = {"k_sec": plan["section_kernel"], "k_row": plan["row_kernel"]}.get(dom, dom)
    # the kernel's name in the rocprofv3 traces (k_gemm_i8 is one template, two products)
    trace_name = {"k_dense_az": "k_gemm_i8_Az", "k_dense_ab": "k_gemm_i8_Ab"}[dom] if mfma else kname
    pmc = load_pmc(f"{args.workload}_{args.backend}_{args.precision}_B{B}", trace_name)
    if mfma:
        kname = "k_gemm_i8 (" + {"k_dense_az": f"A^T z, {NP_Z} digit planes",
                                 "k_dense_ab": f"A beta, {NP_B} digit planes"}[dom] + ")"
    scale = 1e12 if mfma else 1e9
    # headline: the launch duration INSIDE the replayed decode graph (the
    # rocprofv3 graph-trace median of this same bench command, committed under
    # profiles/), where the kernel follows the row kernel's writes on other
    # XCDs; beside it the live HIP-event figure of REP back-to-back launches
    # (inputs still in the caches from the previous launch: a few % faster)
    tag = PROFILE_TAGS.get((args.workload, B, args.backend)) if args.precision == "fp32" else None
    gm = load_graph_median(tag, trace_name) if tag else None
    ev = {"achieved": round(achieved, 1), "frac": round(achieved / peak, 4), "avg_launch_ms": round(dom_ms, 5),
          "timing": f"HIP events on the library stream around {PROFILE_REP} back-to-back launches per kernel, "
                    f"measured live in this run"}
    if gm is not None:
        g_ms = gm[0] * 1e-6
        ach_g = per[dom] / (g_ms * 1e-3) / scale
        head = {"achieved": round(ach_g, 1), "frac": round(ach_g / peak, 4), "avg_launch_ms": round(g_ms, 5),
                "timing": f"in-graph launch duration: median of {gm[1]} graph-replayed launches, rocprofv3 "
                          f"kernel trace of this bench command ({gm[2]})"}
    else:
        head = ev
    roofline = {
        "bound": "mfma" if mfma else "hbm", "kernel": kname, "achieved": head["achieved"], "peak": peak,
        "unit": "TFLOP/s" if mfma else "GB/s", "frac": head["frac"],
        "traffic": None if pmc is None else pmc.get("hbm_bytes_per_launch"),
        ("algorithmic_int8_ops_per_launch" if mfma else "algorithmic_bytes_per_launch"): per[dom],
        **({"ops": "int8 multiply-adds x 2 (TOP/s)"} if mfma else {}),
        "avg_launch_ms": head["avg_launch_ms"], "timing": head["timing"],
        **({"events": ev} if gm is not None else {}),
        "kernel_ms": {k: round(v[0], 5) for k, v in kinds_rep.items() if v[1]},
        "kernel_ms_event_bracketed": {k: round(v[0], 5) for k, v in kinds.items() if v[1]},
        "eager_decode_ms": round(total_ms, 3),
    }

    if kname == "k_secb" and args.precision == "fp32":
        vb = valu_bound(args.workload, kname, head["avg_launch_ms"], plan["cus"])
        if vb is not None:
            roofline["secondary_bound"] = dict(bound="latency", **vb)
    result = {
        "metric": f"decoded codewords/sec (T AMP iters) at L={L},M={M}; achieved HBM GB/s vs roofline",
        "value": round(B * args.steps * world / elapsed, 3),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else "f64",
        "data": "synthetic (RandomState(seed) section indices + N(0, sigma^2) noise, y = A beta0 + w)",
        "config": {"workload": w["desc"], "L": L, "M": M, "n": n, "P": P, "sigma": round(sigma, 6), "T": T,
                   "codewords_per_step_per_gpu": B, "backend": args.backend, "precision": args.precision,
                   "early_stop": False, "parallelism": f"reps sharded over {world} GPU(s)"},
        "roofline": roofline,
    }
    if args.precision == "fp32" and args.backend == "hadamard" and not args.no_fp64:
        # the same workload in binary64 (the reference's precision; the joint
        # decoder's): same seeds, same timing protocol, every rank
        op64 = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="hadamard", precision="fp64",
                                device=device)
        op64.reserve(B, T)
        op64.stage(y, Pl)
        for _ in range(args.warmup):
            op64.run(B, T, early_stop=False)
        op64.wait()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            op64.run(B, T, early_stop=False)
        op64.wait()
        dist.barrier()
        e64 = float(dist.allreduce_max(np.array([time.perf_counter() - t0]))[0])
        result["fp64_leg"] = {"value": round(B * args.steps * world / e64, 3), "unit": "codewords/s",
                              "ms_per_step": round(e64 / args.steps * 1e3, 4), "dtype": "f64",
                              "section_kernel": op64.plan(B)["section_kernel"]}
        del op64
    if rank == 0 and world == 1 and not args.no_dense:
        try:
            result["dense_gemv"] = dense_gemv_probe(device)
        except Exception as e:  # report, never hide
            result["dense_gemv"] = {"error": str(e)}
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(w, args.cpu_procs or None)
        result["cpu_baseline"]["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.finalize()


if __name__ == "__main__":
    main()
