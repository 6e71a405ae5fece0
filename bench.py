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

Beside the headline the default line carries the other BASELINE configs,
each timed on every rank with its own roofline: `fp64_leg` (configs[1] in
binary64), `batched_legs` (configs[2] C3 B = 256 in binary32 / binary64,
configs[3] C4 B = 256), `mc_stream` (configs[3]'s 10 k-rep Monte-Carlo sweep,
one refilled stream, with its own CPU baseline) and `joint_leg` (configs[4],
the joint AMP<->BP step).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
I8_PEAK_TOPS = 5000.0  # dense int8 MFMA: 2x the ~2.5 PF bf16 rate per clock (MI355X_MICROARCH.md, Matrix cores)
F32_PEAK_TFLOPS = 157.3  # f32-input MFMA (v_mfma_f32_32x32x2_f32) = the f32 vector peak (MI355X_MICROARCH.md)
F64_PEAK_TFLOPS = 78.6   # f64 MFMA (v_mfma_f64_16x16x4_f64): half the f32 rate
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


def synth_y(op, Pl, sigma, seeds, with_idx=False):
    """Synthetic reps: RandomState(seed) -> L indices in [0, M),
    then N(0, σ²) noise; x = A β₀ on the device.  with_idx: also the (B, L)
    transmitted section indices."""
    from sparc_ldpc_amd.harness import draw_reps
    L, M, n = op.L, op.M, op.n
    c = np.sqrt(n * Pl)
    B = len(seeds)
    # RandomState(seed).randint(0, M, L) then .randn(n) * sigma, drawn natively
    # (bit for bit NumPy's legacy generator, tests/test_host.py)
    sent, noise = draw_reps(seeds, L, M, n, sigma)
    beta0 = np.zeros((B, L * M))
    for i in range(B):
        beta0[i, np.arange(L) * M + sent[i]] = c
    y = op.Ab_batch(beta0) + noise
    return (y, sent) if with_idx else y


def sec_bytes(L, M, n, w, B, G, s, kernel="k_sec4"):
    """Algorithmic bytes of one section-kernel launch: the bucket
    and Ab tables once (uint16 per slot and per section-row; k_sec43 packs a
    section triple's Ab entries into one uint32 per row), z once per codeword,
    β read + write, Ab partials written."""
    tables = 2 * L * w + (4 * n * G if kernel == "k_sec43" else 2 * L * n)
    return tables + B * (n * s + 2 * L * M * s + G * n * s)


def row_bytes(n, B, G, s):
    """k_row: Ab partials read, y read, z read + write."""
    return B * (G * n * s + 3 * n * s)


def gemv_bytes(L, M, n, s=4):
    """4·n·L·M + 4·(n + L·M) per fp32 GEMV (s = 8: binary64)."""
    return s * n * L * M + s * (n + L * M)


def i8_gemm_ops(L, M, n, B, planes):
    """Algorithmic int8 multiply-adds x 2 of one dense GEMM on the matrix cores:
    `planes` digit planes of B codewords against the n x L·M ±1 matrix (the
    fp32-equivalent GEMM of SURVEY §8d is 2·n·L·M·B flops: this counts each
    digit plane's product, the work the int8 MFMA actually does)."""
    return 2 * planes * B * n * L * M


def _cpu_worker(args, barrier, q):
    """One host process: build the oracle operator (untimed), wait at the
    barrier for every other process, then time Tsample AMP iterations of one
    codeword; puts ("ok", start, end), or ("err", message) on any failure (a
    failing worker breaks the barrier, so no sibling waits for it)."""
    try:
        L, M, n, P, sigma, Tsample, seed = args
        os.environ["OMP_NUM_THREADS"] = "1"
        from oracle import amp_oracle as orc
        Ab, Az, _ = orc.sparc_transforms(L, M, n)
        Pl = P / L * np.ones(L)
        _, y = orc.rep_inputs(L, M, n, Pl, sigma, Ab, seed)
        barrier.wait(timeout=600)  # every process starts its timed loop together
        t0 = time.time()
        beta, _ = orc._amp_core(y, Pl, L, M, Tsample, Ab, Az, None, early_stop=False)  # exactly Tsample iterations
        t1 = time.time()
        # the decisions of the GPU's first codeword (the same seed), after the timed loop
        dec = orc.section_argmax(beta, L, M).astype(np.int32) if seed == 1000 else None
        q.put(("ok", t0, t1, dec))
    except BaseException as e:  # noqa: BLE001 (reported to the parent, never swallowed)
        try:
            barrier.abort()
        finally:
            q.put(("err", f"{type(e).__name__}: {e}", 0.0, None))


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


def cpu_baseline(w, procs=None, Tsample=None, gpu_decisions=None):
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
    ps = [ctx.Process(target=_cpu_worker, args=((L, M, n, P, sigma, Tsample, 1000 + i), barrier, q), daemon=True)
          for i in range(procs)]
    for p in ps:
        p.start()
    spans, errs, dec = [], [], None
    try:
        for _ in ps:
            kind, a, b, d = q.get(timeout=900)
            if kind == "ok":
                spans.append((a, b))
                dec = d if d is not None else dec
            else:
                errs.append(a)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    if errs:
        raise RuntimeError(f"cpu_baseline: {len(errs)} of {procs} workers failed: {errs[0]}")
    wall = max(e for _, e in spans) - min(s for s, _ in spans)
    per_core = float(np.mean([e - s for s, e in spans])) / Tsample
    agree = None
    if dec is not None and gpu_decisions is not None and Tsample == T:
        # the oracle's decisions for seed 1000 (the GPU's codeword 0) after the same T iterations
        agree = {"seed": 1000, "sections": int(dec.size),
                 "sections_differing": int(np.count_nonzero(np.asarray(gpu_decisions).reshape(-1) != dec))}
    return {
        "value": procs * Tsample / wall / T, "unit": "codewords/s", "cores": procs, "kind": "port",
        "cpu": desc, **({"decisions_vs_gpu_codeword0": agree} if agree is not None else {}),
        "sample": f"oracle amp() fp64 NumPy (the reference algorithm), {procs} single-threaded processes x "
                  f"1 codeword x {Tsample} iterations (L={L} M={M} n={n}) in {wall:.1f} s wall, "
                  f"scaled to T={T} iterations/codeword; {per_core * 1e3:.1f} ms/iteration/process",
    }


def dense_gemv_probe(device):
    """North-star GEMVs at L=768 M=512 R=5/6 (n=8294), one codeword, on a
    materialised fp32 A (13.05 GB) streamed once per product: the Hadamard
    design's matrix (dense backend) and an i.i.d. Gaussian design generated on
    the device (matrix backend, sa_create_matrix_random; the north star's
    "Gaussian design-matrix GEMVs"); per-kernel event timing."""
    import sparc_ldpc_amd as sp
    L, M, R, P = 768, 512, 5 / 6, 1.8
    n = int(L * np.log2(M) / R)
    Pl = P / L * np.ones(L)
    gb = gemv_bytes(L, M, n) / 1e9
    out = {"workload": "L=768 M=512 R=5/6 single codeword, dense fp32 A", "bytes_per_gemv": gemv_bytes(L, M, n)}
    for tag, mk in (("hadamard_A", lambda: sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense",
                                                               precision="fp32", device=device)),
                    ("gaussian_A", lambda: sp.SparcOperator.from_random(L, M, n, seed=1, precision="fp32",
                                                                        device=device))):
        op = mk()
        y = synth_y(op, Pl, 0.6, [7])
        op.reserve(1, 4)
        op.stage(y, Pl)
        op.profile(1, 2, early_stop=False)  # warm
        kinds, _ = op.profile(1, 2, early_stop=False, rep=4)
        res = {}
        for k in ("k_dense_az", "k_dense_ab"):
            ms = kinds[k][0]
            res[k] = {"ms": round(ms, 4), "achieved_GBs": round(gb / (ms * 1e-3), 1),
                      "frac": round(gb / (ms * 1e-3) / HBM_PEAK_GBS, 4)}
        out[tag] = res
        del op
    # the round-3 keys: the Hadamard design's GEMVs
    out.update(out["hadamard_A"])
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


PROFILE_TAGS = {  # (workload, codewords, backend, precision) -> scripts/profile_set.sh tag
    ("c2", 1, "hadamard", "fp32"): "c2", ("c4", 1, "hadamard", "fp32"): "c4b1",
    ("c3", 256, "hadamard", "fp32"): "c3", ("c4", 256, "hadamard", "fp32"): "c4",
    ("c3", 256, "dense", "fp32"): "c3dense", ("c4", 1, "dense", "fp32"): "dense_l768",
    ("c2", 1, "hadamard", "fp64"): "c2f64", ("c3", 256, "hadamard", "fp64"): "c3f64",
    ("c4", 256, "hadamard", "fp64"): "c4f64", ("c2", 1, "matrix", "fp32"): "c2matrix",
    ("c3", 256, "matrix", "fp32"): "c3matrix",
}


def load_trace(tag, kernel):
    """The graph-replay durations of `kernel` from the newest committed
    profiles/<round>_<tag>_graph_trace.txt (scripts/graph_trace.py): median
    in-graph duration and exclusive duration (ns), launch count, the sources
    hash the profile was taken of, and the file; or None."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{tag}_graph_trace.txt")))
    if not files:
        return None
    src, hit = None, None
    for line in open(files[-1]):
        if line.startswith("sources sha256 "):
            src = line.split()[-1]
        m = re.match(r"(\S+)\s+n=\s*(\d+)\s+duration median\s+(\d+) ns", line)
        if m and m.group(1) == kernel:
            ex = re.search(r"exclusive median\s+(\d+) ns", line)
            hit = (float(m.group(3)), float(ex.group(1)) if ex else None, int(m.group(2)))
    if hit is None:
        return None
    return {"duration_ns": hit[0], "exclusive_ns": hit[1], "launches": hit[2], "sources": src,
            "file": os.path.relpath(files[-1], ROOT)}


def load_pmc(workload, kernel):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        return d.get(workload, {}).get(kernel)
    except (OSError, ValueError):
        return None


def measure_roofline(op, workload, L, M, n, B, T, precision, ms_per_step):
    """Roofline of the dominant kernel of one decode of B codewords.

    `achieved` = algorithmic bytes (ops) per launch / the kernel's launch
    duration.  The headline duration is the kernel's in-graph duration: the
    graph-replay median of the committed rocprofv3 kernel trace of the same
    command when that profile was taken of these sources (`trace`), else the
    LIVE dispatch-bound HIP-event time of this run (`dispatch`: an eager decode
    with every loop kernel launched through hipExtLaunchKernel with a start /
    stop event pair bound to its own dispatch packet, on the library's stream;
    the mean over the decode's T launches).  Beside it: the live dispatch
    figure (`frac_dispatch`), the repeated-launch figure (`frac_events`: each
    launch issued PROFILE_REP times back to back between one event pair; the
    repeats re-read inputs their predecessor left in the caches, so this is
    an optimistic figure), PMC HBM traffic (only when taken of these sources)
    and a consistency check T x (sum of per-iteration kernel times) <=
    ms_per_step."""
    from sparc_ldpc_amd._lib import source_hash
    kinds, total_ms = op.profile(B, T, early_stop=False)
    kinds_rep, _ = op.profile(B, min(T, 4), early_stop=False, rep=PROFILE_REP)
    kinds_disp, disp_total_ms = op.profile(B, T, early_stop=False, rep=0)
    s = 8 if precision == "fp64" else 4
    plan = op.plan(B)
    mfma = plan["section_kernel"] in ("dense_mfma", "matrix_mfma")
    fmfma = plan["section_kernel"] == "matrix_mfma"
    if op.backend == "hadamard":
        G = plan["partials"]
        per = {"k_sec": sec_bytes(L, M, n, op.w, B, G, s, plan["section_kernel"]), "k_row": row_bytes(n, B, G, s)}
    elif fmfma:  # f32 / f64 MFMA GEMMs of a caller's matrix: 2 n L M B flops per product
        per = {"k_dense_az": 2 * n * L * M * B, "k_dense_ab": 2 * n * L * M * B}
    elif mfma:
        per = {"k_dense_az": i8_gemm_ops(L, M, n, B, NP_Z), "k_dense_ab": i8_gemm_ops(L, M, n, B, NP_B)}
    else:
        per = {"k_dense_az": gemv_bytes(L, M, n, s) * B, "k_dense_ab": gemv_bytes(L, M, n, s) * B,
               "k_dense_den": B * (8 * s * L * M + 2 * s * L * M), "k_row": row_bytes(n, B, 8, s)}
    share = {k: kinds_disp[k][0] * kinds_disp[k][1] for k in per}
    dom = max(share, key=share.get)
    scale = 1e12 if mfma else 1e9
    peak = (F64_PEAK_TFLOPS if precision == "fp64" else F32_PEAK_TFLOPS) if fmfma else (
        I8_PEAK_TOPS if mfma else HBM_PEAK_GBS)

    def frac_of(ms):
        return round(per[dom] / (ms * 1e-3) / scale / peak, 4) if ms and ms > 0 else None

    kname = {"k_sec": plan["section_kernel"], "k_row": plan["row_kernel"]}.get(dom, dom)
    if fmfma:
        trace_name = {"k_dense_az": "k_gemm_f_Az", "k_dense_ab": "k_gemm_f_Ab"}[dom]
        kname = f"k_gemm_f<{'double' if precision == 'fp64' else 'float'}> (" + {
            "k_dense_az": "A^T z", "k_dense_ab": "A beta"}[dom] + ")"
    elif mfma:
        trace_name = {"k_dense_az": "k_gemm_i8_Az", "k_dense_ab": "k_gemm_i8_Ab"}[dom]
        kname = "k_gemm_i8 (" + {"k_dense_az": f"A^T z, {NP_Z} digit planes",
                                 "k_dense_ab": f"A beta, {NP_B} digit planes"}[dom] + ")"
    else:
        trace_name = kname
    src = source_hash()
    disp_ms = kinds_disp[dom][0]
    ev_ms = kinds_rep[dom][0]
    # the trace of the same command, if it was taken of these sources
    tag = PROFILE_TAGS.get((workload, B, op.backend, precision))
    tr = load_trace(tag, trace_name) if tag else None
    matched = tr is not None and tr["sources"] == src
    if matched:
        dom_ms, timing = tr["duration_ns"] * 1e-6, (
            f"in-graph duration: graph-replay median of {tr['launches']} launches in {tr['file']} (rocprofv3 "
            f"kernel trace of this command, taken of these sources {src})")
    else:
        dom_ms, timing = disp_ms, ("live: HIP start / stop events bound to each launch's own dispatch "
                                   "(hipExtLaunchKernel) in an eager decode of this run, mean over its launches")
    achieved = per[dom] / (dom_ms * 1e-3) / scale
    # consistency: the loop kernels' dispatch times per iteration, T times
    per_iter = sum(kinds_disp[k][0] * round(kinds_disp[k][1] / T) for k in kinds_disp if kinds_disp[k][1] >= T)
    roof = {
        "bound": "mfma" if mfma else "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": peak,
        "unit": "TFLOP/s" if mfma else "GB/s", "frac": round(achieved / peak, 4), "traffic": None,
        (("algorithmic_flops_per_launch" if fmfma else "algorithmic_int8_ops_per_launch") if mfma
         else "algorithmic_bytes_per_launch"): per[dom],
        **({"ops": ("multiply-adds x 2 (TFLOP/s)" if fmfma else "int8 multiply-adds x 2 (TOP/s)")} if mfma else {}),
        "avg_launch_ms": round(dom_ms, 5),
        "timing": timing,
        "frac_dispatch": frac_of(disp_ms),
        "dispatch_launch_ms": round(disp_ms, 5),
        "frac_events": frac_of(ev_ms),
        "events_launch_ms": round(ev_ms, 5),
        "events_timing": f"repeated-launch timing: HIP events around {PROFILE_REP} back-to-back launches of each "
                         f"kernel (kernel + same-stream boundary; repeats re-read what their predecessor cached)",
        "kernel_ms_dispatch": {k: round(v[0], 5) for k, v in kinds_disp.items() if v[1]},
        "kernel_ms_events": {k: round(v[0], 5) for k, v in kinds_rep.items() if v[1]},
        "kernel_ms_event_bracketed": {k: round(v[0], 5) for k, v in kinds.items() if v[1]},
        "eager_decode_ms": round(total_ms, 3),
        "consistency": {"per_iteration_ms": round(per_iter, 5), "T": T, "T_x_per_iteration_ms": round(T * per_iter, 4),
                        "ms_per_step": ms_per_step, "ok": bool(T * per_iter <= ms_per_step * 1.02)},
        "sources": src,
    }
    if tr is not None:
        t = {"file": tr["file"], "profile_matches_build": matched, "sources": tr["sources"],
             "launches": tr["launches"], "in_graph_duration_ms": round(tr["duration_ns"] * 1e-6, 5),
             "frac_in_graph": frac_of(tr["duration_ns"] * 1e-6)}
        if tr["exclusive_ns"]:
            ex_ms = tr["exclusive_ns"] * 1e-6
            t["exclusive_ms"] = round(ex_ms, 5)
            t["frac_exclusive"] = frac_of(ex_ms)
        if matched:
            t["live_dispatch_over_trace"] = round(disp_ms / (tr["duration_ns"] * 1e-6), 4)
        roof["trace"] = t
    pmc = load_pmc(f"{workload}_{op.backend}_{precision}_B{B}", trace_name)
    if pmc is not None:
        if pmc.get("sources") == src:
            roof["traffic"] = pmc.get("hbm_bytes_per_launch")
            roof["traffic_over_algorithmic"] = round(pmc["hbm_bytes_per_launch"] / per[dom], 3) if not mfma else None
        else:
            roof["traffic_stale"] = {"hbm_bytes_per_launch": pmc.get("hbm_bytes_per_launch"),
                                     "sources": pmc.get("sources"), "note": "PMC pass of other sources: not used"}
    if op.backend == "hadamard":
        # the whole iteration against the bytes it cannot avoid (VERDICT r05:
        # the Ab partials are the two-kernel design's own hand-off, counted in
        # `frac` but not here): section + row kernel in-graph (or dispatch) times
        tr_row = load_trace(tag, plan["row_kernel"]) if tag else None
        sec_ms = (tr["duration_ns"] if matched and dom == "k_sec" else None)
        row_ms = (tr_row["duration_ns"] if tr_row is not None and tr_row["sources"] == src else None)
        sec_ms = sec_ms * 1e-6 if sec_ms else kinds_disp["k_sec"][0]
        row_ms = row_ms * 1e-6 if row_ms else kinds_disp["k_row"][0]
        G = plan["partials"]
        partials = 2 * B * G * n * s
        minimal = per["k_sec"] + per["k_row"] - partials
        roof["iteration"] = {
            "minimal_bytes": minimal, "partials_bytes": partials, "ms": round(sec_ms + row_ms, 5),
            "frac_minimal": round(minimal / ((sec_ms + row_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": "section + row kernel of one iteration against the tables, z, y and beta bytes it must move "
                    "(the Ab partials written by the section kernel and read by the row kernel excluded)"}
        if B >= 4:
            # SURVEY §8(d)'s roofline for the batched case: the dense GEMM
            # formulation's 4 n L M B flops per iteration (A beta and A^T z),
            # at the rate the factorised operator delivers them
            fl = 4.0 * n * L * M * B
            roof["dense_equivalent"] = {
                "flops_per_iteration": fl, "tflops": round(fl / ((sec_ms + row_ms) * 1e-3) / 1e12, 1),
                "over_f32_mfma_peak": round(fl / ((sec_ms + row_ms) * 1e-3) / 1e12 / F32_PEAK_TFLOPS, 2),
                "note": "the n x (L M) dense products the reference's operator stands for, per second of this "
                        "iteration, against the fp32 MFMA dense peak (the factorised operator never forms them)"}
    if kname == "k_secb" and precision == "fp32":
        vb = valu_bound(workload, kname, dom_ms, plan["cus"])
        if vb is not None:
            roof["secondary_bound"] = dict(bound="latency", **vb)
    return roof


def timed_steps(op, B, T, steps, warmup, sent=None, decide=True):
    """Warmup, then exactly `steps` decoded steps between barrier + device sync
    on both sides.  A step is one decode of the staged batch (sa_run, T
    iterations) plus its decision: the section argmax on the device and the
    copy of the (B, L) indices into a pinned host slot (sa_decide_async),
    which the host collects one step behind (sa_decide_collect) while the next
    decode runs, and scores against the transmitted indices `sent`; the last
    step's decisions are collected inside the timed region.  decide=False
    times the decodes alone.  Returns a dict: this rank's seconds, the max
    over ranks, the timed region's perf_counter stamps and the section errors
    of the timed steps' decisions."""
    from sparc_ldpc_amd import dist
    S = 2

    def run_steps(k0, count, score):
        errs, decided, last = 0, 0, None
        for k in range(k0, k0 + count):
            op.run(B, T, early_stop=False)
            if decide:
                op.decide_async(B, k % S)
                if k > k0:
                    idx = op.decide_collect(B, (k - 1) % S)
                    if score and sent is not None:
                        errs += int(np.count_nonzero(idx != sent))
                    decided += 1
        if decide and count:
            idx = op.decide_collect(B, (k0 + count - 1) % S)
            if score and sent is not None:
                errs += int(np.count_nonzero(idx != sent))
            decided += 1
            last = idx
        return errs, decided, last

    run_steps(0, warmup, False)
    op.wait()
    dist.barrier()
    t0 = time.perf_counter()
    errs, decided, last = run_steps(warmup, steps, True)
    op.wait()
    dist.barrier()
    t1 = time.perf_counter()
    mine = t1 - t0
    return {"mine": mine, "elapsed": float(dist.allreduce_max(np.array([mine]))[0]), "t0": t0, "t1": t1,
            "section_errors": errs, "decided_steps": decided, "last_decisions": last}


# The batched configurations timed beside the headline in the default line
# (VERDICT r05 item 2): BASELINE configs[2] in binary32 and binary64, configs[3]
# at its benched batch, and configs[3]'s 10 k-rep Monte-Carlo sweep as one
# refilled stream (sa_mc_run).
LEGS = (("c3", "c3", "fp32"), ("c3_fp64", "c3", "fp64"), ("c4", "c4", "fp32"))
MC_SIGMAS = tuple(float(v) for v in np.linspace(0.8, 0.4, 10))  # soft_hard_plot's sigma points (sparc_ldpc.py:1318)
MC_REPS_PER_POINT = 1000


def batched_leg(sp, workload, precision, args, device, rank, world, make_op=None):
    """One batched configuration with the headline's protocol (timed_steps:
    decode + decision per step, max over ranks) and its own roofline."""
    w = WORKLOADS[workload]
    L, M, P, T, B, sigma = w["L"], w["M"], w["P"], w["T"], w["B"], w["sigma"]
    n = n_of(w)
    Pl = P / L * np.ones(L)
    op = (make_op(L, M, n, "hadamard", precision, device, None) if make_op is not None else
          sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=precision, device=device))
    y, sent = synth_y(op, Pl, sigma, [1000 + rank * B + i for i in range(B)], with_idx=True)
    op.reserve(B, T)
    op.stage(y, Pl)
    ts = timed_steps(op, B, T, args.leg_steps, args.leg_warmup, sent)
    ms = round(ts["elapsed"] / args.leg_steps * 1e3, 4)
    plan = op.plan(B)
    leg = {"workload": w["desc"], "value": round(B * args.leg_steps * world / ts["elapsed"], 3),
           "unit": "codewords/s", "ms_per_step": ms, "steps": args.leg_steps, "warmup": args.leg_warmup,
           "dtype": "f32" if precision == "fp32" else "f64", "codewords_per_step_per_gpu": B,
           "section_kernel": plan["section_kernel"], "row_kernel": plan["row_kernel"],
           "section_errors_rank0": ts["section_errors"], "decided_steps_rank0": ts["decided_steps"],
           "roofline": measure_roofline(op, workload, L, M, n, B, T, precision, ms)}
    del op
    return leg


def mc_stream_leg(sp, args, device, rank, world, make_op=None):
    """configs[3]'s Monte-Carlo sweep (L=768 M=512 R=5/6 P=1.8, T=64, the exact-
    tau stop on): MC_REPS_PER_POINT reps at each of the 10 sigma points, rep j
    of point i seeded i * 100000 + j, sharded over the ranks; drawn natively
    on the host cores, then decoded on the device as ONE stream through 256
    refilled slots (sa_mc_run).  value = all ranks' reps / the slowest rank's
    device time of the stream (encode of every rep, decode, decisions, bit
    errors); the host draws and the staging are reported beside it."""
    from sparc_ldpc_amd import dist
    from sparc_ldpc_amd.harness import draw_reps
    w = WORKLOADS["c4"]
    L, M, P, T = w["L"], w["M"], w["P"], w["T"]
    n = n_of(w)
    Pl = P / L * np.ones(L)
    op = (make_op(L, M, n, "hadamard", "fp32", device, None) if make_op is not None else
          sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp32", device=device))
    if not op.mc_supported(256):
        return {"error": "the operator does not support the refilled stream"}
    seeds = [[j for j in range(i * 100000, i * 100000 + MC_REPS_PER_POINT) if j % world == rank]
             for i in range(len(MC_SIGMAS))]
    cnt = [len(s) for s in seeds]
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(int)
    idx = np.empty((off[-1], L), dtype=np.int32)
    noise = np.empty((off[-1], n))
    t0 = time.perf_counter()
    for i, sg in enumerate(MC_SIGMAS):
        draw_reps(seeds[i], L, M, n, sg, idx=idx[off[i]:off[i + 1]], noise=noise[off[i]:off[i + 1]])
    t1 = time.perf_counter()
    op.reserve(256, T)
    op.stage_power(256, Pl)
    op.mc_stage(idx, noise)
    t2 = time.perf_counter()
    op.mc_run(256, T, decisions=False)  # warm: tables, graphs
    dist.barrier()
    t3 = time.perf_counter()
    _, its, errs, dev_ms = op.mc_run(256, T, decisions=False)
    t4 = time.perf_counter()
    dev_max = float(dist.allreduce_max(np.array([dev_ms]))[0])
    tot = dist.allreduce_sum(np.array([off[-1], int(errs.sum()), int(its.sum()),
                                       int(np.minimum(its + 1, T).sum())], dtype=np.int64))
    per_point = dist.allreduce_sum(np.array([[int(errs[off[i]:off[i + 1]].sum()) for i in range(len(MC_SIGMAS))],
                                             cnt], dtype=np.int64))
    del op
    return {
        "workload": f"BASELINE configs[3]: L={L} M={M} R=5/6 P={P}, T={T}, exact-tau stop on, "
                    f"{MC_REPS_PER_POINT} reps x {len(MC_SIGMAS)} sigma points (linspace(0.8, 0.4, 10)), "
                    f"one refilled stream of 256 slots per GPU",
        "value": round(float(tot[0]) / (dev_max * 1e-3), 1), "unit": "Monte-Carlo reps/s",
        "reps": int(tot[0]), "stream_device_ms_max_over_ranks": round(dev_max, 3),
        "stream_wall_ms_rank0": round((t4 - t3) * 1e3, 3),
        "codeword_iterations": int(tot[2]), "slot_iterations": int(tot[3]),
        "codeword_iterations_per_s": round(float(tot[2]) / (dev_max * 1e-3), 1),
        "host_draw_ms_rank0": round((t1 - t0) * 1e3, 2), "stage_ms_rank0": round((t2 - t1) * 1e3, 2),
        "ber_per_point": [round(float(e) / (c * L * np.log2(M)), 8) for e, c in zip(per_point[0], per_point[1])],
        "note": "codeword_iterations: the sum of the stop indices (T when a rep ran out); slot_iterations: "
                "the section / row steps the slots ran (min(stop index + 1, T) per rep)",
    }


def mc_cpu_baseline(leg, procs=None, Tsample=8):
    """configs[3]'s CPU baseline: the oracle's AMP iterations at L=768 M=512
    R=5/6 on the host cores (cpu_baseline: `procs` single-threaded processes,
    Tsample iterations each after a barrier), scaled to the reps the stream
    decoded: reps/s = iterations/s / (the stream's slot-iterations per rep,
    the same algorithm's per-rep work, the exact-tau stop included)."""
    w = dict(WORKLOADS["c4"])
    per_rep = leg["slot_iterations"] / leg["reps"]
    base = cpu_baseline(w, procs, Tsample)
    iters_s = base["value"] * w["T"]  # cpu_baseline scales to T iterations per codeword
    return {"value": iters_s / per_rep, "unit": "Monte-Carlo reps/s", "cores": base["cores"], "kind": "port",
            "cpu": base["cpu"], "gpu_over_cpu": round(leg["value"] / (iters_s / per_rep), 1),
            "sample": f"oracle AMP iterations fp64 NumPy at L=768 M=512 n={n_of(w)}: {base['sample']}; "
                      f"as reps at the stream's {per_rep:.2f} iterations per rep"}


def joint_leg(args, device, rank, world):
    """BASELINE configs[4] (scripts/bench_joint.py's measurement, in this
    process): the joint AMP<->BP soft-exchange step, 256 codewords per GPU as
    two concurrent slices, binary64 AMP, rep for rep identical to one decoder
    over the whole batch; its own roofline.  The CPU leg of configs[4] is left
    to scripts/bench_joint.py (minutes of host work)."""
    import importlib.util
    from sparc_ldpc_amd import joint
    spec = importlib.util.spec_from_file_location("bench_joint", os.path.join(ROOT, "scripts", "bench_joint.py"))
    bj = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bj)
    gc.collect()  # the earlier legs' contexts (and streams) gone first
    ns = argparse.Namespace(steps=args.joint_steps, warmup=1, batch=256, ebno=6.888888888888889, soft_iter=2,
                            precision="fp64", plan="", no_cpu=True, cpu_procs=0, no_ref=False, no_twin=False,
                            parts=2)
    try:
        res = bj.measure(ns, device=device, rank=rank, world=world)
    finally:
        while joint._JD_CACHE:  # release the decoders' device memory and threads
            joint._evict(joint._JD_CACHE.popitem(last=False)[1])
    keep = ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "config", "identical_to_one_decoder",
            "roofline", "bp", "errors", "step_share_ms")
    return {k: res[k] for k in keep if k in res}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--backend", default="hadamard", choices=["hadamard", "dense", "matrix"],
                    help="matrix: an i.i.d. Gaussian N(0, 1/n) design generated on the device")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--batch", type=int, default=0, help="override codewords per step")
    ap.add_argument("--plan", default="", help="comma-separated plan options (sa_create_ex), e.g. ONE_PASS")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0)
    ap.add_argument("--cpu-iters", type=int, default=0,
                    help="AMP iterations per CPU-baseline process (default: T, a whole decode)")
    ap.add_argument("--no-fp64", action="store_true", help="skip the binary64 leg of an fp32 run")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the batched legs (configs[2] fp32 / fp64, configs[3], the configs[3] Monte-Carlo "
                         "stream) of the default configs[1] line")
    ap.add_argument("--leg-steps", type=int, default=10)
    ap.add_argument("--leg-warmup", type=int, default=2)
    ap.add_argument("--joint-steps", type=int, default=3, help="timed steps of the configs[4] joint leg (0: skip it)")
    args = ap.parse_args(argv)
    if args.plan and args.backend == "matrix":
        # the device-generated Gaussian design (sa_create_matrix_random) takes
        # no plan options: refuse rather than ignore them
        ap.error("--plan applies to the hadamard / dense backends, not --backend matrix")
    return args


def main(argv=None, make_op=None):
    """The bench; make_op(L, M, n, backend, precision, device, plan) replaces
    the device operator (tests/test_bench_host.py drives the whole N-rank flow
    on the CPU with a stand-in; the bench itself never passes one)."""
    args = parse_args(argv)
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
    ndev = sp.load_library().sa_device_count() if make_op is None else 1
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
    plan = [p for p in args.plan.split(",") if p] or None
    if make_op is not None:
        op = make_op(L, M, n, args.backend, args.precision, device, plan)
    elif args.backend == "matrix":
        op = sp.SparcOperator.from_random(L, M, n, seed=0, precision=args.precision, device=device)
        w["desc"] += "; i.i.d. Gaussian N(0, 1/n) design (device-generated), not the Hadamard operator"
    else:
        op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend=args.backend,
                              precision=args.precision, device=device, plan=plan)
    # per-rank synthetic reps: seeds 1000 + rank*B + i (sharded, no overlap)
    seeds = [1000 + rank * B + i for i in range(B)]
    y, sent = synth_y(op, Pl, sigma, seeds, with_idx=True)
    op.reserve(B, T)
    op.stage(y, Pl)

    ts = timed_steps(op, B, T, args.steps, args.warmup, sent)
    mine, elapsed = ts["mine"], ts["elapsed"]
    # every rank's own rate (weak scaling: the spread shows a slow GPU)
    times = dist.allreduce_sum(np.eye(world)[rank] * mine) if world > 1 else np.array([mine])
    errs = dist.allreduce_sum(np.array([ts["section_errors"], ts["decided_steps"]], dtype=np.float64))
    ms_per_step = round(elapsed / args.steps * 1e3, 4)
    # the decodes alone (no decision), same protocol: the round-4 definition of a step
    ts0 = timed_steps(op, B, T, args.steps, min(args.warmup, 1), decide=False)
    roofline = measure_roofline(op, args.workload, L, M, n, B, T, args.precision, ms_per_step)
    result = {
        "metric": f"decoded codewords/sec (T AMP iters) at L={L},M={M}; achieved HBM GB/s vs roofline",
        "value": round(B * args.steps * world / elapsed, 3),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else "f64",
        "data": "synthetic (RandomState(seed) section indices + N(0, sigma^2) noise, y = A beta0 + w)",
        "config": {"workload": w["desc"], "L": L, "M": M, "n": n, "P": P, "sigma": round(sigma, 6), "T": T,
                   "codewords_per_step_per_gpu": B, "backend": args.backend, "precision": args.precision,
                   "early_stop": False, "parallelism": f"reps sharded over {world} GPU(s)",
                   **({"plan": args.plan} if args.plan else {})},
        "decisions": {"step": "sa_run (T iterations) + sa_decide_async (section argmax on the device, B x L int32 "
                              "copied to a pinned host slot) + sa_decide_collect on the host, one step behind the "
                              "decode in flight; the last step's decisions collected inside the timed region",
                      "decided_steps": int(errs[1]), "section_errors": int(errs[0]),
                      "section_error_rate": round(float(errs[0]) / max(1.0, float(errs[1]) * B * L), 8),
                      "note": "configs[1]'s channel is the reference's amp_test.py:167-169 point (snr 10 dB in its "
                              "20 log10 convention: P / sigma^2 = 3.16, capacity 1.03 b/use at R = 1), where plain "
                              "AMP leaves many sections wrong (the reference studies initialisations there); "
                              "cpu_baseline.decisions_vs_gpu_codeword0 holds the oracle's decisions of codeword 0 "
                              "against these"},
        "decode_only": {"value": round(B * args.steps * world / ts0["elapsed"], 3),
                        "ms_per_step": round(ts0["elapsed"] / args.steps * 1e3, 4),
                        "note": "sa_run alone, beta left on the device (no decision)"},
        "roofline": roofline,
    }
    # the headline's context (and its HIP stream) goes before the legs: a
    # process has GPU_MAX_HW_QUEUES (4) hardware queues, and the joint leg's
    # four streams (two AMP slices, two BP contexts) overlap only on queues of
    # their own (sharing one with a live idle stream: 2.05 k against 2.35 k cw/s)
    del op
    gc.collect()
    if world > 1:
        rates = B * args.steps / np.asarray(times)
        result["per_rank"] = {"value_min": round(float(rates.min()), 3), "value_max": round(float(rates.max()), 3),
                              "ms_per_step": [round(float(t) / args.steps * 1e3, 4) for t in times]}
    if args.precision == "fp32" and args.backend == "hadamard" and not args.no_fp64:
        # the same workload in binary64 (the reference's precision; the joint
        # decoder's): same seeds, same timing protocol, every rank, with its
        # own live roofline
        op64 = (make_op(L, M, n, "hadamard", "fp64", device, None) if make_op is not None else
                sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="hadamard", precision="fp64",
                                 device=device))
        op64.reserve(B, T)
        op64.stage(y, Pl)
        t64 = timed_steps(op64, B, T, args.steps, args.warmup, sent)
        e64 = t64["elapsed"]
        ms64 = round(e64 / args.steps * 1e3, 4)
        result["fp64_leg"] = {"value": round(B * args.steps * world / e64, 3), "unit": "codewords/s",
                              "ms_per_step": ms64, "dtype": "f64", "section_errors_rank0": t64["section_errors"],
                              "section_kernel": op64.plan(B)["section_kernel"],
                              "roofline": measure_roofline(op64, args.workload, L, M, n, B, T, "fp64", ms64)}
        del op64
    if args.workload == "c2" and args.backend == "hadamard" and args.precision == "fp32" and not args.no_legs \
            and not args.batch:
        # the batched configurations, every rank, each with its own roofline
        legs = {}
        for tag, wl, prec in LEGS:
            legs[tag] = batched_leg(sp, wl, prec, args, device, rank, world, make_op)
        result["batched_legs"] = legs
        if make_op is None:
            result["mc_stream"] = mc_stream_leg(sp, args, device, rank, world)
            if args.joint_steps > 0:
                result["joint_leg"] = joint_leg(args, device, rank, world)
    if rank == 0 and not args.no_dense:
        # after the timed region, on rank 0's GPU: the N-rank line carries the
        # dense GEMV probe as well
        try:
            result["dense_gemv"] = dense_gemv_probe(device)
        except Exception as e:  # report, never hide
            result["dense_gemv"] = {"error": str(e)}
    if rank == 0 and not args.no_cpu:
        # after the timed region (every rank), on rank 0's host cores: the
        # N-rank line carries its own CPU baseline
        result["cpu_baseline"] = cpu_baseline(w, args.cpu_procs or None, args.cpu_iters or None,
                                              None if ts["last_decisions"] is None else ts["last_decisions"][0])
        result["cpu_baseline"]["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
        if "reps" in result.get("mc_stream", {}):
            result["mc_stream"]["cpu_baseline"] = mc_cpu_baseline(result["mc_stream"], args.cpu_procs or None)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.finalize()
    return result


if __name__ == "__main__":
    main()
