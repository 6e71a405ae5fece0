#!/usr/bin/env python3
"""Throughput of the joint SPARC + LDPC decoder (BASELINE
configs[4]): L=M=512 P=4 r_sparc=1 (n=4608), T=64, 802.16 rate-5/6 z=192
outer code over all 512 sections, soft information exchange
(soft_amp_ldpc_sim, ldpc/sparc_ldpc.py:547-712) with 2 rounds, at one point
of the waterfall (Eb/N0 = 6.89 dB, the reference's sigma mapping).

A step = one joint decode of a batch of B codewords whose y is already in
HBM: AMP (zero start) -> LLRs -> BP -> bp2sp -> AMP (LDPC start), twice;
early stop on, as the reference runs it.  Per-rep error counts come back to
the host each round (the step includes those small copies).  By default the
batch runs as two concurrent halves (joint.JointPipeline: each half on its own
operator / LDPC contexts and streams, driven from its own host thread), so one
half's BP tail overlaps the other half's AMP; the per-rep error counts are
asserted identical to one decoder over the whole batch.

Prints one JSON line like bench.py: value (codewords/s), the roofline of the
dominant kernel (per-launch HIP events), the BP decoder's launch time, and a
CPU baseline: whole reps of the reference algorithm on the host cores
(oracle AMP in NumPy + the reference's own C sumprod2 built by
oracle/Makefile when present + the reference's Python sp2bp/bp2sp loops).
The CPU leg is the only use of oracle/ here.
"""
from __future__ import annotations

import argparse
import ctypes as ct
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import HBM_PEAK_GBS, load_pmc, load_trace, row_bytes, sec_bytes  # noqa: E402

L, M, P, T, Z = 512, 512, 4.0, 64, 192
N_SPARC = 4608  # L log2 M / r_sparc, r_sparc = 1


def _cpu_rep(args):
    """One soft rep of the reference algorithm, single-threaded; returns
    (seconds, seconds in BP, seconds in AMP, AMP iterations, BP iterations)."""
    sigma, soft_iter, seed = args
    from oracle import amp_oracle as orc
    from oracle import ldpc_oracle as lo
    proto = lo.protograph("802.16", "5/6", Z)
    vdeg, cdeg, intrlv = lo.prepare_decoder(proto, Z)
    Nv, Nc, Nmsg = len(vdeg), len(cdeg), int(np.sum(vdeg))
    so = os.path.join(ROOT, "oracle", "_ref", "c_ldpc.so")
    lib = ct.CDLL(so) if os.path.exists(so) else None

    def decode(ch):
        if lib is None:
            return lo.sumprod2(ch, vdeg, cdeg, intrlv)
        D, LP = ct.POINTER(ct.c_double), ct.POINTER(ct.c_long)
        ch = np.ascontiguousarray(ch, dtype=np.double)
        app = np.zeros(Nv)
        v, c, il = (np.ascontiguousarray(a, dtype=np.int64) for a in (vdeg, cdeg, intrlv))
        it = lib.sumprod2(ch.ctypes.data_as(D), v.ctypes.data_as(LP), c.ctypes.data_as(LP), il.ctypes.data_as(LP),
                          Nv, Nc, Nmsg, app.ctypes.data_as(D))
        return app, it

    rs = np.random.RandomState(seed)
    n = N_SPARC
    Pl = P / L * np.ones(L)
    K = proto.shape[1] * Z - proto.shape[0] * Z
    bits = lo.encode(proto, Z, rs.randint(0, 2, K))
    idx = orc.bits2indices(bits, M)
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    beta0 = np.zeros((L * M, 1))
    beta0[np.arange(L) * M + np.asarray(idx), 0] = np.sqrt(n * Pl)
    y = Ab(beta0) + rs.randn(n, 1) * sigma
    ns = L
    t_amp = t_bp = 0.0
    amp_it = bp_it = 0
    t0 = time.perf_counter()
    ta = time.perf_counter()
    beta, t = orc.amp_test(y, sigma, Pl, L, M, T, Ab, Az)
    t_amp += time.perf_counter() - ta
    amp_it += t + 1
    for _ in range(soft_iter):
        llr = lo.llr_from_beta(beta, Pl, n, L, M, ns)
        tb = time.perf_counter()
        app, it = decode(llr)
        t_bp += time.perf_counter() - tb
        bp_it += it
        post = lo.bp2sp(1 / (1 + np.exp(app)), ns, M)
        ta = time.perf_counter()
        beta, t = orc.amp_test(y, sigma, Pl, L, M, T, Ab, Az, post * np.sqrt(n * np.repeat(Pl, M)))
        t_amp += time.perf_counter() - ta
        amp_it += t + 1
    return time.perf_counter() - t0, t_bp, t_amp, amp_it, bp_it, lib is not None


def cpu_baseline(sigma, soft_iter, procs):
    import multiprocessing as mp
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"  # inherited by the spawned workers before NumPy loads
    try:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_rep, [(sigma, soft_iter, 5000 + i) for i in range(procs)])
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old
    sec = float(np.mean([r[0] for r in res]))
    bp = float(np.mean([r[1] for r in res]))
    amp = float(np.mean([r[2] for r in res]))
    ref_bp = all(r[5] for r in res)
    return {
        "value": procs / sec, "unit": "codewords/s", "cores": procs, "kind": "port",
        "sample": f"{procs} procs x 1 full soft rep (2 rounds): oracle amp() fp64 NumPy "
                  f"({np.mean([r[3] for r in res]):.0f} AMP iterations/rep, {amp:.2f} s), "
                  + ("the reference's C sumprod2 (oracle/_ref/c_ldpc.so)" if ref_bp else "oracle sumprod2")
                  + f" ({np.mean([r[4] for r in res]):.0f} BP iterations/rep, {bp:.3f} s), "
                  f"the reference's sp2bp/bp2sp loops ({sec - amp - bp:.2f} s); {sec:.2f} s/rep/core",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ebno", type=float, default=6.888888888888889)
    ap.add_argument("--soft-iter", type=int, default=2)
    ap.add_argument("--precision", default="fp64", choices=["fp32", "fp64"])
    ap.add_argument("--plan", default="", help="comma-separated plan options (sa_create_ex)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=0)
    ap.add_argument("--no-ref", action="store_true", help="skip the one-decoder reference decode (traces)")
    ap.add_argument("--no-twin", action="store_true",
                    help="the pipeline's slices build their own operator tables (A/B of SparcOperator.twin)")
    ap.add_argument("--parts", type=int, default=2,
                    help="concurrent slices of the batch, each on its own streams (joint.JointPipeline); 1: one decoder")
    args = ap.parse_args()
    print(json.dumps(measure(args)), flush=True)


def measure(args, device=None, rank=0, world=1):
    """One joint measurement (the line main() prints; bench.py's joint leg):
    every rank decodes its own batch (draws seeded 7000 + rank * B + i), the
    timed steps bracketed by a barrier and a device wait on each rank, value =
    all ranks' codewords / the slowest rank's time; the CPU leg on rank 0."""
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd import dist, joint
    from sparc_ldpc_amd.harness import ebno_to_sigma

    lp = sp.LDPCParams("802.16", "5/6", Z)
    R = 5 / 6
    sigma = ebno_to_sigma(args.ebno, P, R)
    jd = joint.joint_decoder(L, M, N_SPARC, lp, T, precision=args.precision, device=device)
    if args.plan:  # A/B of plan options: the same design with sa_create_ex options
        jd.op = sp.SparcOperator(L, M, N_SPARC, sp.make_ordering(L, M, N_SPARC), precision=args.precision,
                                 plan=[p for p in args.plan.split(",") if p])
    B = args.batch
    Pl = P / L * np.ones(L)
    idx, noise = jd.draw([np.random.RandomState(7000 + rank * B + i) for i in range(B)], B, sigma)
    # the whole batch on one decoder: the reference result the pipelined
    # step must reproduce rep for rep
    jd.stage(idx, noise, Pl)
    ref = None if args.no_ref else jd.decode_staged(idx, Pl, "soft", args.soft_iter)
    joint.TWIN_SLICES = not args.no_twin
    runner = joint.joint_pipeline(jd, args.parts) if args.parts > 1 else jd
    runner.stage(idx, noise, Pl)

    for _ in range(args.warmup):
        r = runner.decode_staged(idx, Pl, "soft", args.soft_iter)
    runner.wait() if args.parts > 1 else jd.op.wait()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = runner.decode_staged(idx, Pl, "soft", args.soft_iter)
    runner.wait() if args.parts > 1 else jd.op.wait()
    mine = time.perf_counter() - t0
    dist.barrier()
    elapsed = float(dist.allreduce_max(np.array([mine]))[0]) if world > 1 else mine
    for k in ("amp", "ldpc", "bp_iters") if ref is not None else ():
        assert np.array_equal(ref[k], r[k]), f"joint decode differs from the one-decoder result ({k})"
    if args.parts > 1:
        jd.stage(idx, noise, Pl)  # the whole batch again on part 0, for the per-kernel profile below

    # per-kernel HIP-event times: one eager AMP decode of the staged batch (zero
    # start, early stop) and one BP launch on the LLRs it leaves
    op, code = jd.op, jd.code
    kinds, amp_ms = op.profile(B, T)
    jd._bp(B)
    bp_ms = float(sp.ldpc.load_bp_library().lb_run_event_ms(code._context()))
    _, bp_it = code.fetch_buffers(B, app=False)
    # repeated-launch timing: 4 back-to-back launches per HIP-event pair; and
    # the dispatch-bound event pairs of an eager decode (bench.py measure_roofline)
    kinds_rep, _ = op.profile(B, 4, early_stop=False, rep=4)
    kinds_disp, _ = op.profile(B, T, rep=0)
    s = 8 if args.precision == "fp64" else 4
    plan = op.plan(B)
    G = plan["partials"]
    per = {"k_sec": sec_bytes(L, M, N_SPARC, op.w, B, G, s), "k_row": row_bytes(N_SPARC, B, G, s)}
    launches_per_step = {k: kinds[k][1] * (1 + args.soft_iter) for k in per}  # ~ one AMP decode per round
    share = {k: kinds[k][0] * launches_per_step[k] for k in per}
    share["bp"] = bp_ms * args.soft_iter
    dom = max(("k_sec", "k_row"), key=share.get)
    kname = {"k_sec": plan["section_kernel"], "k_row": plan["row_kernel"]}[dom]
    pmc = load_pmc(f"c5_hadamard_{args.precision}_B{B}", kname)
    from sparc_ldpc_amd._lib import source_hash
    src = source_hash()
    fresh = pmc is not None and pmc.get("sources") == src  # a PMC pass of these sources only
    tr = load_trace("joint", kname)
    matched = tr is not None and tr["sources"] == src
    # the profiled command runs the pipelined step: each traced (and PMC-counted)
    # launch decodes one slice of B / parts codewords while the other slice's
    # kernels share the GPU, so those launches are priced at the slice's bytes
    Bs = B // args.parts
    Gs = op.plan(Bs)["partials"]
    per_slice = {"k_sec": sec_bytes(L, M, N_SPARC, op.w, Bs, Gs, s), "k_row": row_bytes(N_SPARC, Bs, Gs, s)}
    dom_ms = tr["duration_ns"] * 1e-6 if matched else kinds_disp[dom][0]
    dom_bytes = per_slice[dom] if matched else per[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    ms_step = elapsed / args.steps * 1e3
    nmsg = int(code.info()["Nmsg"])
    result = {
        "metric": "joint AMP<->BP decoded codewords/sec (soft exchange, 2 rounds) at L=512,M=512 + 802.16 5/6 LDPC",
        "value": round(B * args.steps * world / elapsed, 3),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if args.precision == "fp64" else "f32",
        "data": "synthetic (RandomState(seed) bits, LDPC-encoded, + N(0, sigma^2) noise; reference draw order)",
        "config": {"workload": "BASELINE configs[4]: L=512 M=512 P=4 r_sparc=1 + 802.16 rate-5/6 z=192, "
                               "soft exchange x2 (soft_amp_ldpc_sim)",
                   "L": L, "M": M, "n": N_SPARC, "T": T, "EbN0_dB": round(args.ebno, 4), "sigma": round(sigma, 6),
                   "codewords_per_step": B, "precision": args.precision, "early_stop": True,
                   "concurrent_slices": args.parts},
        "identical_to_one_decoder": ref is not None,
        "roofline": {
            "bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc.get("hbm_bytes_per_launch") if fresh else None,
            **({"traffic_over_algorithmic": round(pmc["hbm_bytes_per_launch"] / per_slice[dom], 3)} if fresh else {}),
            **({"traffic_stale": {"hbm_bytes_per_launch": pmc.get("hbm_bytes_per_launch"), "sources": pmc.get("sources"),
                                  "note": "PMC pass of other sources: not used"}} if pmc is not None and not fresh else {}),
            "sources": src,
            "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": round(dom_ms, 5),
            "launch_codewords": Bs if matched else B,
            "timing": (f"in-graph duration: graph-replay median in {tr['file']} (rocprofv3 trace of this command, "
                       f"these sources): launches of one slice of {Bs} codewords, the other slice's kernels "
                       f"running beside them") if matched else
                      "live: HIP start / stop events bound to each launch's own dispatch (hipExtLaunchKernel), "
                      "eager decode of this run",
            "algorithmic_bytes_whole_batch": per[dom],
            "frac_dispatch": round(per[dom] / (kinds_disp[dom][0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_events": round(per[dom] / (kinds_rep[dom][0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            **({"trace": {"file": tr["file"], "profile_matches_build": matched, "sources": tr["sources"],
                          "in_graph_duration_ms": round(tr["duration_ns"] * 1e-6, 5)}} if tr is not None else {}),
            "kernel_ms_dispatch": {k: round(v[0], 5) for k, v in kinds_disp.items() if v[1]},
            "kernel_ms_events": {k: round(v[0], 5) for k, v in kinds_rep.items() if v[1]},
            "kernel_ms_event_bracketed": {k: round(v[0], 5) for k, v in kinds.items() if v[1]},
            "amp_launches": {k: v[1] for k, v in kinds.items() if v[1]},
            "eager_amp_decode_ms": round(amp_ms, 3),
        },
        "bp": {"kernel": "k_bp<sumprod2> (8 iterations) + k_bp_tail_var / k_bp_tail_chk", "launch_ms": round(bp_ms, 4),
               "words": B,
               "mean_iterations": round(float(bp_it.mean()), 2), "max_iterations": int(bp_it.max()),
               "edges": nmsg, "edge_updates_per_s": round(float(bp_it.sum()) * nmsg / (bp_ms * 1e-3), 1),
               "bound": "fp64 VALU: the first iterations issue-bound (3 waves per SIMD), the tail one wave per "
                        "SIMD on the dependent Lxor chain of each check"},
        "errors": {"amp_bits_per_round": r["amp"].sum(axis=0).tolist(),
                   "ldpc_bits_per_round": r["ldpc"].sum(axis=0).tolist(), "bits": int(B * L * 9)},
        "step_share_ms": {k: round(v, 3) for k, v in share.items()},
    }
    if rank == 0 and not args.no_cpu:
        procs = args.cpu_procs or min(16, len(os.sched_getaffinity(0)))
        result["cpu_baseline"] = cpu_baseline(sigma, args.soft_iter, procs)
        result["cpu_baseline"]["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    return result


if __name__ == "__main__":
    main()
