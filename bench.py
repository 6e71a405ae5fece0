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
    + write, Ab partials written."""
    fwd = 4 * n * G if kernel == "k_sec43" else 2 * L * n
    return 2 * L * w + fwd + B * (n * s + 2 * L * M * s + G * n * s)


def row_bytes(n, B, G, s):
    """k_row: Ab partials read, y read, z read + write."""
    return B * (G * n * s + 3 * n * s)


def gemv_bytes(L, M, n):
    """4·n·L·M + 4·(n + L·M) per fp32 GEMV."""
    return 4 * n * L * M + 4 * (n + L * M)


def _cpu_worker(args):
    L, M, n, P, sigma, Tsample, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import amp_oracle as orc
    Ab, Az, _ = orc.sparc_transforms(L, M, n)
    Pl = P / L * np.ones(L)
    _, y = orc.rep_inputs(L, M, n, Pl, sigma, Ab, seed)
    t0 = time.perf_counter()
    orc.amp(y, sigma, Pl, L, M, Tsample, Ab, Az)
    return (time.perf_counter() - t0) / Tsample


def cpu_baseline(w, procs, Tsample=4):
    """The oracle (reference algorithm in fp64 NumPy, vectorised FWHT) on the
    host cores: `procs` independent processes, each timing Tsample AMP
    iterations of one codeword; extrapolated to T iterations per codeword."""
    import multiprocessing as mp
    L, M, P, sigma, T = w["L"], w["M"], w["P"], w["sigma"], w["T"]
    n = n_of(w)
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        per_iter = pool.map(_cpu_worker, [(L, M, n, P, sigma, Tsample, 1000 + i) for i in range(procs)])
    sec_per_cw = float(np.mean(per_iter)) * T
    return {
        "value": procs / sec_per_cw, "unit": "codewords/s", "cores": procs, "kind": "port",
        "sample": f"oracle amp() fp64 NumPy, {procs} procs x 1 codeword x {Tsample} iterations "
                  f"(L={L} M={M} n={n}), extrapolated to T={T} iterations/codeword; "
                  f"{np.mean(per_iter) * 1e3:.1f} ms/iteration/core",
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
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # SPARC_BENCH_DIST=gloo: rehearsal of the N-rank path on a box with fewer
    # GPUs than ranks (ranks share device LOCAL_RANK % device_count); the
    # driver's multi-GPU runs use the default, RCCL with one GPU per rank
    backend = os.environ.get("SPARC_BENCH_DIST", "nccl")
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend != "nccl":
            device = local % torch.cuda.device_count()
        torch.cuda.set_device(device)
        dist.init_process_group(backend)  # "nccl" = RCCL over xGMI

    import sparc_ldpc_amd as sp

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
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        op.run(B, T, early_stop=False)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        op.run(B, T, early_stop=False)
    sync_all()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

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
        per = {
            "k_sec": sec_bytes(L, M, n, wv, B, G, s, plan["section_kernel"]),
            "k_row": row_bytes(n, B, G, s),
        }
    else:
        per = {"k_dense_az": gemv_bytes(L, M, n) * B, "k_dense_ab": gemv_bytes(L, M, n) * B,
               "k_dense_den": B * (8 * 4 * L * M + 8 * L * M), "k_row": row_bytes(n, B, 8, s)}
    share = {k: kinds[k][0] * kinds[k][1] for k in per}
    dom = max(share, key=share.get)
    dom_ms = kinds_rep[dom][0]
    achieved = per[dom] / (dom_ms * 1e-3) / 1e9
    pmc = load_pmc(f"{args.workload}_{args.backend}_{args.precision}_B{B}",
                   {"k_sec": plan["section_kernel"], "k_row": plan["row_kernel"]}.get(dom, dom))
    kname = {"k_sec": plan["section_kernel"], "k_row": plan["row_kernel"]}.get(dom, dom)
    roofline = {
        "bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None if pmc is None else pmc.get("hbm_bytes_per_launch"),
        "algorithmic_bytes_per_launch": per[dom], "avg_launch_ms": round(dom_ms, 5),
        "kernel_ms": {k: round(v[0], 5) for k, v in kinds_rep.items() if v[1]},
        "kernel_ms_event_bracketed": {k: round(v[0], 5) for k, v in kinds.items() if v[1]},
        "timing": f"HIP events on the library stream around {PROFILE_REP} back-to-back launches per kernel",
        "eager_decode_ms": round(total_ms, 3),
    }

    result = {
        "metric": "decoded codewords/sec (T AMP iters) at L=512,M=512; achieved HBM GB/s vs roofline",
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
    if rank == 0 and world == 1 and not args.no_dense:
        try:
            result["dense_gemv"] = dense_gemv_probe(device)
        except Exception as e:  # report, never hide
            result["dense_gemv"] = {"error": str(e)}
    if rank == 0 and world == 1 and not args.no_cpu:
        procs = args.cpu_procs or min(16, len(os.sched_getaffinity(0)))
        result["cpu_baseline"] = cpu_baseline(w, procs)
        result["cpu_baseline"]["gpu_over_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
