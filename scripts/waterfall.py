#!/usr/bin/env python3
"""BER-vs-Eb/N0 sweeps on the MI355X next to the reference's published curves.

  plain   : waterfall()'s BER_plain column (sparc_ldpc.py:1126-1282):
            L=M=512 P=4 R=5/6 T=64, Eb/N0 = linspace(3, 10, 10) dB (20*log10),
            MIN_ERRORS=200 / MAX_BLOCKS=250.
  soft / hard / originalHard : the joint waterfall() runs (configs[4]):
            L=M=512 P=4 r_sparc=1 T=64 with the 802.16 rate-5/6 outer code
            (all 512 sections; originalHard: 384 as the shipped call), every
            BER column incl. plain SPARC and LDPC+BPSK, MIN_ERRORS=200 /
            MAX_BLOCKS=250.
  threshold : soft_hardinit_plot() (sparc_ldpc.py:1435-1590): threshold-
            initialised exchange, L=M=512 P=4 r_sparc=1 T=64 + 802.16 rate 5/6
            over all 512 sections, soft_iter=2, sigma = linspace(0.9, 1.4, 10),
            threshold 0.6 or 0.8 (--threshold), MIN_ERRORS = MAX_BLOCKS = 200.
  soft_hard : soft_hard_plot() (sparc_ldpc.py:1285-1432) in full: L=768 M=512
            P=1.8 r_sparc=1 T=64, 802.16 5/6 with sec=569 (z=213), soft
            exchange (2 rounds) and the original hard exchange,
            sigma = linspace(0.8, 0.4, 10), MIN_ERRORS = MAX_BLOCKS = 100.
  l768    : soft_hard_plot()'s BER_sparc column (sparc_ldpc.py:1285-1432):
            L=768 M=512 P=1.8 at the overall rate R=0.8765 (sec=569),
            sigma = linspace(0.8, 0.4, 10), 100 reps per point.

One process per GPU (torchrun); reps sharded by rank, per-round counters
summed over RCCL.  Writes <out>.csv (reference schema) and <out>.json.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", default="plain", choices=["plain", "l768", "soft", "hard", "originalHard", "threshold", "soft_hard"])
    ap.add_argument("--threshold", type=float, default=0.6)
    ap.add_argument("--reps", type=int, default=0,
                    help="l768: reps per sigma point (default: the published 100; BASELINE configs[3] is 1000 x 10)")
    ap.add_argument("--unit-cancel", action="store_true",
                    help="threshold sweep: cancel decided sections with amplitude 1 (the reference before its fix)")
    ap.add_argument("--points", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="codewords per batch (default 64; l768: 256 slots)")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="l768: decode batch by batch instead of one refilled stream")
    ap.add_argument("--out", default="gpurun_out/waterfall")
    ap.add_argument("--precision", default=None, help="fp32 | fp64 (default: fp32 plain sweeps, fp64 joint)")
    args = ap.parse_args()
    import sparc_ldpc_amd as sp
    from sparc_ldpc_amd import dist
    rank, world, _ = dist.init()
    if args.batch is None:
        args.batch = 256 if args.sweep == "l768" else 64
    with open(os.path.join(ROOT, "tests", "golden", "published_ber.json")) as fh:
        pub = json.load(fh)
    t0 = time.time()
    split = None
    if args.sweep == "plain":
        cfg = pub["waterfall_plain"]["config"]
        ebno = np.linspace(3, 10, 10)[:args.points]
        rows = sp.waterfall_plain(cfg["L"], cfg["M"], cfg["P"], cfg["R"], cfg["T"], ebno,
                                  cfg["MIN_ERRORS"], cfg["MAX_BLOCKS"],
                                  csv_filename=args.out + ".csv" if rank == 0 else None,
                                  batch=args.batch, precision=args.precision or "fp32", rank=rank, world=world,
                                  allreduce=dist.allreduce_sum)
        ref = pub["waterfall_plain"]["BER_plain_runs"]
        for i, r in enumerate(rows):
            r["reference_runs"] = [v[i] for v in ref.values()]
    elif args.sweep in ("soft", "hard", "originalHard"):
        cfg = pub["waterfall_joint"]["config"]
        sections = 384 if args.sweep == "originalHard" else 512
        spp = sp.SPARCParams(cfg["L"], cfg["M"], None, cfg["P"], cfg["r_sparc"], cfg["T"])
        lp = sp.LDPCParams("802.16", "5/6", None)
        ebno = np.linspace(3, 10, 10)[:args.points]
        rows = sp.waterfall(spp, lp, csv_filename=args.out + ".csv" if rank == 0 else None, init=args.sweep,
                            MIN_ERRORS=cfg["MIN_ERRORS"], MAX_BLOCKS=cfg["MAX_BLOCKS"], sections=sections,
                            batch=args.batch, precision=args.precision, rank=rank, world=world,
                            allreduce=dist.allreduce_sum, ebno_dbs=ebno)
        ref = pub["waterfall_joint"]["runs"][args.sweep]
        for i, r in enumerate(rows):
            r["reference"] = {k: ref[k][i] for k in ref if k not in ("file", "EbN0_dB")}
    elif args.sweep == "soft_hard":
        cfg = pub["soft_hard"]["config"]
        spp = sp.SPARCParams(cfg["L"], cfg["M"], None, cfg["P"], cfg["r_sparc"], cfg["T"])
        lp = sp.LDPCParams(cfg["standard"], cfg["r_ldpc"], None)
        sig = np.linspace(*cfg["sigma"])[:args.points]
        rows = sp.soft_hard_plot(True, True, cfg["sec"], cfg["soft_iter"], spp, lp,
                                 args.out + ".csv" if rank == 0 else None, None, MIN_ERRORS=cfg["MIN_ERRORS"],
                                 MAX_BLOCKS=cfg["MAX_BLOCKS"], batch=args.batch, precision=args.precision,
                                 rank=rank, world=world, allreduce=dist.allreduce_sum, sigmas=sig)
        ps, ph = pub["soft_hard"]["soft"], pub["soft_hard"]["hard"]
        for i, r in enumerate(rows):
            r["reference"] = dict(BER_sparc=ps["BER_sparc"][i], BER_ldpc_soft=ps["BER_ldpc"][i],
                                  BER_amp_soft=ps["BER_amp"][i], BER_ldpc_hard=ph["BER_ldpc"][i],
                                  BER_amp_hard=ph["BER_amp"][i])
    elif args.sweep == "threshold":
        cfg = pub["threshold_init"]["config"]
        spp = sp.SPARCParams(cfg["L"], cfg["M"], None, cfg["P"], cfg["r_sparc"], cfg["T"])
        lp = sp.LDPCParams(cfg["standard"], cfg["r_ldpc"], None)
        sig = np.linspace(*cfg["sigma"])[:args.points]
        rows = sp.soft_hardinit_plot(spp, lp, args.out + ".csv" if rank == 0 else None, None, cfg["sections"],
                                     MIN_ERRORS=200, MAX_BLOCKS=200, soft_iter=cfg["soft_iter"],
                                     threshold=args.threshold, batch=args.batch, precision=args.precision or "fp64",
                                     rank=rank, world=world, allreduce=dist.allreduce_sum, sigmas=sig,
                                     unit_cancel=args.unit_cancel)
        refs = [r for r in pub["threshold_init"]["runs"] if r["threshold"] == args.threshold]
        for i, r in enumerate(rows):
            r["reference_runs"] = [{k: ref[k][i] for k in ("BER_amp", "BER_ldpc", "BER_plain")} for ref in refs]
    else:
        cfg = pub["soft_hard_BER_sparc"]["config"]
        L, M, P, T = cfg["L"], cfg["M"], cfg["P"], cfg["T"]
        logm = np.log2(M)
        n_coded = L * logm / 1
        R = (L * logm - 9 * 569 * (1 - 5 / 6)) / n_coded
        n = int(L * logm / R)
        Pl = P / L * np.ones(L)
        sigmas = np.linspace(0.8, 0.4, 10)[:args.points]
        reps = args.reps or cfg["reps_per_point"]
        assert reps <= 100000
        # point i's reps: seeds i * 100000 + j, sharded by rank
        seeds = [[j for j in range(i * 100000, i * 100000 + reps) if j % world == rank] for i in range(len(sigmas))]
        cnt = [len(s) for s in seeds]
        off = np.concatenate([[0], np.cumsum(cnt)])
        idx = np.empty((off[-1], L), dtype=np.int32)
        noise = np.empty((off[-1], n))
        drawn = {}

        def draw_all():  # the native draws release the GIL: they run beside the operator set-up
            t = time.time()
            for i, sigma in enumerate(sigmas):
                sp.draw_reps(seeds[i], L, M, n, sigma, idx=idx[off[i]:off[i + 1]], noise=noise[off[i]:off[i + 1]])
            drawn["s"] = time.time() - t

        import threading
        drawer = threading.Thread(target=draw_all) if args.stream else None
        if drawer is not None:
            drawer.start()
        ta = time.time()
        ordering = sp.make_ordering(L, M, n)
        tb = time.time()
        op = sp.SparcOperator(L, M, n, ordering, precision=args.precision or "fp32")
        if args.stream and op.mc_supported(args.batch):
            op.reserve(args.batch, T)  # (the batched kernel's tables)
        tc = time.time()
        if drawer is not None:
            drawer.join()
        if args.stream and op.mc_supported(args.batch):
            # every point's reps in ONE stream through the refilled slots (AMP
            # never reads sigma: it is in the noise), drawn natively on the host
            t2 = time.time()
            phases = {"draw_wait_s": t2 - tc}
            be_all, it_all, dev_ms = sp.mc_stream(op, Pl, T, idx, noise, batch=args.batch, timings=phases)
            t3 = time.time()
            parts = [(be_all[off[i]:off[i + 1]], it_all[off[i]:off[i + 1]]) for i in range(len(sigmas))]
            # codeword-iterations: the sum of the stop indices (T when a rep ran
            # out), as VERDICT r05 counts them; slot-iterations: the section /
            # row steps the slots actually ran (min(stop index + 1, T) per rep)
            split = dict(ordering_s=tb - ta, operator_s=tc - tb, draw_s=drawn["s"], draws_beside_setup=True,
                         stream_s=t3 - t2, stream_phases=phases,
                         decode_device_ms=dev_ms, batch=args.batch,
                         codeword_iterations=int(it_all.sum()), slot_iterations=int(np.minimum(it_all + 1, T).sum()))
        else:
            parts = [sp.mc_decode(op, Pl, sigma, T, seeds[i], batch=args.batch, stream=False)
                     for i, sigma in enumerate(sigmas)]
            split = None
        rows = []
        for i, sigma in enumerate(sigmas):
            be, it = parts[i]
            tot = dist.allreduce_sum(np.array([be.sum(), len(seeds[i]), it.sum()], dtype=np.int64))
            ebno_db = 20 * np.log10(1 / (2 * R) * (P / sigma ** 2))  # sparc_ldpc.py:1414-1416
            rows.append(dict(EbN0_dB=float(ebno_db), BER_sparc=float(tot[0] / (tot[1] * L * logm)),
                             blocks=int(tot[1]), mean_iters=float(tot[2] / tot[1]),
                             reference=pub["soft_hard_BER_sparc"]["BER_sparc"][i]))
    if rank == 0:
        res = dict(sweep=args.sweep, world=world, seconds=time.time() - t0, rows=rows)
        if split is not None:
            # the l768 stream: host draw / stream wall time, its device time and
            # the codeword-iterations it decoded (sum of min(stop index + 1, T))
            split["decode_codeword_iterations_per_s"] = split["codeword_iterations"] / (split["decode_device_ms"] / 1e3)
            res["split"] = split
        with open(args.out + ".json", "w") as fh:
            json.dump(res, fh, indent=1)
        for r in rows:
            print(json.dumps(r))
        print(f"# {args.sweep}: {time.time() - t0:.1f} s on {world} GPU(s)")
    dist.finalize()


if __name__ == "__main__":
    main()
