#!/usr/bin/env python3
"""AMP EXIT curves of threshold-initialised exchange on the MI355X
(amp_exit_curve, ldpc/amp_exit.py:520-631): the reference's __main__
configuration L=256 M=32 P=4 R=1 T=64, SNR 10..13 dB (4 curves, 20 log10),
10 I_a points, threshold 0.7, 350 bins, with the repeat count of its
published figure (amp_exit_threshold_L256M32R1P4Bins350Threshold0_*_200reps).
Writes <out>.json: I_a, SNR, I_e curves, cubic fit, wall time."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=200)
    ap.add_argument("--threshold", type=float, default=0.7)
    ap.add_argument("--points", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/exit_curve")
    args = ap.parse_args()
    import sparc_ldpc_amd as sp
    spp = sp.SPARCParams(L=256, M=32, sigma=None, p=4, r=1, t=64)
    np.random.seed(args.seed)
    t0 = time.time()
    I_a, snr, I_e, poly = sp.amp_exit_curve(spp, 10, 13, args.repeats, args.points, args.threshold,
                                            bin_number=350, batch=args.batch)
    dt = time.time() - t0
    res = dict(config="L=256 M=32 P=4 R=1 T=64, threshold %.2f, 350 bins" % args.threshold,
               repeats=args.repeats, calc_E_calls=int(args.repeats * 4 * args.points), seconds=dt,
               I_a=I_a.tolist(), snr_dB=snr.tolist(), I_e=I_e.tolist(), poly_coeff=poly.tolist())
    with open(args.out + ".json", "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("calc_E_calls", "seconds", "poly_coeff")}))
    for j, s in enumerate(snr):
        print(f"SNR {s:5.2f} dB: " + " ".join(f"{v:.3f}" for v in I_e[j]))


if __name__ == "__main__":
    main()
