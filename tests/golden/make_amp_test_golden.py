"""Golden fixture for the amp_test.py reps loop (amp_test.py:161-253) by
executing the reference's own functions (build container only).

Run from the repo root:  python tests/golden/make_amp_test_golden.py

Same loader and workarounds as make_golden.py (bitarray stub, the
bit-checked vectorised FHT, an explicit zeros beta for the zero start — the
reference's own default sentinel crashes under NumPy 2).  The __main__ block
of amp_test.py is not callable, so this driver performs its steps with the
reference's functions (bits2indices, sparc_transforms,
sparc_transforms_shorter, amp): after ``np.random.seed(seed)`` every rep draws
``randint(0, 2, total_bits)`` then ``randn(n, 1) * sigma`` (no decode consumes
np.random, so all draws are made first, in that order, and the decodes of the
reps then run in parallel processes); the three decodes per rep are
hard init on the shortened operator, soft init from the 0/1 beta_0, no init.
Recorded per rep: the three bit-error counts and decisions; per case the
three BERs accumulated in rep order exactly as the loop does.
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

CASES = {
    # the reference's own parameters (amp_test.py:162-173), 8 reps
    "main": dict(L=512, M=512, L_zero=154, P=4.0, snr_dB=10.0, r_sparc=1.0, T=64, repeats=8, seed=2024),
    # a small configuration with more reps (both precisions are tested on it)
    "small": dict(L=128, M=64, L_zero=40, P=4.0, snr_dB=8.0, r_sparc=1.0, T=64, repeats=24, seed=77),
}


def _decode(args):
    L, M, L_zero, P, sigma, T, n, idx, noise = args
    ref = mg.load_reference()
    ref.fht_inplace = mg.fast_fht
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    beta = np.zeros((L * M, 1))
    for l in range(L):
        beta[l * M + idx[l]] = np.sqrt(n * Pl[l])
    y = (Ab(beta) + noise).reshape(-1, 1)
    beta_0 = beta / np.sqrt(n * P / L)
    beta_0[:L_zero * M] = 0
    y_new = y - Ab(beta_0)
    Ab_n, Az_n = ref.sparc_transforms_shorter(L_zero, M, n, ordering)
    bh = ref.amp(y_new, sigma, Pl[:L_zero], L_zero, M, T, Ab_n, Az_n, mg.zeros(L_zero, M)).reshape(-1)
    bs = ref.amp(y, sigma, Pl, L, M, T, Ab, Az, beta_0).reshape(-1)
    bz = ref.amp(y, sigma, Pl, L, M, T, Ab, Az, mg.zeros(L, M)).reshape(-1)
    rx_h = bh.reshape(L_zero, M).argmax(1)
    rx_s = bs.reshape(L, M).argmax(1)
    rx_z = bz.reshape(L, M).argmax(1)
    e_h = sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(idx[:L_zero], rx_h))
    e_s = sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(idx, rx_s))
    e_z = sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(idx, rx_z))
    return (e_h, e_s, e_z), rx_h, rx_s, rx_z


def main():
    ref = mg.load_reference()
    out, meta = {}, {}
    for name, c in CASES.items():
        L, M, L_zero, P, T, R = c["L"], c["M"], c["L_zero"], c["P"], c["T"], c["repeats"]
        sigma = float(np.sqrt(P / 10 ** (c["snr_dB"] / 20)))   # amp_test.py:167-169
        total_bits = int(L * np.log2(M))
        n = int(L * np.log2(M) / c["r_sparc"])
        np.random.seed(c["seed"])
        jobs = []
        for _ in range(R):
            bits = np.random.randint(0, 2, total_bits).tolist()
            idx = np.asarray(ref.bits2indices(bits, M))
            noise = np.random.randn(n, 1) * sigma
            jobs.append((L, M, L_zero, P, sigma, T, n, idx, noise))
        with mp.get_context("spawn").Pool(min(8, R)) as pool:
            res = pool.map(_decode, jobs)
        counts = np.array([r[0] for r in res], dtype=np.int64)
        ber = [0.0, 0.0, 0.0]
        for i in range(R):
            for j in range(3):
                ber[j] = ber[j] + int(counts[i, j]) / total_bits
        ber = [b / R for b in ber]
        out[f"{name}_counts"] = counts
        out[f"{name}_idx"] = np.stack([j[7] for j in jobs]).astype(np.int16)
        out[f"{name}_rx_hard"] = np.stack([r[1] for r in res]).astype(np.int16)
        out[f"{name}_rx_soft"] = np.stack([r[2] for r in res]).astype(np.int16)
        out[f"{name}_rx_noinit"] = np.stack([r[3] for r in res]).astype(np.int16)
        meta[name] = dict(c, sigma=sigma, n=n, ber_hard=ber[0], ber_soft=ber[1], ber_no_init=ber[2])
        print(name, meta[name], counts.tolist(), flush=True)
    np.savez_compressed(os.path.join(HERE, "amp_test_reps.npz"), **out)
    with open(os.path.join(HERE, "amp_test_reps.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


if __name__ == "__main__":
    main()
