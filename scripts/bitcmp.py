#!/usr/bin/env python3
"""Bit-for-bit comparison of two builds of the AMP library (diagnostic).

  bitcmp.py run OUT.npz         decode a fixed set of batches with the library
                                SPARC_AMP_LIB names, save beta / stop indices
  bitcmp.py cmp A.npz B.npz     report, per case, whether the two are identical
                                (and the largest relative difference if not)

Cases cover every batched-kernel element count (E = 1, 2, 4, 8), both
precisions and the single-codeword kernels, at fixed T and with early stop.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

CASES = [  # L, M, R, B, precision
    (512, 512, 1.0, 8, "fp32"), (512, 512, 1.0, 3, "fp32"), (512, 512, 1.0, 1, "fp32"),
    (768, 512, 5 / 6, 6, "fp32"), (128, 256, 1.0, 16, "fp32"), (64, 128, 1.0, 8, "fp32"),
    (32, 64, 1.0, 8, "fp32"), (16, 16, 1.0, 8, "fp32"), (512, 512, 1.0, 8, "fp64"),
    (64, 128, 1.0, 8, "fp64"), (768, 512, 5 / 6, 1, "fp32"), (768, 512, 5 / 6, 2, "fp64"),
    (512, 512, 1.0, 1, "fp64"), (256, 256, 1.0, 2, "fp32"),
]


def run(out):
    import sparc_ldpc_amd as sp
    res = {}
    sel = os.environ.get("BITCMP_CASES")
    for ci, (L, M, R, B, prec) in enumerate(CASES):
        if sel and str(ci) not in sel.split(","):
            continue
        n = int(L * np.log2(M) / R)
        op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)
        rs = np.random.RandomState(L + M + B)
        P = 4.0
        Pl = P / L * np.ones(L)
        beta = np.zeros((B, L * M))
        for b in range(B):
            beta[b, np.arange(L) * M + rs.randint(0, M, L)] = np.sqrt(n * Pl)
        ys = op.Ab_batch(beta) + 0.6 * rs.randn(B, n)
        key = f"{L}_{M}_{B}_{prec}"
        res[key + "_ys"] = ys
        res[key + "_az"] = op.Az_batch(ys)
        res[key + "_t1"] = op.amp_batch(ys, Pl, 1, early_stop=False)[0]
        res[key + "_t2"] = op.amp_batch(ys, Pl, 2, early_stop=False)[0]
        bb, it = op.amp_batch(ys, Pl, 12, early_stop=False)
        res[key + "_fix"] = bb
        bb, it = op.amp_batch(ys, Pl, 40)
        res[key + "_stop"] = bb
        res[key + "_it"] = it
        print(key, op.plan(B)["section_kernel"], flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k], Bz[k])
        if not same:
            bad += 1
            d = np.abs(A[k] - Bz[k]).max() / max(np.abs(A[k]).max(), 1e-300)
            print(f"{k:28s} DIFFERS (max rel {d:.3g})")
        else:
            print(f"{k:28s} identical")
    print("all identical" if not bad else f"{bad} differ")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
