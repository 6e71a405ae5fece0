"""Binary64 golden fixtures at full size (BASELINE configs[1] and configs[3])
by importing the reference itself (build container only).

Run from the repo root:  python tests/golden/make_fp64_golden.py

c2.npz / c4.npz store the reference's beta as binary32, which pins a binary64
decode only to ~1e-7.  This script re-runs the reference (same rules and
workarounds as make_golden.py, whose loader and bit-checked vectorised FHT it
imports) on the SAME inputs — the y of those fixtures, checked against a fresh
draw — and records beta in binary64:

  c2_f64.npz: L=M=512 R=1 P=4 (n=4608), one codeword: beta at t = 1 and t = 8
              (fixed iteration counts) and at the exact-tau stop (amp_test,
              T = 64), first NS = 128 sections, plus the norms of the whole
              vectors and the stop index;
  c4_f64.npz: L=768 M=512 R=5/6 P=1.8 (n=8294), the two codewords of c4.npz:
              the same quantities, first NS = 64 sections.

It also checks that the binary64 results rounded to binary32 equal the
existing binary32 fixtures bit for bit (the fixtures are reproducible).
Only the reference's own functions are executed; only outputs are recorded.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def decode_set(ref, amp_test_fn, y, Pl, L, M, T, Ab, Az, NS):
    b1 = ref.amp(y, 0, Pl, L, M, 1, Ab, Az, mg.zeros(L, M))
    b8 = ref.amp(y, 0, Pl, L, M, 8, Ab, Az, mg.zeros(L, M))
    bfin, tstop = amp_test_fn(y, 0, Pl, L, M, T, Ab, Az, mg.zeros(L, M))
    out = {"beta_t1": b1[:NS * M].astype(np.float64), "beta_t1_norm": float(np.linalg.norm(b1)),
           "beta_t8": b8[:NS * M].astype(np.float64), "beta_t8_norm": float(np.linalg.norm(b8)),
           "beta_final": bfin[:NS * M].astype(np.float64), "beta_final_norm": float(np.linalg.norm(bfin)),
           "t_stop": int(tstop), "argmax_final": bfin.reshape(L, M).argmax(1)}
    return out, b1, bfin


def main():
    ref = mg.load_reference()
    ref.fht_inplace = mg.fast_fht  # bitwise-equal to the fallback (make_golden.py §1)
    import amp_test as ref_amp_test

    # ---- C2 ------------------------------------------------------------------
    g = np.load(os.path.join(HERE, "c2.npz"))
    L, M, P, T = int(g["L"]), int(g["M"]), float(g["P"]), int(g["T"])
    n = int(g["n"])
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    assert mg.sha(ordering) == str(g["ordering_sha256"])
    _, y = mg.rep_inputs(ref, L, M, n, Pl, float(g["sigma"]), Ab, 1000)
    assert np.array_equal(y, g["y"])
    NS = 128
    t0 = time.time()
    d, b1, bfin = decode_set(ref, ref_amp_test.amp_test, y, Pl, L, M, T, Ab, Az, NS)
    print(f"c2: t_stop={d['t_stop']} {time.time() - t0:.1f} s", flush=True)
    assert np.array_equal(b1.astype(np.float32), g["beta_t1"])
    assert np.array_equal(bfin.astype(np.float32), g["beta_final"])
    assert d["t_stop"] == int(g["t_stop"])
    np.savez_compressed(os.path.join(HERE, "c2_f64.npz"), L=L, M=M, n=n, P=P, T=T, NS=NS, y=y, **d)

    # ---- C4 ------------------------------------------------------------------
    g = np.load(os.path.join(HERE, "c4.npz"))
    L, M, P, T, n = int(g["L"]), int(g["M"]), float(g["P"]), int(g["T"]), int(g["n"])
    NS = int(g["NS"])
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    assert mg.sha(ordering) == str(g["ordering_sha256"])
    out = dict(L=L, M=M, n=n, P=P, T=T, NS=NS)
    for k in (0, 1):
        sigma = float(g[f"sigma_{k}"])
        _, y = mg.rep_inputs(ref, L, M, n, Pl, sigma, Ab, 2000 + k)
        assert np.array_equal(y, g[f"y_{k}"])
        t0 = time.time()
        d, b1, bfin = decode_set(ref, ref_amp_test.amp_test, y, Pl, L, M, T, Ab, Az, NS)
        print(f"c4 sigma={sigma}: t_stop={d['t_stop']} {time.time() - t0:.1f} s", flush=True)
        assert np.array_equal(b1[:NS * M].astype(np.float32), g[f"beta_t1_{k}"])
        assert np.array_equal(bfin[:NS * M].astype(np.float32), g[f"beta_final_{k}"])
        assert d["t_stop"] == int(g[f"t_stop_{k}"])
        out[f"sigma_{k}"] = sigma
        out[f"y_{k}"] = y
        out.update({f"{key}_{k}": v for key, v in d.items()})
    np.savez_compressed(os.path.join(HERE, "c4_f64.npz"), **out)


if __name__ == "__main__":
    main()
