"""Per-section statistics of the reference's full-size binary64 estimates, for
EVERY section (build container only; imports the reference like
make_golden.py / make_fp64_golden.py, whose loader, bit-checked vectorised
FHT and rep draw order it reuses).

Run from the repo root:  python tests/golden/make_section_stats.py

c2_f64.npz / c4_f64.npz / c4.npz hold beta element-wise for the first
128 / 64 sections only (file size); the other sections were pinned through the
vector norm alone.  This records, for all L sections of the same decodes
(c2: L = M = 512, one codeword; c4: L = 768, the two codewords of c4.npz), at
t = 1, t = 8 (fixed iteration counts) and at the exact-tau stop (amp_test):

  e2[l] = sum_j beta[l, j]^2          (the section's energy, <= c_l^2)
  m1[l] = sum_j j * beta[l, j]        (its first moment over the entry index)
  mx[l] = max_j beta[l, j]

(sum_j beta[l, j] is c_l for every section by construction, so it is not
recorded.)  The inputs are the fixtures' own y, checked against a fresh draw.
Only the reference's own functions are executed; only their outputs are
recorded, into sections.npz.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def stats(beta, L, M):
    b = np.asarray(beta, dtype=np.float64).reshape(L, M)
    return {"e2": (b * b).sum(axis=1), "m1": (b * np.arange(M)[None, :]).sum(axis=1), "mx": b.max(axis=1)}


def decode_stats(ref, amp_test_fn, y, Pl, L, M, T, Ab, Az, prefix):
    out = {}
    for t in (1, 8):
        b = ref.amp(y, 0, Pl, L, M, t, Ab, Az, mg.zeros(L, M))
        out.update({f"{prefix}_t{t}_{k}": v for k, v in stats(b, L, M).items()})
    bfin, tstop = amp_test_fn(y, 0, Pl, L, M, T, Ab, Az, mg.zeros(L, M))
    out.update({f"{prefix}_final_{k}": v for k, v in stats(bfin, L, M).items()})
    out[f"{prefix}_t_stop"] = int(tstop)
    return out


def main():
    ref = mg.load_reference()
    ref.fht_inplace = mg.fast_fht  # bitwise-equal to the fallback (make_golden.py §1)
    import amp_test as ref_amp_test
    out = {}
    # ---- C2 ----
    g = np.load(os.path.join(HERE, "c2.npz"))
    L, M, P, T, n = int(g["L"]), int(g["M"]), float(g["P"]), int(g["T"]), int(g["n"])
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    assert mg.sha(ordering) == str(g["ordering_sha256"])
    _, y = mg.rep_inputs(ref, L, M, n, Pl, float(g["sigma"]), Ab, 1000)
    assert np.array_equal(y, g["y"])
    t0 = time.time()
    out.update(decode_stats(ref, ref_amp_test.amp_test, y, Pl, L, M, T, Ab, Az, "c2"))
    assert out["c2_t_stop"] == int(g["t_stop"])
    print(f"c2 {time.time() - t0:.1f} s", flush=True)
    # ---- C4 ----
    g = np.load(os.path.join(HERE, "c4.npz"))
    L, M, P, T, n = int(g["L"]), int(g["M"]), float(g["P"]), int(g["T"]), int(g["n"])
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    assert mg.sha(ordering) == str(g["ordering_sha256"])
    for k in (0, 1):
        _, y = mg.rep_inputs(ref, L, M, n, Pl, float(g[f"sigma_{k}"]), Ab, 2000 + k)
        assert np.array_equal(y, g[f"y_{k}"])
        t0 = time.time()
        out.update(decode_stats(ref, ref_amp_test.amp_test, y, Pl, L, M, T, Ab, Az, f"c4_{k}"))
        assert out[f"c4_{k}_t_stop"] == int(g[f"t_stop_{k}"])
        print(f"c4 codeword {k} {time.time() - t0:.1f} s", flush=True)
    np.savez_compressed(os.path.join(HERE, "sections.npz"), **out)


if __name__ == "__main__":
    main()
