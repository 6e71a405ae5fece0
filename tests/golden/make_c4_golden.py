"""Golden fixture for BASELINE configs[3] (L=768 M=512 R=5/6 P=1.8, n=8294,
w=16384) by importing the reference itself (build container only).

Run from the repo root:  python tests/golden/make_c4_golden.py

Same rules and workarounds as make_golden.py (which it imports for the
reference loader, the bit-checked vectorised FHT and the rep draw order):
only the reference's own functions are executed, and only their outputs are
recorded.  Two codewords at sigma = 0.8 and 0.6 (the ends of the σ range of
soft_hard_plot, sparc_ldpc.py:1323, are 0.8 and 0.4): y; beta at t = 1 and
at the exact-tau stop (fp32, the first NS = 64 sections only, to keep the file
small, plus the vector norms); per-section argmax; stop index.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def main():
    ref = mg.load_reference()
    ref.fht_inplace = mg.fast_fht  # bitwise-equal to the fallback (make_golden.py §1)
    import amp_test as ref_amp_test
    L, M, P, R, T = 768, 512, 1.8, 5 / 6, 64
    n = int(L * np.log2(M) / R)
    Pl = P / L * np.ones(L)
    Ab, Az, ordering = ref.sparc_transforms(L, M, n)
    NS = 64
    out = dict(L=L, M=M, n=n, P=P, T=T, NS=NS, ordering_sha256=mg.sha(ordering))
    for k, sigma in enumerate((0.8, 0.6)):
        idx, y = mg.rep_inputs(ref, L, M, n, Pl, sigma, Ab, 2000 + k)
        t0 = time.time()
        b1 = ref.amp(y, 0, Pl, L, M, 1, Ab, Az, mg.zeros(L, M))
        bfin, tstop = ref_amp_test.amp_test(y, 0, Pl, L, M, T, Ab, Az, mg.zeros(L, M))
        print(f"sigma={sigma}: t_stop={tstop} {time.time() - t0:.1f} s", flush=True)
        out.update({f"sigma_{k}": sigma, f"idx_{k}": idx, f"y_{k}": y,
                    f"beta_t1_{k}": b1[:NS * M].astype(np.float32),
                    # norm of the whole t = 1 vector as stored in fp32
                    f"beta_t1_norm_{k}": float(np.linalg.norm(b1.astype(np.float32).astype(np.float64))),
                    f"beta_final_{k}": bfin[:NS * M].astype(np.float32),
                    f"t_stop_{k}": tstop, f"argmax_final_{k}": bfin.reshape(L, M).argmax(1),
                    f"beta_final_norm_{k}": float(np.linalg.norm(bfin))})
    np.savez_compressed(os.path.join(HERE, "c4.npz"), **out)


if __name__ == "__main__":
    main()
