"""Diagnostic: phase shares of the single-codeword section kernel (k_sec4)
from s_memtime stamps of workgroup 0, wave 0 (cycles at the shader clock).
Run with SPARC_AMP_LIB=sparc_ldpc_amd/libsparc_amp_stamps.so on the GPU box
(`make -C sparc_ldpc_amd/csrc stamps`)."""
import ctypes as ct
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparc_ldpc_amd as sp
from bench import WORKLOADS, n_of, synth_y

w = dict(WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c2"])
if len(sys.argv) > 2:  # batch override (e.g. c4 1: the single-codeword k_sec43)
    w["B"] = int(sys.argv[2])
L, M, P, T, B = w["L"], w["M"], w["P"], w["T"], w["B"]
n = n_of(w)
Pl = P / L * np.ones(L)
op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=os.environ.get("STAMPS_PREC", "fp32"),
                      plan=[p for p in os.environ.get("STAMPS_PLAN", "").split(",") if p])
y = synth_y(op, Pl, w["sigma"], list(range(B)))
op.reserve(B, T); op.stage(y, Pl)
lib = sp.load_library()
lib.sa_debug_stamps.argtypes = [ct.POINTER(ct.c_ulonglong)]
# stamp order in time (index 10: after an explicit wait for every global load
# issued so far, i.e. the bucket-table / previous-beta / Ab-table loads)
if op.plan(B)["section_kernel"] == "k_secb":
    order = [0, 1, 2, 3, 4, 5, 6, 7]
    names = ["loads+tau", "z->LDS+bar", "gather", "fwht+denoise+fwht", "T->LDS+bar", "rows", "drain"]
else:
    order = [0, 1, 2, 10, 3, 4, 5, 6, 7, 8, 9]
    names = ["tau+loads", "z->LDS+bar", "wait tables", "gather", "fwht1", "denoise", "fwht2", "ts+bar", "rows",
             "drain"]
acc = np.zeros(len(order) - 1)
allw = []
for rep in range(20):
    op.run(B, T, early_stop=False); op.wait()
    st = (ct.c_ulonglong * 256)()
    lib.sa_debug_stamps(st)
    a = np.array(st[:], dtype=np.float64).reshape(16, 16)
    waves = [w for w in range(16) if a[w, order[0]] > 0 and a[w, order[-1]] > 0]
    v = a[0, order]
    acc += np.diff(v)
    allw.append(a[waves][:, order] - a[0, order[0]])  # every wave's stamps from wave 0's start
acc /= 20
for nm, c in zip(names, acc):
    print(f"{nm:12s} {c:9.0f} cycles  {c / acc.sum() * 100:5.1f}%   (wave 0)")
print(f"total {acc.sum():.0f} cycles")
# per-wave view: when each wave reaches the end of each phase (cycles after
# wave 0's start; mean over the 20 decodes), min / max over the waves
W = np.mean(np.stack(allw), axis=0)
print(f"{W.shape[0]} waves stamped; phase ends (cycles from wave 0's start): min / max over waves, and the spread")
for j, nm in enumerate(names):
    col = W[:, j + 1]
    print(f"  end of {nm:12s} min {col.min():9.0f}  max {col.max():9.0f}  spread {col.max() - col.min():8.0f}")
print("  per wave, end of the last compute phase before the T barrier:",
      " ".join(f"{x:.0f}" for x in W[:, min(4, W.shape[1] - 1)]))
