"""Diagnostic: phase shares of k_secb (batched) from s_memtime stamps (workgroup 0)."""
import ctypes as ct
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparc_ldpc_amd as sp
from bench import WORKLOADS, n_of, synth_y
w = dict(WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c3"])
L, M, P, T, B = w["L"], w["M"], w["P"], w["T"], w["B"]
n = n_of(w); Pl = P / L * np.ones(L)
op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n))
y = synth_y(op, Pl, w["sigma"], list(range(B)))
op.reserve(B, T); op.stage(y, Pl)
lib = sp.load_library(); lib.sa_debug_stamps.argtypes = [ct.POINTER(ct.c_ulonglong)]
names = ["tau", "z->LDS+bar", "gather", "fwht+denoise x CB", "ts+bar+bbp", "rows", "drain"]
acc = np.zeros(7)
for rep in range(10):
    op.run(B, T, early_stop=False); op.wait()
    st = (ct.c_ulonglong * 16)(); lib.sa_debug_stamps(st)
    acc += np.diff(np.array(st[:8], dtype=np.float64))
acc /= 10
for nm, c in zip(names, acc):
    print(f"{nm:18s} {c:9.0f} cycles  {c / acc.sum() * 100:5.1f}%")
print(f"total {acc.sum():.0f} cycles")
