"""Diagnostic: in-kernel shader clock of the int8 GEMM (k_gemm_i8) on the
dense backend's batched path, from s_memtime / s_memrealtime stamps of
workgroup 0 around its K loop (MI355X_MICROARCH.md: MFMA-dense loops hold
1.5-1.7 GHz).  Run with SPARC_AMP_LIB=sparc_ldpc_amd/libsparc_amp_stamps.so
(`make -C sparc_ldpc_amd/csrc stamps`) on the GPU box."""
import ctypes as ct
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparc_ldpc_amd as sp  # noqa: E402
from bench import WORKLOADS, n_of, synth_y  # noqa: E402

w = dict(WORKLOADS["c3"])
L, M, P, T, B = w["L"], w["M"], w["P"], w["T"], w["B"]
n = n_of(w)
Pl = P / L * np.ones(L)
op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense")
y = synth_y(op, Pl, w["sigma"], list(range(B)))
op.reserve(B, T)
op.stage(y, Pl)
lib = sp.load_library()
lib.sa_debug_stamps.argtypes = [ct.POINTER(ct.c_ulonglong)]
t0 = time.time()
clk = []
while time.time() - t0 < 3.0:  # >= 2 s of back-to-back launches first (the guide's recipe)
    op.run(B, T, early_stop=False)
    op.wait()
    st = (ct.c_ulonglong * 16)()
    lib.sa_debug_stamps(st)
    dt, dr = st[14] - st[12], st[15] - st[13]
    if dr > 0 and time.time() - t0 > 2.0:
        clk.append(dt / dr * 0.1)  # GHz
print(f"k_gemm_i8 in-kernel clock (workgroup 0, last GEMM of each decode): median {np.median(clk):.3f} GHz "
      f"over {len(clk)} decodes (min {min(clk):.3f}, max {max(clk):.3f})")
