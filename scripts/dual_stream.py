"""Diagnostic: does running two batched decodes on two contexts (two HIP
streams) concurrently beat one context with the whole batch?  c3-like:
L=M=512 n=4608 T=64, fp32 (or fp64 with argv[1] == 'fp64')."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparc_ldpc_amd as sp
from bench import synth_y

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
L = M = 512; n = 4608; T = 64; P = 4.0; sigma = float(np.sqrt(4.0 / 10 ** 0.5))
Pl = P / L * np.ones(L)
ords = sp.make_ordering(L, M, n)
ops = [sp.SparcOperator(L, M, n, ords, precision=prec, device=0) for _ in range(2)]

def setup(op, B, base):
    y = synth_y(op, Pl, sigma, [base + i for i in range(B)])
    op.reserve(B, T); op.stage(y, Pl)

def timeit(fn, reps=5):
    fn(); [o.wait() for o in ops]
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    [o.wait() for o in ops]
    return (time.perf_counter() - t0) / reps

for B in (256, 512):
    setup(ops[0], B, 0)
    t1 = timeit(lambda: ops[0].run(B, T, early_stop=False))
    setup(ops[0], B // 2, 0); setup(ops[1], B // 2, 10000)
    t2 = timeit(lambda: (ops[0].run(B // 2, T, early_stop=False), ops[1].run(B // 2, T, early_stop=False)))
    print(f"{prec} B={B}: one context {B / t1:9.1f} cw/s | two contexts x {B // 2} concurrently {B / t2:9.1f} cw/s", flush=True)
