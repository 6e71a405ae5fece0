import sys; sys.path.insert(0, '.')
import numpy as np
import sparc_ldpc_amd as sp
from sparc_ldpc_amd.joint import draw_reps
from sparc_ldpc_amd.harness import _popcount
L, M, n, T, sigma = 64, 16, 256, 30, 0.93
code = sp.code("802.16", "5/6", 8)
np.random.seed(1)
idx, noise = draw_reps(code, L, M, n, np.random, 1, sigma)
Pl = 4.0 / L * np.ones(L)
op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n, 0), None, "fp64")
op.reserve(1, T)
op.stage_power(1, Pl)
op.encode(idx, noise)
for rep in range(2):
    op.run(1, T)
    op.wait()
    rx = op.decide(1)
    b, it = op.fetch(1)
    print(sys.argv[1:], rep, "errs", int(_popcount(np.bitwise_xor(idx.astype(np.int64), rx.astype(np.int64))).sum()),
          "norm", float(np.linalg.norm(b)), "nan", int(np.isnan(b).sum()), flush=True)
