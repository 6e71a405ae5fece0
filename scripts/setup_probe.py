"""Where the l768 sweep's host set-up time goes (diagnostic): the HIP runtime's
first call, the ordering, the operator (tables built and uploaded), the
batched kernel's bank-aware tables (reserve), the native draws alone."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
t0 = time.time()
import sparc_ldpc_amd as sp  # noqa: E402
t1 = time.time()
lib = sp.load_library()
ndev = lib.sa_device_count()
t2 = time.time()
L, M, T = 768, 512, 64
R = (L * 9 - 9 * 569 * (1 - 5 / 6)) / (L * 9)
n = int(L * 9 / R)
o = sp.make_ordering(L, M, n)
t3 = time.time()
op = sp.SparcOperator(L, M, n, o, precision="fp32")
t4 = time.time()
op.reserve(256, T)
t5 = time.time()
op2 = sp.SparcOperator(L, M, n, o, precision="fp32")
t6 = time.time()
idx, noise = sp.draw_reps(range(10000), L, M, n, 0.6)
t7 = time.time()
print(f"import {t1 - t0:.3f} first HIP call {t2 - t1:.3f} ordering {t3 - t2:.3f} operator {t4 - t3:.3f} "
      f"reserve (banked tables) {t5 - t4:.3f} second operator {t6 - t5:.3f} draws {t7 - t6:.3f} s")
