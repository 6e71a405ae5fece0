"""Time the HIP BP decoder (802.16 rate 5/6 z=192, the C5 outer code) on
device-resident LLRs: B words per launch, per Eb/N0."""
import ctypes as ct
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from sparc_ldpc_amd import ldpc  # noqa: E402

c = ldpc.code("802.16", "5/6", 192)
lib = ldpc.load_bp_library()
rs = np.random.RandomState(0)
D = ct.POINTER(ct.c_double)
BS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 256, 1024]
for B in BS:
    for ebno in (3.0, 3.5, 4.5):
        U = rs.randint(0, 2, (B, c.K))
        X = c.encode_batch(U)
        r = c.K / c.N
        sigma = np.sqrt(1.0 / (2 * r * 10 ** (ebno / 10)))
        CH = np.ascontiguousarray(2 * ((1 - 2 * X) + sigma * rs.randn(B, c.N)) / sigma ** 2)
        ctx = c._context()
        assert lib.lb_stage(ctx, B, CH.ctypes.data_as(D)) == 0
        lib.lb_run(ctx, B, 0, 0.7, 200); lib.lb_wait(ctx)
        ms = []
        for _ in range(3):
            lib.lb_run(ctx, B, 0, 0.7, 200); lib.lb_wait(ctx)
            ms.append(lib.lb_run_event_ms(ctx))
        it = np.empty(B, dtype=np.intc)
        app = np.empty((B, c.N))
        lib.lb_fetch(ctx, B, app.ctypes.data_as(D), it.ctypes.data_as(ct.POINTER(ct.c_int)))
        errs = int(((app < 0) != X).sum())
        t = min(ms)
        print(f"B={B:5d} EbN0={ebno:.1f} dB  {t:9.3f} ms  {B / t * 1e3:10.0f} words/s  "
              f"mean it {it.mean():6.2f} max it {it.max():3d}  us/word-iter {t * 1e3 / max(1, it.sum()):.3f}  bit errs {errs}",
              flush=True)
