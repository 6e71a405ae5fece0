"""ADVICE r05 (ldpc_bp.hip device-sized tail): the cost of the tail launches a
non-blocking decode (lb_run) queues up to max_iter even when no word enters
the tail.  802.16 rate 5/6 z=192 (the C5 outer code), B words at an easy
Eb/N0 where every word converges inside the first phase: lb_run with the
device-sized tail (tail_at = 8: 2 x 192 queued launches that return at once),
the same with the tail off (lb_set_tail(0): one launch), and the host-sized
lb_decode (which stops issuing once every word is done)."""
import ctypes as ct
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from sparc_ldpc_amd import ldpc  # noqa: E402

c = ldpc.code("802.16", "5/6", 192)
lib = ldpc.load_bp_library()
D = ct.POINTER(ct.c_double)
rs = np.random.RandomState(0)
for B in (128, 256):
    U = rs.randint(0, 2, (B, c.K))
    X = c.encode_batch(U)
    ebno = 8.0
    sigma = np.sqrt(1.0 / (2 * (c.K / c.N) * 10 ** (ebno / 10)))
    CH = np.ascontiguousarray(2 * ((1 - 2 * X) + sigma * rs.randn(B, c.N)) / sigma ** 2)
    ctx = c._context()
    res = {}
    for tag, tail in (("device_tail", -1), ("tail_off", 0)):
        lib.lb_set_tail(ctx, tail)
        assert lib.lb_stage(ctx, B, CH.ctypes.data_as(D)) == 0
        lib.lb_run(ctx, B, 0, 0.7, 200); lib.lb_wait(ctx)
        ms = []
        for _ in range(5):
            lib.lb_run(ctx, B, 0, 0.7, 200); lib.lb_wait(ctx)
            ms.append(lib.lb_run_event_ms(ctx))
        it = np.empty(B, dtype=np.intc)
        app = np.empty((B, c.N))
        lib.lb_fetch(ctx, B, app.ctypes.data_as(D), it.ctypes.data_as(ct.POINTER(ct.c_int)))
        res[tag] = (min(ms), int(it.max()))
    lib.lb_set_tail(ctx, -1)
    app = np.empty((B, c.N))
    it = np.empty(B, dtype=np.intc)
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        lib.lb_decode(ctx, B, CH.ctypes.data_as(D), app.ctypes.data_as(D), it.ctypes.data_as(ct.POINTER(ct.c_int)), 0, 0.7, 200)
        t.append((time.perf_counter() - t0) * 1e3)
    print(f"B={B} Eb/N0={ebno} dB max iterations {res['tail_off'][1]}: lb_run device-sized tail "
          f"{res['device_tail'][0]:.3f} ms, tail off {res['tail_off'][0]:.3f} ms (queued empty launches "
          f"{res['device_tail'][0] - res['tail_off'][0]:.3f} ms); lb_decode host-sized {min(t):.3f} ms wall",
          flush=True)
