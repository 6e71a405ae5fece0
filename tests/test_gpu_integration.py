"""GPU: the ctypes bindings INTEGRATION.md §2 shows a maintainer adding on the
reference side (the ldpc/py/ldpc.py:859-929 pattern) are executed as written,
block by block, against the library itself, and their results checked:
sa_create + sa_amp against the oracle's amp() (sparc_ldpc.py:189-222), the
host-operator loop around the caller's callables, and the Monte-Carlo stream
(sa_draw_reps + sa_mc_stage + sa_mc_run, amp_test.py:183-246) against the
batched decode of the same seeds.  A stale or wrong snippet fails here."""
import os
import re

import numpy as np
import pytest

from oracle import amp_oracle as orc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. The C ABI"):text.index("## 3. ")]
    return re.findall(r"```python\n(.*?)```", sec, re.S)


def _lib_path():
    import sparc_ldpc_amd._lib as _l
    return _l.LIB_PATH


def test_integration_snippets_run_as_written(lib_gpu):
    import ctypes as ct

    import sparc_ldpc_amd as sp
    blocks = [b.replace("/path/to/sparc_ldpc_amd/libsparc_amp.so", _lib_path()) for b in _blocks()]
    assert len(blocks) == 4, "INTEGRATION.md §2: sa_amp, matrix, host-operator and Monte-Carlo blocks"
    amp_blk, mat_blk, host_blk, mc_blk = blocks

    L, M, T = 128, 256, 12
    n = L * 8  # R = 1
    P = 4.0
    Pl = P / L * np.ones(L)
    rs = np.random.RandomState(5)
    sent = rs.randint(0, M, L)
    c = np.sqrt(n * Pl[0])
    b0 = np.zeros((L * M, 1))
    b0[np.arange(L) * M + sent, 0] = c
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    y = oAb(b0) + 0.4 * rs.randn(n, 1)

    # block 1: sa_create + sa_amp (the Hadamard operator of the reference's ordering)
    ns = {"np": np, "ct": ct, "L": L, "M": M, "n": n, "T": T, "y": y, "Pl": Pl,
          "sparc_transforms": orc.sparc_transforms}
    exec(amp_blk, ns)
    ref = orc.amp(y, 0, Pl, L, M, T, oAb, oAz)
    assert np.linalg.norm(ns["beta"] - ref) <= 1e-5 * np.linalg.norm(ref)

    # block 2: a caller's dense design (small, the binary64 matrix on the host)
    Lm, Mm, nm = 8, 16, 64
    A = np.random.RandomState(1).randn(nm, Lm * Mm) / np.sqrt(nm)
    ns.update(L=Lm, M=Mm, n=nm, A=A)
    exec(mat_blk, ns)
    lib, ctx = ns["lib"], ns["ctx"]
    Plm = P / Lm * np.ones(Lm)
    bm = np.zeros((Lm * Mm, 1))
    bm[np.arange(Lm) * Mm + rs.randint(0, Mm, Lm), 0] = np.sqrt(nm * Plm[0])
    ym = A @ bm + 0.3 * rs.randn(nm, 1)
    D = ct.POINTER(ct.c_double)
    beta_m = np.empty(Lm * Mm)
    assert lib.sa_amp(ctx, 1, ym.ctypes.data_as(D), Plm.ctypes.data_as(D), 6, None, beta_m.ctypes.data_as(D),
                      None, 0) == 0, lib.sa_last_error()
    lib.sa_destroy(ctx)
    ref_m = orc.amp(ym, 0, Plm, Lm, Mm, 6, lambda b: A @ b, lambda z: A.T @ z)
    assert np.linalg.norm(beta_m - ref_m.ravel()) <= 1e-5 * np.linalg.norm(ref_m)

    # block 3: the host-operator loop around the caller's own callables (binary64)
    ns.update(L=L, M=M, n=n, Ab=oAb, Az=oAz, y=np.ascontiguousarray(y.ravel()))
    exec(host_blk, ns)
    assert np.linalg.norm(ns["beta"] - ref.ravel()) <= 1e-11 * np.linalg.norm(ref)
    ns["lib"].sa_destroy(ns["ctx"])

    # block 4: the Monte-Carlo stream (256 slots) against the batched decode of the same seeds
    reps, sigma = 300, 0.5
    ns.update(reps=reps, sigma=sigma)
    exec(mc_blk, ns)
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision="fp32")
    be0, it0 = sp.mc_decode_batched(op, Pl, sigma, T, list(range(reps)), batch=64)
    np.testing.assert_array_equal(ns["errs"], be0)
    np.testing.assert_array_equal(ns["its"], it0)
    assert ns["ms"][0] > 0 and 0 <= ns["ber"] < 0.5
