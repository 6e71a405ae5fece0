"""The fused row step (k_sec4f / k_sec43f, SPARC_AMP_FUSE=1): the row step of
iteration t-1 (k_row2) at the head of the section kernel of iteration t, with
an in-kernel hand-off of z_t between the workgroups.

The sums are k_row2's in k_row2's order, so the fused decode must equal the
two-kernel decode BIT FOR BIT: β̂, the stop index and the final residual z, in
both precisions, with and without the exact-τ stop (sparc_ldpc.py:189-222,
amp_test.py:29-35).  A stale read anywhere in the hand-off would show as a
differing bit, so every decode is also repeated (graph replays) and compared.
"""
import os

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sp(lib_gpu):
    import sparc_ldpc_amd as s
    return s


def _op(sp, L, M, n, prec, fuse):
    old = os.environ.get("SPARC_AMP_FUSE")
    os.environ["SPARC_AMP_FUSE"] = "1" if fuse else "0"
    try:
        return sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), precision=prec)
    finally:
        if old is None:
            del os.environ["SPARC_AMP_FUSE"]
        else:
            os.environ["SPARC_AMP_FUSE"] = old


def _decode(op, y, Pl, T, early_stop, reps=1):
    op.reserve(1, T)
    op.stage(y.reshape(1, -1), Pl)
    outs = []
    for _ in range(reps):
        op.run(1, T, early_stop=early_stop)
        op.wait()
        b, it = op.fetch(1)
        outs.append((b.copy(), int(it[0]), op.fetch_z(1).copy()))
    return outs


CASES = [  # golden, y key, L, M, plan name of the fused kernel
    ("c2.npz", "y", "k_sec4f"),
    ("c4.npz", "y_0", "k_sec43f"),
    ("c4.npz", "y_1", "k_sec43f"),
]


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("early_stop", [False, True])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_fused_bit_identical_to_two_kernel_path(sp, prec, early_stop, case):
    fname, ykey, kname = CASES[case]
    g = golden(fname)
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    Pl = float(g["P"]) / L * np.ones(L)
    y = np.asarray(g[ykey], dtype=np.float64).reshape(-1)
    fused = _op(sp, L, M, n, prec, True)
    plain = _op(sp, L, M, n, prec, False)
    if prec == "fp64" and kname == "k_sec4f" and plain.plan(1)["section_kernel"] == "k_sec43":
        kname = "k_sec43f"  # binary64 runs L = 2 x CUs (c2 on 256 CUs) on the triple kernel
    assert fused.plan(1)["section_kernel"] == kname
    assert plain.plan(1)["section_kernel"] == kname[:-1]
    ref = _decode(plain, y, Pl, T, early_stop)[0]
    got = _decode(fused, y, Pl, T, early_stop, reps=6)
    for b, it, z in got:
        assert it == ref[1]
        assert np.array_equal(b, ref[0]), np.abs(b - ref[0]).max()
        assert np.array_equal(z, ref[2]), np.abs(z - ref[2]).max()
    if early_stop and ykey == "y_1":
        assert ref[1] < T  # this codeword stops early: the stop path is covered


@pytest.mark.parametrize("T", [1, 2, 3])
def test_fused_short_decodes(sp, T):
    """T = 1 (no fused launch: K_0 and the last row step), 2, 3."""
    g = golden("c2.npz")
    L, M, n = int(g["L"]), int(g["M"]), int(g["n"])
    Pl = float(g["P"]) / L * np.ones(L)
    y = g["y"].reshape(-1)
    ref = _decode(_op(sp, L, M, n, "fp32", False), y, Pl, T, False)[0]
    got = _decode(_op(sp, L, M, n, "fp32", True), y, Pl, T, False, reps=2)
    for b, it, z in got:
        assert it == ref[1] and np.array_equal(b, ref[0]) and np.array_equal(z, ref[2])


def test_fused_profile_and_batches(sp):
    """The per-launch profile (repeated launches re-arm the arrival target)
    runs through, and batches of more than one codeword keep the two-kernel
    path (the fused kernel needs one workgroup per CU at most)."""
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), 8
    Pl = float(g["P"]) / L * np.ones(L)
    op = _op(sp, L, M, n, "fp32", True)
    op.reserve(2, T)
    op.stage(np.stack([g["y"].reshape(-1)] * 2)[:1], Pl)
    kinds, total = op.profile(1, T, early_stop=False, rep=4)
    assert kinds["k_sec"][1] == T and kinds["k_row"][1] == 2  # ROW_INIT0 + the last row step
    assert total > 0
    assert op.plan(2)["section_kernel"] == "k_sec4"
    op.run(1, T, early_stop=False)
    op.wait()  # a timed-out arrival poll would raise here
