"""GPU parity of the dense backend's batched path: Ab / Az as int8 matrix-core
GEMMs (k_gemm_i8, sparc_ldpc_amd/csrc/dense_i8.hip) on the exact +-1 matrix
with fixed-point vectors of three (z) / four (beta) base-256 digits, for
B >= 4 codewords; and the dense backend's section sizes that are not powers
of two.

Tolerances: the GEMM is exact for the quantised vectors; the quantisation
error is at most 2^-23 of max|v_b| per element and the output is rounded to binary32,
so an operator product is within 1e-6 norm-relative of the fp64 oracle (per
codeword); decodes keep the fp32 contract of the rest of the suite (1e-5
norm-relative, identical section argmax away from near-ties).
"""
import numpy as np
import pytest

from conftest import golden
from oracle import amp_oracle as orc

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def sp(lib_gpu):
    import sparc_ldpc_amd
    return sparc_ldpc_amd


@pytest.mark.parametrize("L,M,R,B", [(16, 8, 1.0, 5), (24, 512, 1.0, 8), (64, 64, 5 / 6, 70), (9, 128, 0.8, 4)])
def test_mfma_operator_products_vs_oracle(sp, L, M, R, B):
    """A beta and A^T z of a batch (sparc_ldpc.py:143-146) against the oracle's
    reference operator, per codeword; codeword tiles of 64 (B = 70: two),
    padded rows (n, L*M not multiples of 256) and K padding covered."""
    n = int(L * np.log2(M) / R)
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense")
    assert op.plan(B)["section_kernel"] == "dense_mfma"
    assert op.plan(3)["section_kernel"] == "dense"
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    rs = np.random.RandomState(L + B)
    beta = rs.randn(B, L * M) * rs.choice([1e-3, 1.0, 30.0], size=(B, 1))  # per-codeword scales differ
    z = rs.randn(B, n)
    z[1] = 0.0  # an all-zero codeword: scale 1, exact zero product
    ab = op.Ab_batch(beta)
    az = op.Az_batch(z)
    for b in range(B):
        assert rel(ab[b], oAb(beta[b].reshape(-1, 1))) <= 1e-6, b
        if b == 1:
            assert not np.any(az[b])
        else:
            assert rel(az[b], oAz(z[b].reshape(-1, 1))) <= 1e-6, b


def test_mfma_decode_vs_oracle(sp):
    """Batched AMP (sparc_ldpc.py:189-222) through the GEMM path vs the oracle,
    per codeword, at fixed t (no early stop) and with the exact-tau stop."""
    L, M, R, P, B, T = 64, 64, 1.0, 2.0, 9, 10
    n = int(L * np.log2(M) / R)
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense")
    Pl = P / L * np.ones(L)
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.6, oAb, 100 + b)[1].reshape(-1) for b in range(B)])
    bb, it = op.amp_batch(ys, Pl, T, early_stop=False)
    assert np.all(it == T)
    for b in range(B):
        ref = orc._amp_core(ys[b].reshape(-1, 1), Pl, L, M, T, oAb, oAz, None, early_stop=False)[0]
        assert rel(bb[b], ref) <= 1e-5, b
        assert np.array_equal(orc.section_argmax(bb[b], L, M), orc.section_argmax(ref, L, M))
    # beta0 start (amp_test.py:231: a 0/1 start) through the quantised init product
    b0 = np.zeros((B, L * M))
    b0[:, ::M] = 1.0
    bb0, _ = op.amp_batch(ys, Pl, 4, beta0=b0, early_stop=False)
    for b in range(B):
        ref = orc._amp_core(ys[b].reshape(-1, 1), Pl, L, M, 4, oAb, oAz, b0[b].reshape(-1, 1), early_stop=False)[0]
        assert rel(bb0[b], ref) <= 1e-5, b


def test_mfma_c2_batch_golden(sp):
    """BASELINE configs[2]'s shape (L = M = 512, n = 4608) on the dense GEMM
    path: the golden C2 codeword in slot 0 of a batch of 64, at t = 1 and at
    convergence (sparc_ldpc.py:202-209, amp_test.py:161-176)."""
    g = golden("c2.npz")
    L, M, n, T = int(g["L"]), int(g["M"]), int(g["n"]), int(g["T"])
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense")
    assert op.plan(64)["section_kernel"] == "dense_mfma"
    Pl = float(g["P"]) / L * np.ones(L)
    rs = np.random.RandomState(3)
    ys = np.stack([g["y"].reshape(-1)] + [g["y"].reshape(-1) + 0.1 * rs.randn(n) for _ in range(63)])
    bt1, _ = op.amp_batch(ys, Pl, 1)
    assert rel(bt1[0], g["beta_t1"]) <= 1e-5
    bb, it = op.amp_batch(ys, Pl, T)
    assert rel(bb[0], g["beta_final"]) <= 1e-5
    assert np.array_equal(orc.section_argmax(bb[0], L, M), g["argmax_final"])
    assert 0 <= it[0] <= T


@pytest.mark.parametrize("L,M,n", [(20, 100, 300), (6, 600, 2000), (9, 48, 200)])
def test_dense_any_section_size_vs_oracle(sp, L, M, n):
    """M not a power of two (the reference's sub_fht takes any M,
    sparc_ldpc.py:32-79; w = 2^ceil(log2(max(M+1, n+1)))): the dense backend's
    fp32 GEMVs (B = 1) and int8 GEMMs (B = 6), and the decode, vs the oracle;
    and the same decode on the matrix-free Hadamard backend (padded sections,
    test_gpu_parity.py::test_hadamard_any_section_size_vs_oracle)."""
    op = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="dense")
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    rs = np.random.RandomState(M)
    beta = rs.randn(6, L * M)
    z = rs.randn(6, n)
    for B in (1, 6):
        ab = op.Ab_batch(beta[:B])
        az = op.Az_batch(z[:B])
        for b in range(B):
            assert rel(ab[b], oAb(beta[b].reshape(-1, 1))) <= 2e-6
            assert rel(az[b], oAz(z[b].reshape(-1, 1))) <= 2e-6
    Pl = 1.5 / L * np.ones(L)
    ys = np.stack([orc.rep_inputs(L, M, n, Pl, 0.4, oAb, 5 + b)[1].reshape(-1) for b in range(6)])
    for B in (1, 6):
        bb, _ = op.amp_batch(ys[:B], Pl, 8, early_stop=False)
        for b in range(B):
            ref = orc._amp_core(ys[b].reshape(-1, 1), Pl, L, M, 8, oAb, oAz, None, early_stop=False)[0]
            assert rel(bb[b], ref) <= 1e-5
            assert np.array_equal(orc.section_argmax(bb[b], L, M), orc.section_argmax(ref, L, M))
    had = sp.SparcOperator(L, M, n, sp.make_ordering(L, M, n), backend="hadamard", precision="fp64")
    hb, _ = had.amp_batch(ys[:6], Pl, 8, early_stop=False)
    for b in range(6):
        ref = orc._amp_core(ys[b].reshape(-1, 1), Pl, L, M, 8, oAb, oAz, None, early_stop=False)[0]
        assert rel(hb[b], ref) <= 1e-11
