"""GPU parity of a caller's own dense design on the device (SA_BACKEND_MATRIX,
``sparc_ldpc_amd.dense_transforms``): the reference's amp() takes any pair of
callables (sparc_ldpc.py:189,213,220), e.g. ``lambda b: A @ b`` /
``lambda z: A.T @ z`` for an i.i.d. Gaussian A (BASELINE north_star's
"Gaussian design-matrix GEMVs").  Checked against the oracle's loop with those
NumPy lambdas on the same A:

  * operator products: 1e-6 (binary32) / 1e-13 (binary64) norm-relative;
  * decodes: 1e-5 (binary32) / 1e-11 (binary64) norm-relative and identical
    section argmax — one codeword (fp32 / fp64 GEMVs) and batches (f32 / f64
    MFMA GEMMs, dense_mfma.hip), with shapes whose L*M and n are not whole GEMM
    stages and a section size that is not a power of two.
"""
import numpy as np
import pytest

from oracle import amp_oracle as orc

pytestmark = pytest.mark.gpu

TOL = {"fp32": 1e-5, "fp64": 1e-11}
OPTOL = {"fp32": 1e-6, "fp64": 1e-13}


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def sp(lib_gpu):
    import sparc_ldpc_amd
    return sparc_ldpc_amd


def gaussian_case(L, M, n, P, sigma, B, seed):
    """A ~ N(0, 1/n) i.i.d. (unit-norm columns on average), B codewords:
    one-hot sections at amplitude sqrt(n Pl), y = A beta0 + sigma w."""
    rs = np.random.RandomState(seed)
    A = rs.randn(n, L * M) / np.sqrt(n)
    Pl = P / L * np.ones(L)
    idx = rs.randint(0, M, (B, L))
    beta0 = np.zeros((B, L * M))
    for b in range(B):
        beta0[b, np.arange(L) * M + idx[b]] = np.sqrt(n * Pl)
    ys = beta0 @ A.T + sigma * rs.randn(B, n)
    return A, Pl, idx, ys


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("L,M,n", [(32, 64, 384), (7, 48, 100), (20, 100, 333)])
def test_matrix_operator_products(sp, prec, L, M, n):
    """A beta and A^T z: one codeword (GEMV) and batches of 4 and 70 (GEMMs:
    a partial codeword tile, K splits)."""
    A, _, _, _ = gaussian_case(L, M, n, 1.0, 0.5, 1, 11)
    Ab, Az = sp.dense_transforms(A, L, M, precision=prec)
    rs = np.random.RandomState(2)
    b1 = rs.randn(L * M, 1); z1 = rs.randn(n, 1)
    assert Ab(b1).shape == (n, 1) and Az(z1).shape == (L * M, 1)
    assert rel(Ab(b1), A @ b1) <= OPTOL[prec]
    assert rel(Az(z1), A.T @ z1) <= OPTOL[prec]
    op = Ab.op
    for B in (4, 70):
        bb = rs.randn(B, L * M); zz = rs.randn(B, n)
        assert rel(op.Ab_batch(bb), bb @ A.T) <= OPTOL[prec], B
        assert rel(op.Az_batch(zz), zz @ A) <= OPTOL[prec], B
        assert op.plan(B)["section_kernel"] == "matrix_mfma"
    assert op.plan(1)["section_kernel"] == "dense"


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_gaussian_amp_vs_oracle_lambdas(sp, prec):
    """amp() on the device with dense_transforms(A) against the oracle's amp()
    with lambda b: A @ b, lambda z: A.T @ z: fixed T before convergence, and
    at convergence (section argmax equal, every section recovered)."""
    L, M, P, sigma = 64, 128, 2.0, 0.5
    n = int(L * np.log2(M))  # R = 1
    A, Pl, idx, ys = gaussian_case(L, M, n, P, sigma, 1, 5)
    y = ys[0].reshape(-1, 1)
    Ab, Az = sp.dense_transforms(A, L, M, precision=prec)
    lAb, lAz = (lambda b: A @ b), (lambda z: A.T @ z)
    for T in (1, 3, 6):
        ref = orc._amp_core(y, Pl, L, M, T, lAb, lAz, None, early_stop=False)[0]
        b = sp.amp(y, 0, Pl, L, M, T, Ab, Az, early_stop=False)
        assert rel(b, ref) <= TOL[prec], T
    ref = orc.amp(y, 0, Pl, L, M, 25, lAb, lAz)
    b = sp.amp(y, 0, Pl, L, M, 25, Ab, Az)
    assert rel(b, ref) <= TOL[prec]
    assert np.array_equal(orc.section_argmax(b, L, M), orc.section_argmax(ref, L, M))
    assert np.array_equal(orc.section_argmax(b, L, M), idx[0])
    if prec == "fp64":  # the exact-tau stop index within a few iterations of the reference's
        _, t = sp.amp_test(y, 0, Pl, L, M, 40, Ab, Az, precision="operator")
        _, rt = orc.amp_test(y, 0, Pl, L, M, 40, lAb, lAz)
        assert abs(t - rt) <= 3


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
@pytest.mark.parametrize("L,M,n,B", [(64, 128, 448, 70), (9, 48, 123, 6)])
def test_gaussian_batched_decode_vs_oracle(sp, prec, L, M, n, B):
    """B codewords through the MFMA GEMM path, each against the oracle loop
    with the NumPy lambdas; with a beta0 start as well."""
    A, Pl, idx, ys = gaussian_case(L, M, n, 2.0, 0.4, B, 7)
    Ab, Az = sp.dense_transforms(A, L, M, precision=prec)
    op = Ab.op
    assert op.plan(B)["section_kernel"] == "matrix_mfma"
    lAb, lAz = (lambda b: A @ b), (lambda z: A.T @ z)
    T = 5
    bb, it = op.amp_batch(ys, Pl, T, early_stop=False)
    for i in sorted({0, 1, B // 2, B - 1}):
        ref = orc._amp_core(ys[i].reshape(-1, 1), Pl, L, M, T, lAb, lAz, None, early_stop=False)[0]
        assert rel(bb[i], ref) <= TOL[prec], i
    b0 = np.abs(np.random.RandomState(3).randn(B, L * M)) * 0.1
    bb0, _ = op.amp_batch(ys, Pl, 3, beta0=b0, early_stop=False)
    for i in (0, B - 1):
        ref = orc._amp_core(ys[i].reshape(-1, 1), Pl, L, M, 3, lAb, lAz, b0[i].reshape(-1, 1),
                            early_stop=False)[0]
        assert rel(bb0[i], ref) <= TOL[prec], i
    # converged batch: every codeword's sections recovered, the stop fired
    bc, itc = op.amp_batch(ys, Pl, 60)
    dec = bc.reshape(B, L, M).argmax(2)
    assert np.array_equal(dec, idx)
    assert (itc < 60).all()


def test_matrix_refuses_ordering_only_entry_points(sp):
    A, Pl, idx, ys = gaussian_case(8, 16, 40, 1.0, 0.3, 2, 1)
    Ab, Az = sp.dense_transforms(A, 8, 16, precision="fp32")
    op = Ab.op
    op.stage_power(2, Pl)
    with pytest.raises(sp.SparcAmpError):
        op.encode(idx)
    with pytest.raises(ValueError):
        op.subset([0, 1])
    with pytest.raises(AssertionError):
        sp.dense_transforms(A[:, :-1], 8, 16)


@pytest.mark.parametrize("prec", ["fp32", "fp64"])
def test_device_gaussian_design(sp, prec):
    """sa_create_matrix_random: the device-generated N(0, 1/n) design.  Its
    columns (A e_j, through the GEMV and the GEMM paths alike) have the right
    moments, the same seed gives the same matrix bit for bit and another seed
    another one, A^T is the adjoint of A, and AMP over it recovers every
    section at high SNR."""
    L, M, n = 16, 64, 200
    Ab, Az = sp.gaussian_transforms(L, M, n, seed=7, precision=prec)
    op = Ab.op
    E = np.eye(L * M)
    cols = op.Ab_batch(E).T  # (n, L*M): column j = A e_j (GEMM path, B = L*M)
    single = np.hstack([Ab(E[j].reshape(-1, 1)) for j in (0, 5, L * M - 1)])
    assert np.array_equal(single, cols[:, [0, 5, L * M - 1]]) or rel(single, cols[:, [0, 5, L * M - 1]]) <= 1e-7
    x = cols.reshape(-1) * np.sqrt(n)
    assert abs(x.mean()) < 5 / np.sqrt(x.size) and abs(x.std() - 1) < 0.02
    assert abs(np.mean(x ** 4) - 3) < 0.1  # Gaussian kurtosis
    again = sp.SparcOperator.from_random(L, M, n, seed=7, precision=prec).Ab_batch(E[:8])
    other = sp.SparcOperator.from_random(L, M, n, seed=8, precision=prec).Ab_batch(E[:8])
    assert np.array_equal(again, cols[:, :8].T)
    assert not np.allclose(other, again)
    rs = np.random.RandomState(1)
    z = rs.randn(n, 1)
    assert rel(Az(z), cols.T @ z) <= OPTOL[prec] * 10
    P = 2.0
    Pl = P / L * np.ones(L)
    idx = rs.randint(0, M, L)
    b0 = np.zeros((L * M, 1)); b0[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
    y = Ab(b0) + 0.05 * rs.randn(n, 1)
    b = sp.amp(y, 0, Pl, L, M, 30, Ab, Az)
    assert np.array_equal(orc.section_argmax(b, L, M), idx)
    ref = orc.amp(y, 0, Pl, L, M, 30, lambda v: cols @ v, lambda v: cols.T @ v)
    assert rel(b, ref) <= 1e-4
