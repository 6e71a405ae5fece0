"""GPU parity of the host-operator loop: amp() with operators that are not
this package's (the reference's amp() takes any pair of callables,
sparc_ldpc.py:189-222).  The callables run where the caller wrote them; τ,
the exact-τ stop, η and the Onsager residual run on the device in binary64
(SA_BACKEND_HOST).  Checked against the oracle's loop with the SAME
callables: the only differences are summation orders (1e-11 norm-relative).
Covers the reference's Hadamard operator as plain NumPy closures and an
i.i.d. Gaussian design (BASELINE north_star's "Gaussian design-matrix").
"""
import numpy as np
import pytest

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


class Counted:
    """A callable that counts its calls and checks the reference's shapes."""

    def __init__(self, f, rows):
        self.f, self.rows, self.calls = f, rows, 0

    def __call__(self, x):
        assert x.shape[-1] == 1 and x.ndim == 2
        self.calls += 1
        return self.f(x)


def test_reference_operator_as_foreign_callables(sp):
    """The oracle's sparc_transforms closures (sparc_ldpc.py:140-147) passed to
    amp(): fixed T, with the stop, amp_test's t, and a β₀ start."""
    L, M, P, sigma = 32, 64, 2.0, 0.5
    n = int(L * np.log2(M))
    Pl = P / L * np.ones(L)
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    idx, y = orc.rep_inputs(L, M, n, Pl, sigma, oAb, 77)
    ref = orc._amp_core(y, Pl, L, M, 12, oAb, oAz, None, early_stop=False)[0]
    Ab, Az = Counted(oAb, n), Counted(oAz, L * M)
    b = sp.amp(y, 0, Pl, L, M, 12, Ab, Az, early_stop=False)
    assert b.shape == (L * M, 1)
    assert rel(b, ref) <= 1e-11
    assert Ab.calls == 12 and Az.calls == 12  # once each per iteration, as in the reference loop
    # exact-tau stop: the converged estimate, and t within a few iterations of the oracle's
    bs, t = sp.amp_test(y, 0, Pl, L, M, 64, oAb, oAz)
    rs, rt = orc.amp_test(y, 0, Pl, L, M, 64, oAb, oAz)
    assert rel(bs, rs) <= 1e-11 and abs(t - rt) <= 3
    assert np.array_equal(orc.section_argmax(bs, L, M), idx)
    # beta0 (amp_test.py:231: an unscaled 0/1 start)
    b0 = np.zeros((L * M, 1))
    b0[np.arange(L) * M + idx] = 1.0
    r0 = orc._amp_core(y, Pl, L, M, 6, oAb, oAz, b0, early_stop=False)[0]
    assert rel(sp.amp(y, 0, Pl, L, M, 6, oAb, oAz, b0, early_stop=False), r0) <= 1e-11


def test_gaussian_design_foreign_callables(sp):
    """An i.i.d. Gaussian design A ~ N(0, 1/n) applied by NumPy matmuls: the
    same loop as the oracle's with the same callables, and every section
    recovered at high SNR."""
    L, M, P = 64, 16, 1.0
    n = int(L * np.log2(M) / 0.5)
    rs = np.random.RandomState(11)
    A = rs.randn(n, L * M) / np.sqrt(n)
    Ab = lambda b: A @ b       # noqa: E731
    Az = lambda z: A.T @ z     # noqa: E731
    Pl = P / L * np.ones(L)
    idx = rs.randint(0, M, L)
    b0 = np.zeros((L * M, 1))
    b0[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
    y = Ab(b0) + 0.3 * rs.randn(n, 1)
    ref = orc._amp_core(y, Pl, L, M, 20, Ab, Az, None, early_stop=False)[0]
    b = sp.amp(y, 0.3, Pl, L, M, 20, Ab, Az, early_stop=False)
    assert rel(b, ref) <= 1e-11
    assert np.array_equal(orc.section_argmax(b, L, M), idx)


def test_host_context_refuses_device_operator_calls(sp):
    from sparc_ldpc_amd.operators import host_loop
    loop = host_loop(8, 4, 16)
    z = np.zeros((1, 16))
    out = np.empty((1, 32))
    with pytest.raises(sp.SparcAmpError):
        sp._lib.check(loop._lib.sa_Az(loop._ctx, 1, sp._lib.dptr(z), sp._lib.dptr(out)))


def test_foreign_callables_any_section_size(sp):
    """M not a power of two through the host-operator loop (the reference's
    operator with M = 100)."""
    L, M, n = 12, 100, 250
    Pl = 1.0 / L * np.ones(L)
    oAb, oAz, _ = orc.sparc_transforms(L, M, n)
    _, y = orc.rep_inputs(L, M, n, Pl, 0.3, oAb, 3)
    ref = orc._amp_core(y, Pl, L, M, 10, oAb, oAz, None, early_stop=False)[0]
    assert rel(sp.amp(y, 0, Pl, L, M, 10, oAb, oAz, early_stop=False), ref) <= 1e-11
