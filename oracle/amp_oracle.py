"""CPU oracle for the SPARC AMP hot path — TEST INFRASTRUCTURE ONLY.

This module is a NumPy restatement of the reference algorithm in
``Spimp/sparc_ldpc`` (``ldpc/sparc_ldpc.py``).  It exists so that ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg have a
CPU checker.  Nothing under ``sparc_ldpc_amd/`` imports it, and the product
path never routes through it: the product runs the HIP library
(``sparc_ldpc_amd/csrc``) or fails.

Parity status: pinned.  ``tests/golden/make_golden.py`` imported the
reference itself in the build container and wrote the fixtures under
``tests/golden/``.  ``tests/test_oracle.py`` checks this restatement against
those fixtures bit for bit in fp64.  ``pyfht`` (the reference's optional C
FWHT, an unpinned third-party dependency absent from the image) is replaced
by the reference's own in-file fallback definition (sparc_ldpc.py:16-29).
The vectorised transform below performs the same butterflies in the same
order, so its fp64 results are bitwise equal to that fallback; the fixtures
check this too.

Every function cites the reference lines it restates.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "fht_inplace", "sub_fht", "block_sub_fht", "sparc_transforms",
    "sparc_transforms_shorter", "pa_parameterised", "amp", "amp_test",
    "bits2indices", "section_argmax", "ber_indices", "make_ordering",
    "dense_design_matrix", "rep_inputs",
]


def fht_inplace(x: np.ndarray) -> None:
    """Unnormalised natural-order Walsh-Hadamard transform, in place.

    Restates the fallback at sparc_ldpc.py:19-29: butterfly stride N/2 -> 1,
    ``x[j] += x[j|i]; x[j|i] = old_x[j] - x[j|i]``.  Works on the leading axis
    so a (w, B) array transforms B columns at once (same per-column order).
    """
    N = x.shape[0]
    tail = x.shape[1:]
    i = N >> 1
    while i:
        v = x.reshape((N // (2 * i), 2, i) + tail)
        a = v[:, 0].copy()
        b = v[:, 1]
        v[:, 0] = a + b
        v[:, 1] = a - b
        i >>= 1


def _w_of(n: int, m: int) -> int:
    # sparc_ldpc.py:52 / :110
    return 2 ** int(np.ceil(np.log2(max(m + 1, n + 1))))


def make_ordering(L: int, M: int, n: int, seed: int = 0) -> np.ndarray:
    """Row sub-sampling table, sparc_ldpc.py:107-117.

    ``RandomState(seed)``; ``idxs = arange(1, w, uint32)``; per section a
    *cumulative* in-place shuffle, keep the first n.
    """
    w = _w_of(n, M)
    rng = np.random.RandomState(seed)
    ordering = np.empty((L, n), dtype=np.uint32)
    idxs = np.arange(1, w, dtype=np.uint32)
    for ll in range(L):
        rng.shuffle(idxs)
        ordering[ll] = idxs[:n]
    return ordering


def sub_fht(n, m, seed=0, ordering=None):
    """sparc_ldpc.py:32-79 — one n x m block of the sub-sampled Hadamard matrix."""
    assert n > 0, "n must be positive"
    assert m > 0, "m must be positive"
    w = _w_of(n, m)
    if ordering is not None:
        assert ordering.shape == (n,)
    else:
        rng = np.random.RandomState(seed)
        idxs = np.arange(1, w, dtype=np.uint32)
        rng.shuffle(idxs)
        ordering = idxs[:n]

    def Ax(x):  # :65-70
        assert x.size == m, "x must be m long"
        y = np.zeros(w)
        y[w - m:] = x.reshape(m)
        fht_inplace(y)
        return y[ordering]

    def Ay(y):  # :72-77
        assert y.size == n, "input must be n long"
        x = np.zeros(w)
        x.flat[ordering] = y
        fht_inplace(x)
        return x[w - m:]

    return Ax, Ay, ordering


def block_sub_fht(n, m, l, seed=0, ordering=None):
    """sparc_ldpc.py:81-136 — L blocks; Ax accumulates sections in order 0..L-1."""
    assert n > 0 and m > 0 and l > 0
    if ordering is not None:
        assert ordering.shape == (l, n)
    else:
        ordering = make_ordering(l, m, n, seed)

    def Ax(x):  # :120-126
        assert x.size == l * m
        x = np.asarray(x).reshape(-1)
        out = np.zeros(n)
        for ll in range(l):
            ax, _, _ = sub_fht(n, m, ordering=ordering[ll])
            out += ax(x[ll * m:(ll + 1) * m])
        return out

    def Ay(y):  # :128-134
        assert y.size == n
        out = np.empty(l * m)
        for ll in range(l):
            _, ay, _ = sub_fht(n, m, ordering=ordering[ll])
            out[ll * m:(ll + 1) * m] = ay(y)
        return out

    return Ax, Ay, ordering


def sparc_transforms(L, M, n, seed=0):
    """sparc_ldpc.py:140-147 — (Ab, Az, ordering); both scaled by 1/sqrt(n)."""
    Ax, Ay, ordering = block_sub_fht(n, M, L, ordering=None, seed=seed)

    def Ab(b):
        return Ax(b).reshape(-1, 1) / np.sqrt(n)

    def Az(z):
        return Ay(z).reshape(-1, 1) / np.sqrt(n)

    return Ab, Az, ordering


def sparc_transforms_shorter(L, M, n, ordering):
    """sparc_ldpc.py:154-168 — operator over the first L rows of ``ordering``."""
    Ax, Ay, _ = block_sub_fht(n, M, L, ordering=ordering[:L, :])

    def Ab(b):
        return Ax(b).reshape(-1, 1) / np.sqrt(n)

    def Az(z):
        return Ay(z).reshape(-1, 1) / np.sqrt(n)

    return Ab, Az


def pa_parameterised(L, C, P, a, f):
    """sparc_ldpc.py:172-186 — exponential power allocation, flattened after fL."""
    pa = 2 ** (-2 * a * C * np.arange(L) / L)
    pa[int(f * L):] = pa[int(f * L)]
    pa /= pa.sum() / P
    return pa


def _amp_core(y, Pl, L, M, T, Ab, Az, beta, early_stop=True):
    """The loop of sparc_ldpc.py:189-222 (== amp_test.py:14-50), returning (beta, t).

    ``beta`` is None for the zero start.  The reference's sentinel
    ``β.all()==None`` (sparc_ldpc.py:192) no longer recognises its own default
    under NumPy >= 2, so callers pass None explicitly here; the zero start is
    bit-identical to passing zeros because y - Ab(0) == y exactly.
    ``early_stop=False`` (bench.py's CPU baseline only) skips the :204 test so
    that exactly T iterations run, as in the GPU bench.
    """
    P = np.sum(Pl)
    n = y.size
    if beta is None:
        β = np.zeros((L * M, 1))
        z = y
    else:
        β = np.asarray(beta, dtype=np.float64).reshape(L * M, 1)
        z = y - Ab(β)
    last_τ = 0
    t = None
    for t in range(T):
        τ = np.sqrt(np.sum(z ** 2) / n)                      # :203
        if early_stop and τ == last_τ:                        # :204 exact-equality stop
            return β, t
        last_τ = τ
        s = β + Az(z)                                         # :213
        rt_n_Pl = np.sqrt(n * Pl).repeat(M).reshape(-1, 1)    # :214
        u = s * rt_n_Pl / τ ** 2                              # :215
        max_u = u.max()                                       # :216 global max
        exps = np.exp(u - max_u)                              # :217
        sums = exps.reshape(L, M).sum(axis=1).repeat(M).reshape(-1, 1)  # :218
        β = (rt_n_Pl * exps / sums).reshape(-1, 1)            # :219
        z = y - Ab(β) + (z / τ ** 2) * (P - np.sum(β ** 2) / n)  # :220
    return β, t


def amp(y, σ_n, Pl, L, M, T, Ab, Az, β=None):
    """sparc_ldpc.py:189-222.  ``σ_n`` is unused by the reference as well."""
    y = np.asarray(y, dtype=np.float64)
    if y.ndim == 1:
        y = y.reshape(-1, 1)
    b, _ = _amp_core(y, np.asarray(Pl, dtype=np.float64), L, M, T, Ab, Az, β)
    return b


def amp_test(y, σ_n, Pl, L, M, T, Ab, Az, β=None):
    """amp_test.py:14-50 — as amp() but also returns the loop index t.

    t is the index at which the exact-τ stop fired, or T-1 when the loop ran
    out (Python's ``for`` variable after exhaustion).
    """
    y = np.asarray(y, dtype=np.float64)
    if y.ndim == 1:
        y = y.reshape(-1, 1)
    return _amp_core(y, np.asarray(Pl, dtype=np.float64), L, M, T, Ab, Az, β)


def bits2indices(bits, m):
    """sparc_ldpc.py:317-341 — MSB-first, log2(m) bits per section."""
    logm = int(np.log2(m))
    assert len(bits) % logm == 0
    b = np.asarray(bits, dtype=np.int64).reshape(-1, logm)
    weights = 1 << np.arange(logm - 1, -1, -1, dtype=np.int64)
    return (b * weights).sum(axis=1).tolist()


def section_argmax(beta, L, M):
    """sparc_ldpc.py:452-455 — first index of the max in each section."""
    return np.asarray(beta).reshape(L, M).argmax(axis=1)


def ber_indices(a, b, total_bits):
    """sparc_ldpc.py:462 — sum of popcount(a ^ b) / total_bits."""
    x = np.bitwise_xor(np.asarray(a, dtype=np.int64), np.asarray(b, dtype=np.int64))
    return sum(bin(int(v)).count("1") for v in x) / total_bits


def dense_design_matrix(L, M, n, ordering):
    """Materialise A (n x L*M) from the FWHT definition; used to cross-check.

    A[r, l*M + c] = (-1)^popcount(ordering[l, r] & (w - M + c)) / sqrt(n)
    (natural-order Hadamard, sparc_ldpc.py:65-77 + :143-146).
    """
    w = _w_of(n, M)
    cols = (w - M + np.arange(M, dtype=np.uint64))
    A = np.empty((n, L * M))
    for l in range(L):
        o = ordering[l].astype(np.uint64)[:, None] & cols[None, :]
        pc = np.zeros(o.shape, dtype=np.uint64)
        v = o.copy()
        while np.any(v):
            pc += v & np.uint64(1)
            v >>= np.uint64(1)
        A[:, l * M:(l + 1) * M] = np.where(pc & np.uint64(1), -1.0, 1.0)
    return A / np.sqrt(n)


def rep_inputs(L, M, n, Pl, sigma, Ab, seed):
    """Synthetic Monte-Carlo rep: RandomState(seed) draws the
    section indices uniform in [0, M) and the noise N(0, σ²); encoding and
    channel follow sparc_ldpc.py:436-446."""
    rs = np.random.RandomState(seed)
    idx = rs.randint(0, M, L)
    beta0 = np.zeros((L * M, 1))
    beta0[np.arange(L) * M + idx, 0] = np.sqrt(n * np.asarray(Pl))
    x = Ab(beta0)
    y = (x + rs.randn(n, 1) * sigma).reshape(-1, 1)
    return idx, y
