"""AMP decoder entry points: drop-ins for ldpc/sparc_ldpc.py:189-222 and
ldpc/amp_test.py:14-50, running the whole iteration loop on the MI355X.

``amp(y, σ_n, Pl, L, M, T, Ab, Az, β)`` keeps the reference's positional
order (every call site is positional: sparc_ldpc.py:449,524,637,698,796,846,
954,1017; amp_exit.py:238; amp_test.py:214,231,240).  With the operator
objects of this package's ``sparc_transforms`` / ``sparc_transforms_shorter``
(what every reference call site passes) the whole loop runs on the device.
Like the reference, ``amp`` also accepts any other pair of callables: those
are the caller's operator and run where the caller wrote them, while τ, the
exact-τ stop, η and the Onsager residual still run on the device
(``HostOperatorLoop``, binary64).
"""
from __future__ import annotations

import warnings

import numpy as np

from .operators import AbOp, AzOp, SparcOperator, _cached_operator, host_loop

__all__ = ["amp", "amp_test", "amp_batch", "operator_of"]


def operator_of(Ab, Az) -> SparcOperator:
    if not (isinstance(Ab, AbOp) and isinstance(Az, AzOp)):
        raise TypeError(
            "amp() runs on the MI355X and needs the Ab/Az objects returned by "
            "sparc_ldpc_amd.sparc_transforms / sparc_transforms_shorter; got "
            f"{type(Ab).__name__}/{type(Az).__name__}")
    if Ab.op is not Az.op:
        raise ValueError("Ab and Az belong to different operators")
    return Ab.op


def _beta0(β, L, M):
    """None / the reference's ``np.array([None])`` sentinel -> zero start.

    The reference tests ``β.all()==None`` (sparc_ldpc.py:192); under NumPy 2
    that no longer recognises its own default and the call crashes
    (SURVEY §0.5).  Any all-None object array is treated as "absent" here;
    a numeric β₀ of any shape with L*M values is used as given (amp_test.py
    passes unscaled 0/1 vectors, :203-204).
    """
    if β is None:
        return None
    a = np.asarray(β)
    if a.dtype == object:
        if all(v is None for v in a.reshape(-1)):
            return None
        a = a.astype(np.float64)
    a = np.asarray(a, dtype=np.float64)
    assert a.size == L * M, "β must hold L*M values"  # β.reshape(L*M,1), :197
    return a.reshape(1, L * M)


def _run(y, Pl, L, M, T, Ab, Az, β, early_stop):
    if isinstance(Ab, AbOp) and isinstance(Az, AzOp) and Ab.op is not Az.op:
        # two of this package's operators that do not belong together: a
        # caller's mistake, not a foreign operator for the host loop
        raise ValueError("Ab and Az belong to different operators")
    if not (isinstance(Ab, AbOp) and isinstance(Az, AzOp)):
        # the caller's own operator (sparc_ldpc.py:189 takes any callables)
        if not (callable(Ab) and callable(Az)):
            raise TypeError(f"Ab and Az must be callable; got {type(Ab).__name__}/{type(Az).__name__}")
        y = np.asarray(y, dtype=np.float64)
        loop = host_loop(L, M, y.size)
        b, it = loop.run(y, Pl, T, Ab, Az, _beta0(β, L, M), early_stop)
        return b, it
    op = operator_of(Ab, Az)
    assert L == op.L and M == op.M, "L, M must match the operator"
    y = np.asarray(y, dtype=np.float64)
    assert y.size == op.n, "y must be n long"  # n = y.size, :191
    Pl = np.asarray(Pl, dtype=np.float64).reshape(-1)
    assert Pl.size == L, "Pl must hold one power per section"
    out, iters = op.amp_batch(y.reshape(1, -1), Pl, T, _beta0(β, L, M), early_stop)
    return out.reshape(-1, 1), int(iters[0])


def amp(y, σ_n, Pl, L, M, T, Ab, Az, β=None, *, early_stop=True):
    """sparc_ldpc.py:189-222 -> β̂ of shape (L*M, 1), float64.

    σ_n is accepted and ignored, as in the reference.
    """
    b, _ = _run(y, Pl, L, M, T, Ab, Az, β, early_stop)
    return b


def _sibling(Ab, Az, precision):
    """The same design (ordering, backend, device) as a cached operator of
    another device precision; None when Ab/Az are not this package's
    matrix-free operators or already run in `precision`."""
    if not (isinstance(Ab, AbOp) and isinstance(Az, AzOp) and Ab.op is Az.op):
        return None
    op = Ab.op
    if op.precision == precision or op.backend != "hadamard":
        return None
    sib = _cached_operator(op.L, op.M, op.n, op.ordering, op.backend, precision, op.device)
    return AbOp(sib), AzOp(sib)


_SWAP_WARNED = False


def amp_test(y, σ_n, Pl, L, M, T, Ab, Az, β=None, *, early_stop=True, precision="fp64"):
    """amp_test.py:14-50 -> (β̂, t): t is the loop index at which the exact
    τ stop fired, or T-1 when the loop ran out (Python's loop variable).

    The stop index is part of this function's contract, and it depends on
    the arithmetic: τ repeats exactly once the iterates reach a fixed point
    to the last ulp (sparc_ldpc.py:204), which binary32 iterates reach
    earlier than the reference's binary64 ones (C4 codeword 0: t = 38 in
    binary32 against the reference's 63).  So by default the decode runs in
    binary64 (``precision="fp64"``: a binary32 operator of this package is
    swapped for its cached binary64 twin, same design), where t lies within
    3 iterations of the reference's (tests/test_gpu_parity.py::
    test_stop_index_vs_reference).  ``precision="operator"`` keeps the
    operator's own precision (binary32: the stop index of binary32 iterates,
    bounded in the same test; β̂ within the fp32 contract either way)."""
    if precision not in ("fp64", "fp32", "operator"):
        raise ValueError("precision must be 'fp64', 'fp32' or 'operator'")
    if precision != "operator":
        sib = _sibling(Ab, Az, precision)
        if sib is not None:
            global _SWAP_WARNED
            if not _SWAP_WARNED:  # once per process: the swap changes the arithmetic and the cost
                _SWAP_WARNED = True
                warnings.warn(f"amp_test decodes a {Ab.op.precision} operator in {precision} (a cached twin of the "
                              f"same design) so that its stop index follows the reference's binary64 "
                              f"iterates; pass precision='operator' to keep the operator's own precision",
                              stacklevel=2)
            Ab, Az = sib
    b, it = _run(y, Pl, L, M, T, Ab, Az, β, early_stop)
    return b, (it if it < T else T - 1)


def amp_batch(y, Pl, T, Ab, Az=None, beta0=None, *, early_stop=True):
    """Batched decode of B independent codewords sharing one operator.

    y: (B, n); beta0: None or (B, L*M).  Returns (β̂ (B, L*M), iters (B,)),
    iters as in ``SparcOperator.amp_batch``.
    """
    op = Ab if isinstance(Ab, SparcOperator) else operator_of(Ab, Az)
    y = np.asarray(y, dtype=np.float64)
    if y.ndim == 1:
        y = y.reshape(1, -1)
    return op.amp_batch(y, Pl, T, beta0, early_stop)
