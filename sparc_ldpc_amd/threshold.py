"""Threshold-initialised exchange and AMP EXIT analysis.

Drop-ins for ``amp_exit.hard_initialisation`` / ``prep_y`` / ``calc_E`` and the
EXIT helpers (ldpc/amp_exit.py:28-351), and for ``soft_amp_ldpc_hardinit``
(ldpc/sparc_ldpc.py:862-1047).  Per codeword: sections whose soft LDPC (or a
priori) output has one entry above the threshold are hard-decided and
cancelled from y; AMP then runs on a shortened operator over the remaining
sections (``sparc_transforms_shorter`` with a fancy-indexed ordering, as the
reference does).  The device does the work: bp2sp + threshold decisions
(``sa_threshold``), cancellation (``sa_cancel``), AMP on the shortened operator,
sp2bp + LLRs (``sa_llr``), and BP.  AMP runs in fp64 (see joint.joint_decoder).
"""
from __future__ import annotations

import csv
import math

import numpy as np

from . import ldpc as _ldpc
from .harness import SPARCParams, LDPCParams, pa_parameterised, _popcount
from .operators import AbOp, SparcOperator, make_ordering, sparc_transforms_shorter

__all__ = ["J", "J_inverse", "gen_bits", "hard_initialisation", "prep_y", "remove_common_zeros", "calc_E",
           "hist_E", "calc_I_e", "polynomial", "soft_amp_ldpc_hardinit", "ber_from_LLRs"]


# ---- J-function approximations (amp_exit.py:28-46) ----------------------------------
def J_inverse(I):
    assert I >= 0 and I <= 1
    if I == 1:
        I = np.clip(I, a_min=None, a_max=0.9999)
        print("Warning clipping I from 1 to 0.9999")
    if I <= 0.3646:
        return 1.09542 * (I ** 2) + 0.214217 * I + 2.33727 * np.sqrt(I)
    return -0.706692 * np.log(0.386013 * (1 - I)) + 1.75017 * I


def J(sigma):
    assert sigma >= 0
    if sigma <= 1.6363:
        return -0.0421061 * (sigma ** 3) + 0.209252 * (sigma ** 2) + -0.00640081 * sigma
    if sigma < 10:
        return 1 - np.exp(0.00181491 * (sigma ** 3) - 0.142675 * (sigma ** 2) - 0.0822054 * sigma + 0.0549608)
    return 1


def gen_bits(length):
    """amp_exit.py:48-50: +-1 bits."""
    return (np.random.randint(0, 2, length) * -2) + 1


def ber_from_LLRs(M, LLR, input_indices, total_bits):
    """sparc_ldpc.py:343-356."""
    logm = int(round(math.log2(M)))
    bits = (np.asarray(LLR) < 0.0).astype(np.int64).reshape(-1, logm)
    idx = (bits * (1 << np.arange(logm - 1, -1, -1))).sum(axis=1)
    return float(_popcount(np.bitwise_xor(np.asarray(input_indices, np.int64), idx)).sum()) / total_bits


_OPS = {}


def _op(L, M, n, seed=0, precision="fp64", device=None):
    """Operator over the seed's ordering (cached), or a fresh random design for
    seed=None (block_sub_fht with RandomState(None), sparc_ldpc.py:107-117)."""
    key = (L, M, n, seed, precision, device)
    op = _OPS.get(key) if seed is not None else None
    if op is None:
        op = SparcOperator(L, M, n, make_ordering(L, M, n, seed), None, precision, device)
        if seed is not None:
            _OPS[key] = op
    return op


def hard_initialisation(beta, L, M, n, ordering, y, Pl, Ab, threshold=0.5, ldpc_sections=None):
    """amp_exit.py:56-122 with the reference's signature and returns
    (y_new, Ab_new, Az_new, amp_sections, L_amp_sections).  ``beta`` is a host
    array of section posteriors (as the reference's callers pass it) and is
    modified in place like the reference's (one-hot c_l for decided sections,
    zeros elsewhere); y - Ab(beta) runs through the device operator ``Ab``."""
    if ldpc_sections is None:
        ldpc_sections = L
    beta_0 = beta
    amp_sections = []
    c = np.sqrt(n * np.asarray(Pl, dtype=np.float64))
    v = beta_0.reshape(-1)
    for l in range(L):
        sec = v[l * M:(l + 1) * M]
        hit = np.nonzero(sec > threshold)[0] if l >= L - ldpc_sections else np.array([], dtype=np.int64)
        sec[:] = 0
        if hit.size == 1:
            sec[hit[0]] = c[l]
        else:
            amp_sections.append(l)
    y_new = y - Ab(beta_0)
    if amp_sections:
        kw = {}
        if isinstance(Ab, AbOp):  # the shortened operator inherits the caller's backend / precision
            kw = dict(backend=Ab.op.backend, precision=Ab.op.precision, device=Ab.op.device)
        Ab_new, Az_new = sparc_transforms_shorter(len(amp_sections), M, n, np.asarray(ordering)[amp_sections, :], **kw)
    else:
        Ab_new = Az_new = None
    return y_new, Ab_new, Az_new, amp_sections, len(amp_sections)


def prep_y(X, L, M, n, sigma_w, P, a=None, f=None, C=None):
    """amp_exit.py:125-159: (y, Ab, Az, Pl, ordering) for +-1 bits X."""
    from .operators import sparc_transforms
    Pl = P / L * np.ones(L) if a is None else pa_parameterised(L, C, P, a, f)
    Xb = (np.asarray(X) - 1) * -1 / 2
    logm = int(round(math.log2(M)))
    idx = (Xb.reshape(L, logm).astype(np.int64) * (1 << np.arange(logm - 1, -1, -1))).sum(axis=1)
    Ab, Az, ordering = sparc_transforms(L, M, n)
    beta0 = np.zeros((L * M, 1))
    beta0[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
    x = Ab(beta0)
    w = np.random.randn(n, 1) * sigma_w
    return (x + w).reshape(-1, 1), Ab, Az, Pl, ordering


def _amp_on_undecided(op, idx_full, Pl, T, M):
    """Cancel decided sections (idx >= 0) from op's staged y and run AMP on the
    rest through a shortened operator; returns (amp_sections, LLRs (len*logm,))."""
    amp_sections = np.nonzero(idx_full[0] < 0)[0]
    if amp_sections.size == 0:
        return amp_sections, None
    sub = op.subset(amp_sections)
    sub.reserve(1, T)
    op.cancel(idx_full, sub)
    sub.stage_power(1, np.asarray(Pl)[amp_sections])
    sub.run(1, T)
    sub.wait()
    return amp_sections, sub.llr(1, 0, amp_sections.size)[0]


def calc_E(X, I_a, snr_dB, sparcparams: SPARCParams, csv_filename=None, threshold=0.5, precision="fp64"):
    """amp_exit.py:185-270: extrinsic LLRs of AMP with threshold hard
    initialisation from synthetic a-priori LLRs A = mu_a X + N_a.  Draws
    np.random in the reference's order (N_a, then the channel noise)."""
    L, M, P, T = sparcparams.L, sparcparams.M, sparcparams.p, sparcparams.t
    logm = int(np.log2(M))
    n = int(L * np.log2(M) / sparcparams.r)
    snr = 10 ** (snr_dB / 20)
    sigma_w = np.sqrt(P / snr)
    sigma_a = J_inverse(I_a)
    mu_a = (sigma_a ** 2) / 2
    X = np.asarray(X)
    N_a = np.random.randn(len(X)) * sigma_a
    A = mu_a * X + N_a
    a, f, C = sparcparams.a, sparcparams.f, sparcparams.C
    Pl = P / L * np.ones(L) if a is None else pa_parameterised(L, C, P, a, f)
    Xb = ((X - 1) * -1 / 2).astype(np.int64).reshape(L, logm)
    idx = (Xb * (1 << np.arange(logm - 1, -1, -1))).sum(axis=1).astype(np.int32)[None, :]
    w = np.random.randn(n, 1) * sigma_w
    op = _op(L, M, n, 0, precision)
    op.reserve(1, T)
    op.stage_power(1, Pl)
    op.encode(idx, w.reshape(1, -1))
    dec = op.threshold(1, 0, L, A, threshold)  # every section is thresholded (ldpc_sections = L)
    E = A
    amp_sections, llr = _amp_on_undecided(op, dec, Pl, T, M)
    if llr is not None:
        pos = (np.arange(logm)[None, :] + logm * amp_sections[:, None]).reshape(-1)
        E[pos] = llr
    np.clip(E, -55, 55, out=E)
    if csv_filename is not None:
        with open(csv_filename, "a") as fh:
            wr = csv.DictWriter(fh, fieldnames=["I_a", "snr_dB", "X", "E"])
            wr.writeheader()
            wr.writerow({"I_a": I_a, "snr_dB": snr_dB, "X": X, "E": E})
    return E


def remove_common_zeros(a, b):
    """amp_exit.py:162-178."""
    rm = np.intersect1d(np.where(a == 0)[0], np.where(b == 0)[0])
    return np.delete(a, rm, None), np.delete(b, rm, None)


def hist_E(X, E, bin_number=500, max_bin=40, min_bin=-40, plot=False, snr_dB="Not given"):
    """amp_exit.py:272-326 (no plotting): (PE_pos, PE_neg, mean_pos, mean_neg, var_pos, var_neg, bin_width)."""
    assert len(E) == len(X)
    X = np.asarray(X)
    ip, ineg = np.where(X == 1)[0], np.where(X == -1)[0]
    bin_width = (max_bin - min_bin) / (bin_number - 1)
    edges = np.linspace(min_bin, max_bin, bin_number)
    PE_pos, _ = np.histogram(E[ip], bins=edges, density=True)
    PE_neg, _ = np.histogram(E[ineg], bins=edges, density=True)
    mids = 0.5 * (edges[1:] + edges[:-1])
    mean_pos = np.average(mids, weights=PE_pos)
    mean_neg = np.average(mids, weights=PE_neg)
    var_pos = np.average((mids - mean_pos) ** 2, weights=PE_pos)
    var_neg = np.average((mids - mean_neg) ** 2, weights=PE_neg)
    return PE_pos, PE_neg, mean_pos, mean_neg, var_pos, var_neg, bin_width


def calc_I_e(PE_pos, PE_neg, bin_width):
    """amp_exit.py:328-351: extrinsic mutual information from the two histograms."""
    PE_pos, PE_neg = remove_common_zeros(PE_pos, PE_neg)
    with np.errstate(divide="ignore", invalid="ignore"):
        integral_neg = PE_neg * np.log2(2 * PE_neg / (PE_neg + PE_pos))
        integral_pos = PE_pos * np.log2(2 * PE_pos / (PE_neg + PE_pos))
    integral_neg[np.isnan(integral_neg)] = 0
    integral_pos[np.isnan(integral_pos)] = 0
    return 1 / 2 * (bin_width * sum(integral_neg) + bin_width * sum(integral_pos))


def polynomial(I_a, I_e):
    """amp_exit.py:400-414: least-squares cubic fit, c[i] multiplies I_a**i."""
    I_a = np.asarray(I_a, dtype=np.float64)
    a = np.stack([I_a ** i for i in range(4)], axis=1)
    return np.linalg.lstsq(a, I_e, rcond=-1)[0]


def soft_amp_ldpc_hardinit(sparcparams: SPARCParams, ldpcparams: LDPCParams, soft_iter, threshold,
                           precision="fp64"):
    """sparc_ldpc.py:862-1047: threshold-initialised exchange, one rep from the
    global np.random stream.  Returns (ber_amp list, ber_ldpc list, R)."""
    L, M, P, sigma, T = sparcparams.L, sparcparams.M, sparcparams.p, sparcparams.sigma, sparcparams.t
    n = int(L * np.log2(M) / sparcparams.r)
    logm = int(np.log2(M))
    total_bits = int(logm * L)
    Pl = P / L * np.ones(L)
    code = _ldpc.code(ldpcparams.standard, ldpcparams.r_ldpc, ldpcparams.z, ldpcparams.ptype)
    nl, kl = code.N, code.K
    assert nl <= total_bits and nl % logm == 0
    if ldpcparams.standard in ("802.11n", "802.16"):
        prot = np.random.randint(0, 2, kl)
        ldpc_bits = code.encode(prot)
        unprot = np.random.randint(0, 2, int(total_bits - nl))
        bits = np.concatenate([unprot, ldpc_bits])
        seed = 0
    else:  # all-zero codeword, fresh random design (sparc_ldpc.py:916-922)
        bits = np.zeros(total_bits, dtype=np.int64)
        seed = None
    idx = (bits.reshape(L, logm) * (1 << np.arange(logm - 1, -1, -1))).sum(axis=1).astype(np.int32)
    op = _op(L, M, n, seed, precision)
    z = np.random.randn(n, 1) * sigma
    op.reserve(1, T)
    op.stage_power(1, Pl)
    op.encode(idx[None, :], z.reshape(1, -1))
    op.run(1, T)
    op.wait()
    rx = op.decide(1)[0]
    ber_amp = [float(_popcount(np.bitwise_xor(idx.astype(np.int64), rx.astype(np.int64))).sum()) / total_bits]
    ber_ldpc = []
    ns = nl // logm
    l0 = L - ns
    LLR = op.llr(1, 0, L)[0]
    for i in range(soft_iter):
        app, _ = code.decode(LLR[l0 * logm:])
        LLR[l0 * logm:] = app
        ber_ldpc.append(ber_from_LLRs(M, LLR, idx, total_bits))
        if i == soft_iter - 1:
            break
        dec = op.threshold(1, l0, ns, app, threshold)
        full = -np.ones((1, L), dtype=np.int32)
        full[0, l0:] = dec[0]
        amp_sections, llr = _amp_on_undecided(op, full, Pl, T, M)
        if llr is not None:
            pos = (np.arange(logm)[None, :] + logm * amp_sections[:, None]).reshape(-1)
            LLR[pos] = llr
        ber_amp.append(ber_from_LLRs(M, LLR, idx, total_bits))
    R = (L * logm - (nl - kl)) / n
    return ber_amp, ber_ldpc, R
