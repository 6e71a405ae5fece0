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
import sys
import math

import numpy as np

from . import ldpc as _ldpc
from .harness import SPARCParams, LDPCParams, pa_parameterised, _popcount
from .operators import AbOp, SparcOperator, make_ordering, sparc_transforms_shorter

__all__ = ["J", "J_inverse", "gen_bits", "hard_initialisation", "prep_y", "remove_common_zeros", "calc_E",
           "hist_E", "calc_I_e", "polynomial", "soft_amp_ldpc_hardinit", "ber_from_LLRs", "soft_hardinit_plot",
           "exit_draws", "calc_E_batch", "amp_exit_curve"]

_RLDPC = {"5/6": 5 / 6, "1/2": 1 / 2, "0.45": 0.45, "3/8": 3 / 8}  # sparc_ldpc.py:1458-1467


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


def soft_hardinit_plot(sparcparams: SPARCParams, ldpcparams: LDPCParams, csv_filename=None, png_filename=None,
                       sections=None, datapoints=10, MIN_ERRORS=100, MAX_BLOCKS=500, soft_iter=3, threshold=0.6,
                       batch=64, seed0=0, precision="fp64", rank=0, world=1, allreduce=None, sigmas=None,
                       unit_cancel=False):
    """The threshold-initialised exchange sweep of sparc_ldpc.py:1435-1590 on the GPU.

    Per sigma of linspace(0.9, 1.4, datapoints) (:1488): blocks of
    soft_amp_ldpc_hardinit at r_sparc and of plain SPARC at the same overall
    rate R = (L log2 M - nl (1 - R_ldpc)) / n (:1480-1481), until MIN_ERRORS
    PLAIN block errors or MAX_BLOCKS blocks (:1503-1524); BER columns are
    means over the blocks; Eb/N0 = 20 log10(p / (2 R sigma^2)) (:1533-1535).
    IEEE 802.11n / 802.16 codes share the seed-0 design, so blocks run
    ``batch`` at a time from seeded RandomStates (JointDecoder mode
    "threshold": per-codeword section masks), sharded over ranks like
    joint.waterfall; the designed protographs draw a fresh random design per
    block in the reference (:916-922), so those blocks run one at a time
    (soft_amp_ldpc_hardinit, global np.random).  Returns the rows
    (EbN0_dB, BER_amp [soft_iter], BER_ldpc [soft_iter], BER_plain, blocks,
    block_errors); rank 0 appends the reference's CSV (:1537-1542).
    unit_cancel=True cancels decided sections with amplitude 1 (the
    reference's behaviour before the fix noted at amp_exit.py:97-98, which its
    published threshold-init CSVs reflect; batched path only).
    No plots (figure code is out of scope)."""
    from .harness import mc_decode, amp_ldpc_sim
    from .joint import joint_decoder, mc_joint, _ber_point_multi
    L, M = sparcparams.L, sparcparams.M
    logm = int(np.log2(M))
    p, r_sparc, T = sparcparams.p, sparcparams.r, sparcparams.t
    if ldpcparams.r_ldpc not in _RLDPC:
        raise ValueError("Invalid choice of ldpc rate, please choose a different one.")
    Rldpc = _RLDPC[ldpcparams.r_ldpc]
    if sections is None:
        sections = L
    nl = logm * sections
    z = ldpcparams.z
    std = ldpcparams.standard in ("802.11n", "802.16")
    if z is None:
        z = int(nl / 24) if std else int(nl / 40)
    ldp = LDPCParams(ldpcparams.standard, ldpcparams.r_ldpc, z, ldpcparams.ptype)
    n_f = L * logm / r_sparc
    R = (L * logm - nl * (1 - Rldpc)) / n_f
    SIGMA = np.linspace(0.9, 1.4, datapoints) if sigmas is None else np.asarray(sigmas, dtype=np.float64)
    n = int(L * np.log2(M) / r_sparc)
    n_plain = int(L * np.log2(M) / R)
    total_bits = L * logm
    Pl = p / L * np.ones(L)
    rows = []
    if std:
        jd = joint_decoder(L, M, n, ldp, T, precision=precision)
        assert jd.ns == sections, "sections must match the LDPC code length"
        plain = SparcOperator(L, M, n_plain, make_ordering(L, M, n_plain, 0), None, precision)
    for pi, sigma in enumerate(SIGMA):
        sigma = float(sigma)
        if std:
            def round_fn(seeds, sigma=sigma):
                rj = mc_joint(jd, Pl, sigma, seeds, "threshold", soft_iter, batch, threshold, unit_cancel)
                be_plain, _ = mc_decode(plain, Pl, sigma, T, [s + 5_000_000 for s in seeds], batch=batch)
                return be_plain, np.concatenate([rj["amp"], rj["ldpc"]], axis=1)

            res = _ber_point_multi(round_fn, total_bits, MIN_ERRORS, MAX_BLOCKS, batch, rank, world, allreduce,
                                   seed0 + pi * 10_000_000)
            cols = np.asarray(res["cols"])
            ber_amp, ber_ldpc = cols[:soft_iter], cols[soft_iter:]
            ber_plain, nblocks, nerr = res["BER"], res["blocks"], res["block_errors"]
        else:
            sp_c = SPARCParams(L, M, sigma, p, r_sparc, T)
            sp_plain = SPARCParams(L, M, sigma, p, R, T)
            cum_amp, cum_ldpc, cum_plain = np.zeros(soft_iter), np.zeros(soft_iter), 0.0
            nerr = nblocks = 0
            while nerr < MIN_ERRORS:
                ba, bl, _ = soft_amp_ldpc_hardinit(sp_c, ldp, soft_iter, threshold, precision=precision)
                bpl = amp_ldpc_sim(sp_plain)[0]
                cum_amp += np.asarray(ba[:soft_iter])
                cum_ldpc += np.asarray(bl[:soft_iter])
                cum_plain += bpl
                nerr += 1 if bpl else 0
                nblocks += 1
                if nblocks >= MAX_BLOCKS:
                    break
            ber_amp, ber_ldpc, ber_plain = cum_amp / nblocks, cum_ldpc / nblocks, cum_plain / nblocks
        ebno_db = 20 * np.log10(1 / (2 * R) * (p / sigma ** 2))
        rows.append(dict(EbN0_dB=float(ebno_db), sigma=sigma, BER_amp=[float(x) for x in ber_amp],
                         BER_ldpc=[float(x) for x in ber_ldpc], BER_plain=float(ber_plain), blocks=int(nblocks),
                         block_errors=int(nerr)))
    if csv_filename and rank == 0:
        with open(csv_filename, "a", newline="") as fh:
            wr = csv.DictWriter(fh, fieldnames=["EbN0_dB", "BER_amp", "BER_ldpc", "BER_plain"])
            wr.writeheader()
            for r in rows:
                wr.writerow({"EbN0_dB": r["EbN0_dB"], "BER_amp": np.array(r["BER_amp"]),
                             "BER_ldpc": np.array(r["BER_ldpc"]), "BER_plain": r["BER_plain"]})
    return rows


# ---- batched EXIT measurement (amp_exit.py:185-270, 520-631) ------------------------

_MASKED = {}


def exit_draws(items, L, M, n, P, rng=np.random):
    """The np.random draws of a sequence of calc_E calls as amp_exit_curve makes
    them (amp_exit.py:581-589, 218-219, 153): per item (I_a, snr_dB) in order,
    X = gen_bits(L log2 M), N_a = randn(L log2 M) sigma_a, w = randn(n, 1) sigma_w.
    Returns X (B, L logm) +-1, A = mu_a X + N_a (B, L logm), w (B, n)."""
    logm = int(round(math.log2(M)))
    B = len(items)
    X = np.empty((B, L * logm), dtype=np.int64)
    A = np.empty((B, L * logm))
    w = np.empty((B, n))
    for b, (I_a, snr_dB) in enumerate(items):
        X[b] = (rng.randint(0, 2, L * logm) * -2) + 1                     # gen_bits, :48-50
        sigma_a = J_inverse(I_a)
        A[b] = (sigma_a ** 2) / 2 * X[b] + rng.randn(L * logm) * sigma_a  # :215-222
        sigma_w = np.sqrt(P / 10 ** (snr_dB / 20))                        # :205-206
        w[b] = rng.randn(n, 1).reshape(-1) * sigma_w                      # prep_y, :153
    return X, A, w


def calc_E_batch(X, A, w, sparcparams: SPARCParams, threshold=0.5, precision="fp64"):
    """calc_E (amp_exit.py:185-270) for B calls at once: every section whose
    a-priori bp2sp has exactly one entry above the threshold is decided and
    cancelled from y; AMP then runs over each codeword's own undecided
    sections (a per-codeword section mask, SparcOperator.stage_power_batch,
    instead of one shortened operator per call) and their LLRs replace A;
    clipped to +-55.  X, A: (B, L log2 M); w: (B, n).  Returns E (B, L log2 M)."""
    L, M, P, T = sparcparams.L, sparcparams.M, sparcparams.p, sparcparams.t
    logm = int(np.log2(M))
    n = int(L * np.log2(M) / sparcparams.r)
    X = np.asarray(X)
    A = np.ascontiguousarray(A, dtype=np.float64)
    B = X.shape[0]
    a, f, C = sparcparams.a, sparcparams.f, sparcparams.C
    Pl = P / L * np.ones(L) if a is None else pa_parameterised(L, C, P, a, f)
    Xb = ((X - 1) * -1 // 2).astype(np.int64).reshape(B, L, logm)
    idx = (Xb * (1 << np.arange(logm - 1, -1, -1))).sum(axis=2).astype(np.int32)
    op = _op(L, M, n, 0, precision)
    op.reserve(B, T)
    op.stage_power(B, Pl)
    op.encode(idx, np.ascontiguousarray(w, dtype=np.float64).reshape(B, n))
    dec = op.threshold(B, 0, L, A, threshold)  # every section is thresholded
    E = A.copy()
    und = dec < 0
    if und.any():
        key = (L, M, n, precision)
        mk = _MASKED.get(key)
        if mk is None:
            mk = _MASKED[key] = op.subset(np.arange(L))
        mk.reserve(B, T)
        mk.stage_power(B, Pl)  # c_l of the LLR kernel
        op.cancel(dec, mk)
        mk.stage_power_batch(B, np.where(und, Pl[None, :], 0.0))
        mk.run(B, T)
        mk.wait()
        llr = mk.llr(B, 0, L).reshape(B, L, logm)
        E.reshape(B, L, logm)[und] = llr[und]
    np.clip(E, -55, 55, out=E)
    return E


def amp_exit_curve(sparcparams: SPARCParams, low_snr_dB, high_snr_dB, repeats, x_axis_points, threshold,
                   poly_curve=0, bin_number=500, batch=256, precision="fp64", export_csv_filename=None):
    """amp_exit_curve (amp_exit.py:520-631) on the GPU: the AMP EXIT curves of
    threshold-initialised exchange at 4 SNRs (linspace(low, high, 4) dB,
    20 log10), I_a = linspace(0, 0.99, x_axis_points), averaged over
    `repeats`; histograms with bin_number bins over [-60, 60]; the cubic fit
    of curve `poly_curve`.  The calc_E calls draw from the global np.random
    stream in the reference's order (repeat, SNR, I_a) and are decoded
    `batch` at a time (calc_E_batch).  No plots and no CSV import (analysis
    and figure code are out of scope); export_csv_filename appends the
    reference's rows (I_a, snr_dB, X, E), arrays written in full.
    Returns (I_a_range, snr_dB, I_e (4, x_axis_points), poly_coeff)."""
    L, M, P = sparcparams.L, sparcparams.M, sparcparams.p
    n = int(L * np.log2(M) / sparcparams.r)
    curves = 4
    I_a_range = np.linspace(0, 0.99, x_axis_points)
    snr_dB = np.linspace(low_snr_dB, high_snr_dB, curves)
    items = [(k, j, i) for k in range(repeats) for j in range(curves) for i in range(x_axis_points)]
    I_e_accum = np.zeros((curves, x_axis_points))
    for s0 in range(0, len(items), batch):
        chunk = items[s0:s0 + batch]
        X, A, w = exit_draws([(I_a_range[i], snr_dB[j]) for (_, j, i) in chunk], L, M, n, P)
        E = calc_E_batch(X, A, w, sparcparams, threshold, precision)
        for b, (_, j, i) in enumerate(chunk):
            if export_csv_filename is not None:
                with open(export_csv_filename, "a") as fh:
                    wr = csv.DictWriter(fh, fieldnames=["I_a", "snr_dB", "X", "E"])
                    wr.writeheader()
                    full = dict(threshold=sys.maxsize, max_line_width=sys.maxsize)
                    wr.writerow({"I_a": I_a_range[i], "snr_dB": snr_dB[j], "X": np.array2string(X[b], **full),
                                 "E": np.array2string(E[b], **full)})
            PE_pos, PE_neg, _, _, _, _, bw = hist_E(X[b], E[b], bin_number=bin_number, max_bin=60, min_bin=-60)
            I_e_accum[j, i] += calc_I_e(PE_pos, PE_neg, bw)
    I_e_accum /= repeats
    return I_a_range, snr_dB, I_e_accum, polynomial(I_a_range, I_e_accum[poly_curve, :])
