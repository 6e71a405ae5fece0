"""Monte-Carlo harness around the AMP hot path.

Drop-ins for the reference's per-codeword simulator (plain-SPARC branch of
``amp_ldpc_sim``, ldpc/sparc_ldpc.py:359-545), its helpers
(``SPARCParams`` :227-246, ``bits2indices`` :317-341, ``pa_parameterised``
:172-186) and the BER sweep of ``waterfall``'s plain branch (:1126-1282), plus
a batched Monte-Carlo driver that keeps the codeword batch on the device and
shards reps across ranks.

The per-codeword functions consume ``np.random``'s global state in the same
order as the reference, so a seeded call reproduces the reference's message
and noise draws exactly.
"""
from __future__ import annotations

import math
import csv
import os

import numpy as np

from .amp import amp, amp_test
from .operators import SparcOperator, make_ordering, sparc_transforms, sparc_transforms_shorter

__all__ = [
    "SPARCParams", "LDPCParams", "pa_parameterised", "bits2indices", "ber_of",
    "amp_ldpc_sim", "mc_decode", "mc_decode_batched", "mc_stream", "draw_reps", "ebno_to_sigma", "ber_point", "waterfall_plain", "amp_test_reps", "amp_init_test",
]


class SPARCParams:
    """sparc_ldpc.py:227-246 (same fields)."""

    def __init__(self, L, M, sigma, p, r, t, a=None, f=None, C=None):
        self.L = L
        self.M = M
        self.sigma = sigma
        self.p = p
        self.r = r
        self.t = t
        self.a = a
        self.f = f
        self.C = C


class LDPCParams:
    """sparc_ldpc.py:250-255 (same fields); consumed by sparc_ldpc_amd.joint."""

    def __init__(self, standard, r_ldpc, z, ptype='A'):
        self.standard = standard
        self.r_ldpc = r_ldpc
        self.z = z
        self.ptype = ptype


def pa_parameterised(L, C, P, a, f):
    """sparc_ldpc.py:172-186: exponential power allocation flattened after fL."""
    pa = 2 ** (-2 * a * C * np.arange(L) / L)
    pa[int(f * L):] = pa[int(f * L)]
    pa /= pa.sum() / P
    return pa


def bits2indices(bits, m):
    """sparc_ldpc.py:317-341: MSB-first, log2(m) bits per section."""
    logm = int(math.log(m, 2))
    assert len(bits) % logm == 0
    b = np.asarray(bits, dtype=np.int64).reshape(-1, logm)
    w = 1 << np.arange(logm - 1, -1, -1, dtype=np.int64)
    return (b * w).sum(axis=1).tolist()


_POP8 = np.array([bin(i).count("1") for i in range(256)], dtype=np.int64)


def _popcount(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    c = np.zeros(x.shape, dtype=np.int64)
    while np.any(x):
        c += _POP8[(x & np.uint64(0xFF)).astype(np.int64)]
        x >>= np.uint64(8)
    return c


def ber_of(sent, decided, total_bits):
    """sparc_ldpc.py:462: Σ popcount(sent ^ decided) / total_bits (per row)."""
    s = np.asarray(sent, dtype=np.int64)
    d = np.asarray(decided, dtype=np.int64)
    return _popcount(np.bitwise_xor(s, d)).sum(axis=-1) / total_bits


def amp_ldpc_sim(sparcparams: SPARCParams, ldpcparams=None, a=None, f=None, C=None, *,
                 backend=None, precision=None):
    """sparc_ldpc.py:359-545: one Monte-Carlo rep.  With an LDPC code this is
    the original hard exchange (``joint.amp_ldpc_sim_ldpc``); without one,
    plain SPARC returning (ber_amp, None, None, R) like the reference.
    Draw order of np.random: randint(0, 2, total_bits) (:423-424), then
    randn(n, 1) (:445).
    """
    if ldpcparams is not None:
        from .joint import amp_ldpc_sim_ldpc
        return amp_ldpc_sim_ldpc(sparcparams, ldpcparams, backend=backend, precision=precision)
    L, M, P = sparcparams.L, sparcparams.M, sparcparams.p
    sigma, r_sparc, T = sparcparams.sigma, sparcparams.r, sparcparams.t
    a, f, C = sparcparams.a, sparcparams.f, sparcparams.C
    n = int(L * np.log2(M) / r_sparc)
    logm = np.log2(M)
    total_bits = int(logm * L)
    Pl = P / L * np.ones(L) if a is None else pa_parameterised(L, C, P, a, f)
    bits = np.random.randint(0, 2, int(total_bits)).tolist()
    idx = bits2indices(bits, M)
    Ab, Az, ordering = sparc_transforms(L, M, n, backend=backend, precision=precision)
    β0 = np.zeros((L * M, 1))
    β0[np.arange(L) * M + np.asarray(idx), 0] = np.sqrt(n * Pl)
    x = Ab(β0)
    z = np.random.randn(n, 1) * sigma
    y = (x + z).reshape(-1, 1)
    β = amp(y, sigma, Pl, L, M, T, Ab, Az).reshape(-1)
    rx = β.reshape(L, M).argmax(axis=1)
    ber_amp = float(ber_of(idx, rx, total_bits))
    R = (L * logm) / n
    return ber_amp, None, None, R


def _draw_reps(seeds, L, M, n, sigma):
    """Rep with seed s: ``RandomState(s)`` draws the L section indices uniform
    in [0, M) (the law of random bits -> bits2indices) and then the noise
    N(0, σ²) (n values) — SURVEY §8d's synthetic inputs.  (NumPy; draw_reps
    is the same on the host cores natively.)"""
    idx = np.empty((len(seeds), L), dtype=np.int32)
    noise = np.empty((len(seeds), n))
    for i, s in enumerate(seeds):
        rs = np.random.RandomState(s)
        idx[i] = rs.randint(0, M, L)
        noise[i] = rs.randn(n)
    noise *= sigma
    return idx, noise


def draw_threads() -> int:
    """Host threads for draw_reps: the job's CPU share (OMP_NUM_THREADS, 16 on
    the GPU box), at most the machine's."""
    want = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(want, os.cpu_count() or 1))


def draw_reps(seeds, L, M, n, sigma, idx=None, noise=None, threads=None):
    """_draw_reps' reps (RandomState(s).randint(0, M, L), then .randn(n) * σ),
    bit for bit, drawn by libsparc_amp's native restatement of NumPy's legacy
    generator over several host threads (sa_draw_reps).  idx / noise: optional
    (R, L) int32 / (R, n) fp64 arrays (or views) to fill."""
    from . import _lib
    lib = _lib.load()
    seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
    R = len(seeds)
    idx = np.empty((R, L), dtype=np.int32) if idx is None else idx
    noise = np.empty((R, n)) if noise is None else noise
    assert idx.shape == (R, L) and idx.dtype == np.int32 and idx.flags.c_contiguous
    assert noise.shape == (R, n) and noise.dtype == np.float64 and noise.flags.c_contiguous
    ct = _lib.ct
    _lib.check(lib.sa_draw_reps(seeds.ctypes.data_as(ct.POINTER(ct.c_uint32)), R, int(L), int(M), int(n),
                                float(sigma), idx.ctypes.data_as(ct.POINTER(ct.c_int32)),
                                noise.ctypes.data_as(ct.POINTER(ct.c_double)),
                                draw_threads() if threads is None else int(threads)))
    return idx, noise


def mc_stream(op: SparcOperator, Pl, T, idx, noise, batch=256, early_stop=True, timings=None):
    """Decode staged reps (idx (R, L), noise (R, n)) as one stream through
    ``batch`` slots with per-slot refill (SparcOperator.mc_run): a slot whose
    exact-τ stop fires takes the next rep at once.  Returns per-rep int64
    (bit_errors, iters) and the stream's device milliseconds; ``timings``
    (a dict) receives the host wall seconds of its phases."""
    import time
    t0 = time.perf_counter()
    op.reserve(batch, T)
    op.stage_power(batch, np.asarray(Pl, dtype=np.float64))
    t1 = time.perf_counter()
    op.mc_stage(idx, noise)
    t2 = time.perf_counter()
    _, its, errs, ms = op.mc_run(batch, T, early_stop=early_stop, decisions=False)
    if timings is not None:
        timings.update(setup_s=t1 - t0, stage_s=t2 - t1, run_s=time.perf_counter() - t2)
    return errs.astype(np.int64), its.astype(np.int64), ms


def mc_decode(op: SparcOperator, Pl, sigma, T, seeds, batch=256, early_stop=True, stream=None):
    """Monte-Carlo reps on one device (the rep body of sparc_ldpc.py:423-462
    on SURVEY §8d's synthetic inputs, ``_draw_reps``).  Returns per-rep int64
    arrays (bit_errors, iters) in seed order.

    stream (default: wherever the operator supports it, mc_supported): the
    reps drawn natively on the host cores (draw_reps) and decoded as one
    stream through ``batch`` refilled slots (mc_stream); else batch by batch
    (mc_decode_batched).  The per-rep results are the same either way
    (tests/test_gpu_mc_stream.py)."""
    seeds = list(seeds)
    if stream is None:
        stream = op.mc_supported(batch)
    if not stream or not seeds:
        return mc_decode_batched(op, Pl, sigma, T, seeds, batch, early_stop)
    idx, noise = draw_reps(seeds, op.L, op.M, op.n, sigma)
    be, it, _ = mc_stream(op, Pl, T, idx, noise, batch, early_stop)
    return be, it


def mc_decode_batched(op: SparcOperator, Pl, sigma, T, seeds, batch=256, early_stop=True):
    """mc_decode batch by batch: encoding x = A β₀ + noise (sa_encode), the
    decode and the section decisions on the device, every batch run until its
    slowest codeword stops; the host draws the next batch while the device
    decodes the current one."""
    L, M, n = op.L, op.M, op.n
    Pl = np.asarray(Pl, dtype=np.float64)
    seeds = list(seeds)
    bit_errors = np.zeros(len(seeds), dtype=np.int64)
    iters = np.zeros(len(seeds), dtype=np.int64)
    if not seeds:
        return bit_errors, iters
    chunks = [seeds[i:i + batch] for i in range(0, len(seeds), batch)]
    op.reserve(len(chunks[0]), T)
    op.stage_power(len(chunks[0]), Pl)
    nxt = _draw_reps(chunks[0], L, M, n, sigma)
    s0 = 0
    for k, chunk in enumerate(chunks):
        idx, noise = nxt
        B = len(chunk)
        op.encode(idx, noise)
        op.run(B, T, early_stop=early_stop)
        # host draws of the next batch overlap the device decode
        nxt = _draw_reps(chunks[k + 1], L, M, n, sigma) if k + 1 < len(chunks) else None
        rx = op.decide(B).astype(np.int64)
        bit_errors[s0:s0 + B] = _popcount(np.bitwise_xor(idx.astype(np.int64), rx)).sum(axis=1)
        iters[s0:s0 + B] = op.iters(B)
        s0 += B
    return bit_errors, iters


def ebno_to_sigma(ebno_db, P, R):
    """waterfall's mapping (sparc_ldpc.py:1184,1199-1200), 20*log10 convention."""
    ebno = 10 ** (ebno_db / 20)
    snr = ebno / (1 / (2 * R))
    return float(np.sqrt(P / snr))


def ber_point(decode_round, total_bits, min_errors, max_blocks, batch, rank=0, world=1,
              allreduce=None, seed_base=0):
    """One Eb/N0 point with the reference's stopping rule (sparc_ldpc.py:1217-1245):

        while nblockerrors < MIN_ERRORS:
            decode one block; ber_cum += ber; nblockerrors += (ber > 0); nblocks += 1
            if nblocks >= MAX_BLOCKS: break
        BER = ber_cum / nblocks

    Blocks are decoded in rounds of batch*world (rank r takes the seeds of
    ``dist.shard_seeds``); each round's per-block bit errors are summed over
    ranks into global seed order (an all-gather by sum, batch*world int64)
    and consumed block by block, so the result equals a sequential run over
    the same seeds whatever the world size.  ``decode_round(seeds)`` returns
    the per-block (bit_errors, iters) of this rank's seeds.
    """
    from .dist import shard_seeds
    ber_cum = 0.0
    nerr = nblocks = iters = errbits = 0
    rnd = 0
    while nerr < min_errors:
        seeds = shard_seeds(seed_base, rnd, batch, rank, world)
        be, it = decode_round(seeds)
        glob = np.zeros((2, batch * world), dtype=np.int64)
        glob[0, rank::world] = be   # global position of seed base + rnd*B*W + j is j
        glob[1, rank::world] = it
        if allreduce is not None:
            glob = allreduce(glob)
        done = False
        for j in range(batch * world):
            if nerr >= min_errors:
                done = True
                break
            b = int(glob[0, j])
            ber_cum += b / total_bits
            errbits += b
            iters += int(glob[1, j])
            nerr += 1 if b > 0 else 0
            nblocks += 1
            if nblocks >= max_blocks:
                done = True
                break
        if done:
            break
        rnd += 1
    return dict(BER=ber_cum / nblocks, blocks=nblocks, block_errors=nerr, bit_errors=errbits,
                mean_iters=iters / nblocks)


def waterfall_plain(L, M, P, R, T, ebno_dbs, min_errors=200, max_blocks=250, csv_filename=None,
                    batch=64, seed0=0, backend=None, precision=None, rank=0, world=1, allreduce=None):
    """BER_plain column of waterfall() (sparc_ldpc.py:1126-1282) on the GPU:
    plain SPARC at rate R, 20*log10 Eb/N0 -> sigma mapping, the reference's
    MIN_ERRORS / MAX_BLOCKS rule (``ber_point``), reps sharded over ranks.
    Writes the reference CSV schema (:1257-1264) when csv_filename is given
    (only the BER_plain column is produced; the LDPC columns are 0).
    """
    n = int(L * np.log2(M) / R)
    ordering = make_ordering(L, M, n, 0)
    op = SparcOperator(L, M, n, ordering, backend, precision)
    Pl = P / L * np.ones(L)
    total_bits = int(L * np.log2(M))
    rows = []
    for pi, ebno_db in enumerate(ebno_dbs):
        sigma = ebno_to_sigma(ebno_db, P, R)

        def round_fn(seeds, sigma=sigma):
            return mc_decode(op, Pl, sigma, T, seeds, batch=batch)

        r = ber_point(round_fn, total_bits, min_errors, max_blocks, batch, rank, world, allreduce,
                      seed_base=seed0 + pi * 10_000_000)
        rows.append(dict(EbN0_dB=float(ebno_db), BER_amp_1=0.0, BER_ldpc=0.0, BER_amp_2=0.0,
                         BER_ldpc_2=0.0, BER_plain=r["BER"], BER_bpsk=0.0, blocks=r["blocks"],
                         block_errors=r["block_errors"], mean_iters=r["mean_iters"]))
    if csv_filename and rank == 0:
        fields = ['EbN0_dB', 'BER_amp_1', 'BER_ldpc', 'BER_amp_2', 'BER_ldpc_2', 'BER_plain', 'BER_bpsk']
        with open(csv_filename, 'a', newline='') as fh:
            wr = csv.DictWriter(fh, fieldnames=fields)
            wr.writeheader()
            for row in rows:
                wr.writerow({k: row[k] for k in fields})
    return rows


def amp_test_reps(L=512, M=512, L_zero=154, P=4, snr_dB=10, r_sparc=1, T=64, repeats=100,
                  backend=None, precision=None, batch=64, rank=0, world=1, allreduce=None, return_counts=False):
    """The reps loop of amp_test.py:161-253, batched on the device and sharded
    over ranks.  Per rep the reference draws the message bits and the noise
    (:185-199), then decodes three times and adds each decode's BER:

      * hard init (:201-221): the sections from L_zero on are taken as decoded
        with the 0/1 start beta_0 = beta / sqrt(n P / L) (its first L_zero
        sections zeroed); y' = y - Ab(beta_0) is decoded by AMP on the
        shortened operator over the first L_zero sections
        (sparc_transforms_shorter), BER over those sections;
      * soft init (:223-232): AMP over all L sections from beta_0;
      * no init (:234-241): AMP from zero.

    Every rank draws every rep from np.random in the reference's order (so a
    seeded call reproduces the reference's reps, whatever the world size) and
    decodes the reps i with i % world == rank, ``batch`` at a time: encode,
    cancellation, the three decodes and the decisions all on the device,
    sharing one full and one shortened operator.  The per-rep bit-error counts
    are summed over ranks (``allreduce``, dist.allreduce_sum) and the BERs
    accumulated in rep order as the reference does (ber += errors / total_bits).
    Returns (ber_hard, ber_soft, ber_no_init), plus the (repeats, 3) int64
    error counts with ``return_counts``.
    """
    snr = 10 ** (snr_dB / 20)
    sigma = np.sqrt(P / snr)
    Pl = P / L * np.ones(L)
    logm = np.log2(M)
    total_bits = int(L * logm)
    n = int(L * np.log2(M) / r_sparc)
    mine = [i for i in range(repeats) if i % world == rank]
    idx = np.empty((len(mine), L), dtype=np.int32)
    noise = np.empty((len(mine), n))
    w = 1 << np.arange(int(logm) - 1, -1, -1, dtype=np.int64)
    k = 0
    for i in range(repeats):
        bits = np.random.randint(0, 2, total_bits)          # :185
        z = np.random.randn(n, 1) * sigma                   # :198
        if i % world == rank:
            idx[k] = (bits.reshape(L, -1).astype(np.int64) * w).sum(axis=1)  # bits2indices, :187
            noise[k] = z.reshape(-1)
            k += 1
    ordering = make_ordering(L, M, n, 0)
    op = SparcOperator(L, M, n, ordering, backend, precision)
    op_h = SparcOperator(L_zero, M, n, ordering[:L_zero], backend, precision)
    scale = 1.0 / np.sqrt(n * P / L)                         # beta_0 = beta / sqrt(n P / L), :202
    counts = np.zeros((repeats, 3), dtype=np.int64)
    for s0 in range(0, len(mine), batch):
        ib = idx[s0:s0 + batch]
        B = ib.shape[0]
        op.reserve(B, T)
        op_h.reserve(B, T)
        op.stage_power(B, Pl)
        op_h.stage_power(B, Pl[:L_zero])
        op.encode(ib, noise[s0:s0 + B])                      # y = Ab(beta) + z, :193-199
        ib0 = ib.copy()
        ib0[:, :L_zero] = -1                                 # beta_0[:L_zero*M] = 0, :204
        op.cancel(ib0, op_h, scale)                          # y_new = y - Ab(beta_0), :208-210
        op_h.run(B, T)
        rx_h = op_h.decide(B).astype(np.int64)
        op.stage_onehot(ib0, scale)
        op.run(B, T, beta0=True)                             # soft init, :225
        rx_s = op.decide(B).astype(np.int64)
        op.run(B, T)                                         # no init, :235
        rx_z = op.decide(B).astype(np.int64)
        reps = mine[s0:s0 + B]
        ib64 = ib.astype(np.int64)
        counts[reps, 0] = _popcount(np.bitwise_xor(ib64[:, :L_zero], rx_h)).sum(axis=1)
        counts[reps, 1] = _popcount(np.bitwise_xor(ib64, rx_s)).sum(axis=1)
        counts[reps, 2] = _popcount(np.bitwise_xor(ib64, rx_z)).sum(axis=1)
    if world > 1:
        if allreduce is None:
            raise ValueError("amp_test_reps: world > 1 needs allreduce (dist.allreduce_sum)")
        counts = allreduce(counts)
    ber = [0.0, 0.0, 0.0]
    for i in range(repeats):                                 # the reference's float accumulation
        for j in range(3):
            ber[j] = ber[j] + int(counts[i, j]) / total_bits
    out = (ber[0] / repeats, ber[1] / repeats, ber[2] / repeats)
    return (out, counts) if return_counts else out


def amp_init_test(L, M, snr_dB, P, r_sparc, backend=None, precision=None):
    """amp_test.py:53-110: one rep decoded twice, from the transmitted beta
    itself and from zero (amp_test with T = 64); returns ([ber_init],
    [ber_no_init]) and prints the iteration counts like the reference.
    Draws: np.random randint(0, 2, L log2 M) then randn(n, 1) sigma."""
    logm = np.log2(M)
    total_bits = int(L * logm)
    sigma = np.sqrt(P / 10 ** (snr_dB / 20))
    n = int(L * np.log2(M) / r_sparc)
    Pl = P / L * np.ones(L)
    idx = np.asarray(bits2indices(np.random.randint(0, 2, total_bits).tolist(), M))
    Ab, Az, _ = sparc_transforms(L, M, n, backend=backend, precision=precision)
    beta = np.zeros((L * M, 1))
    beta[np.arange(L) * M + idx, 0] = np.sqrt(n * Pl)
    y = (Ab(beta) + np.random.randn(n, 1) * sigma).reshape(-1, 1)
    beta_init, t_init = amp_test(y, 0, Pl, L, M, 64, Ab, Az, beta)
    beta_no_init, t_no_init = amp_test(y, 0, Pl, L, M, 64, Ab, Az)
    ber_init = [float(ber_of(idx, beta_init.reshape(L, M).argmax(1), total_bits))]
    ber_no_init = [float(ber_of(idx, beta_no_init.reshape(L, M).argmax(1), total_bits))]
    print("For initialised amp, BER= ", ber_init, " and iterations= ", t_init)
    print("For amp with all zero beta_0, BER= ", ber_no_init, " and iterations= ", t_no_init)
    return ber_init, ber_no_init
