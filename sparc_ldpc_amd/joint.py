"""Joint SPARC + LDPC decoding on the GPU (BASELINE
configs[4]: L=M=512 with the 802.16 rate-5/6 outer code, AMP <-> BP rounds).

The three information-exchange schemes of the reference, per codeword and
batched:

* ``originalHard`` — ``amp_ldpc_sim`` with an LDPC code (sparc_ldpc.py:359-545):
  AMP, BP on the LDPC sections, cancel their hard decisions from y, AMP again
  on the remaining sections (a ``sparc_transforms_shorter`` operator).
* ``soft`` — ``soft_amp_ldpc_sim`` (:547-712): AMP, then ``soft_iter`` rounds of
  BP -> bp2sp -> AMP re-initialised with the soft LDPC output.
* ``hard`` — ``hardinitbeta_amp_ldpc_sim`` (:715-860): AMP, BP, AMP
  re-initialised with the one-hot hard decisions.
* ``threshold`` — ``soft_amp_ldpc_hardinit`` (:862-1047): AMP, then rounds of
  BP -> threshold decisions (amp_exit.hard_initialisation) -> cancel the
  decided sections from y -> AMP over the undecided ones.  Batched, each
  codeword has its own undecided set: the shortened operator of the reference
  becomes a per-codeword section mask (sections with Pl = 0,
  ``SparcOperator.stage_power_batch``) on one full-size operator.

Every step of a round runs on the device: encoding (``sa_encode``), AMP
(``sa_run``), the section->bit LLRs (``sa_llr``), belief propagation
(``libldpc_bp``), and the soft / hard hand-back (``sa_soft_beta0``,
``sa_hard_cancel``, ``sa_stage_onehot``); LLRs and a-posteriori values move
between the two libraries as device pointers.  The host draws the message
bits and the noise and LDPC-encodes the protected bits (numpy), exactly in
the reference's draw order, and counts bit errors.
"""
from __future__ import annotations

import csv
import math
from collections import OrderedDict

import numpy as np

from . import ldpc as _ldpc
from .harness import SPARCParams, LDPCParams, pa_parameterised, ebno_to_sigma
from .operators import SparcOperator, make_ordering

__all__ = ["JointDecoder", "JointPipeline", "joint_decoder", "draw_reps", "amp_ldpc_sim_ldpc", "soft_amp_ldpc_sim",
           "hardinitbeta_amp_ldpc_sim", "sim_ldpc", "waterfall", "soft_hard_plot", "sp2bp", "bp2sp", "mc_joint"]

MODES = ("originalHard", "soft", "hard", "threshold")


def sp2bp(beta, L, M):
    """sparc_ldpc.py:257-281 on the host (helper for scripts; the joint
    decoder uses the device kernel behind ``sa_llr``).  p[b] = P(bit b = 1),
    section bits MSB first; the sums run over ascending entry index."""
    logm = int(np.log2(M))
    beta = np.asarray(beta, dtype=np.float64).reshape(L, M)
    j = np.arange(M)
    p = np.zeros((L, logm))
    for t in range(logm):
        sel = (j >> (logm - 1 - t)) & 1 == 1
        acc = np.zeros(L)
        for jj in np.nonzero(sel)[0]:  # sequential, the reference's order
            acc = acc + beta[:, jj]
        p[:, t] = acc
    return p.reshape(-1)


def bp2sp(v, L, M):
    """sparc_ldpc.py:283-314 on the host: product of bit marginals, normalised."""
    logm = int(np.log2(M))
    v = np.asarray(v, dtype=np.float64).reshape(L, logm)
    bits = (np.arange(M)[:, None] >> np.arange(logm - 1, -1, -1)[None, :]) & 1  # (M, logm) MSB first
    sp = np.ones((L, M))
    for t in range(logm):
        sp = sp * np.where(bits[None, :, t] == 1, v[:, None, t], 1 - v[:, None, t])
    S = np.zeros(L)
    for m in range(M):
        S = S + sp[:, m]
    return (sp / S[:, None]).reshape(-1)


def draw_reps(code, L, M, n, rs, B, sigma):
    """Message and noise of B reps in the reference's draw order: randint(0,2,K)
    protected bits, LDPC encode, randint(0,2,total-N) unprotected bits,
    randn(n,1)*sigma (sparc_ldpc.py:419-446 / :606-634); message = unprotected
    bits then codeword, MSB-first log2(M) bits per section.  ``rs``: a list of
    B RandomStates, or one generator (np.random for the global stream) when B = 1.
    Returns (section indices (B, L) int32, noise (B, n))."""
    reps = rs if isinstance(rs, (list, tuple)) else [rs]
    assert len(reps) == B
    logm = int(round(math.log2(M)))
    total = L * logm
    K, N = code.K, code.N
    prot = np.empty((B, K), dtype=np.int64)
    unprot = np.empty((B, total - N), dtype=np.int64)
    noise = np.empty((B, n))
    for i, r in enumerate(reps):
        prot[i] = r.randint(0, 2, K)
        unprot[i] = r.randint(0, 2, total - N)  # encoding draws nothing in between
        noise[i] = r.randn(n, 1).reshape(-1) * sigma
    bits = np.concatenate([unprot, code.encode_batch(prot)], axis=1).reshape(B, L, logm)
    w = 1 << np.arange(logm - 1, -1, -1)
    return (bits * w).sum(axis=2).astype(np.int32), noise


class JointDecoder:
    """AMP operator + LDPC code + the shortened operator of the unprotected
    sections, for B-codeword batches of the joint schemes."""

    def __init__(self, L, M, n, code, T, backend=None, precision=None, device=None, seed=0, twin_of=None,
                 ordering=None):
        """twin_of: another JointDecoder whose operator tables this one shares
        (SparcOperator.twin: own stream and workspace, one copy of the tables).
        ordering: the design's (L, n) ordering (default: make_ordering(..., seed))."""
        self.L, self.M, self.n, self.T = int(L), int(M), int(n), int(T)
        self.logm = int(round(math.log2(M)))
        self.code = code
        nl = code.N
        assert nl <= L * self.logm, "LDPC code longer than the SPARC message"
        assert nl % self.logm == 0, "LDPC code must cover whole sections"
        self.ns = nl // self.logm
        self.l0 = self.L - self.ns
        if twin_of is not None and twin_of.op.backend == "hadamard":
            self.op = twin_of.op.twin()
            self.sub = twin_of.sub.twin() if twin_of.sub is not None else None
        else:
            if ordering is None:
                ordering = twin_of.op.ordering if twin_of is not None else make_ordering(L, M, n, seed)
            self.op = SparcOperator(L, M, n, ordering, backend, precision, device)
            self.sub = self.op.subset(np.arange(self.l0)) if self.l0 > 0 else None
        self._pipeline = None  # joint_pipeline's cached JointPipeline over this decoder
        self.total_bits = self.L * self.logm
        self.R = (self.L * self.logm - (code.N - code.K)) / n  # sparc_ldpc.py:541
        self._masked = None  # full-size operator for the per-codeword masked decodes (threshold mode)
        self._after_first_amp = None  # JointPipeline's stagger signal

    # -- message / channel draws (the reference's order) --------------------------
    def draw(self, rs, B, sigma):
        return draw_reps(self.code, self.L, self.M, self.n, rs, B, sigma)

    # -- one batch ------------------------------------------------------------------
    def _bp(self, B, dectype="sumprod2"):
        d_ch, d_app, _ = self.code.device_buffers(B)
        self.op.llr(B, self.l0, self.ns, out=d_ch)
        self.code.run_buffers(B, dectype)
        return d_app

    def run(self, idx, noise, Pl, mode="soft", soft_iter=2, threshold=0.5, unit_cancel=False):
        """Decode B codewords (section indices idx (B, L), noise (B, n)).

        Returns dict of per-rep bit-error COUNTS: 'amp' (B, rounds), 'ldpc'
        (B, rounds), 'ldpc_amp' (B,) for originalHard, and 'bp_iters'."""
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        self.stage(idx, noise, Pl)
        return self.decode_staged(idx, Pl, mode, soft_iter, threshold, unit_cancel)

    def stage(self, idx, noise, Pl):
        """Encode on the device: y = A beta(idx) + noise becomes the staged input."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        B = idx.shape[0]
        self.op.reserve(B, self.T)
        if self.sub is not None:
            self.sub.reserve(B, self.T)
        self.op.stage_power(B, np.asarray(Pl, dtype=np.float64))
        self.op.encode(idx, noise)
        self.code.device_buffers(B)
        self._noise = np.asarray(noise, dtype=np.float64).reshape(B, self.n)

    def decode_staged(self, idx, Pl, mode="soft", soft_iter=2, threshold=0.5, unit_cancel=False):
        """The joint decode of the staged batch (see run); idx only scores the
        decisions.  unit_cancel (threshold mode only): cancel decided sections
        with amplitude 1 instead of sqrt(n Pl_l), the reference's behaviour
        before the fix its comment at amp_exit.py:97-98 records, with which its
        published threshold-init CSVs were evidently produced (see
        DESIGN.md §10)."""
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}")
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        B = idx.shape[0]
        Pl = np.asarray(Pl, dtype=np.float64)
        op, T, l0 = self.op, self.T, self.l0
        op.run(B, T)
        op.wait()
        if self._after_first_amp is not None:
            self._after_first_amp()
        rx = op.decide(B)
        errs_amp = [self._errs(idx, rx)]
        errs_ldpc = []
        bp_iters = []
        out = {}
        if mode == "originalHard":
            d_app = self._bp(B)
            bp_iters.append(self.code.fetch_buffers(B, app=False)[1])
            idx_l = op.hard_cancel(B, l0, self.ns, d_app, dst=self.sub if l0 > 0 else None)
            dec = rx.copy()
            dec[:, l0:] = idx_l
            errs_ldpc.append(self._errs(idx, dec))
            if l0 > 0:
                self.sub.stage_power(B, Pl[:l0])
                self.sub.run(B, T)
                self.sub.wait()
                dec[:, :l0] = self.sub.decide(B)
                out["ldpc_amp"] = self._errs(idx, dec)
        elif mode == "soft":
            for _ in range(soft_iter):
                d_app = self._bp(B)
                bp_iters.append(self.code.fetch_buffers(B, app=False)[1])
                idx_l = op.hard_cancel(B, l0, self.ns, d_app)
                dec = rx.copy()
                dec[:, l0:] = idx_l
                errs_ldpc.append(self._errs(idx, dec))
                op.soft_beta0(B, l0, self.ns, d_app)
                op.run(B, T, beta0=True)
                op.wait()
                rx = op.decide(B)
                errs_amp.append(self._errs(idx, rx))
        elif mode == "threshold":
            self._threshold_rounds(B, idx, Pl, soft_iter, threshold, errs_amp, errs_ldpc, bp_iters, unit_cancel)
        else:  # hard
            d_app = self._bp(B)
            bp_iters.append(self.code.fetch_buffers(B, app=False)[1])
            idx_l = op.hard_cancel(B, l0, self.ns, d_app)
            dec = rx.copy()
            dec[:, l0:] = idx_l
            errs_ldpc.append(self._errs(idx, dec))
            op.stage_onehot(dec)
            op.run(B, T, beta0=True)
            op.wait()
            errs_amp.append(self._errs(idx, op.decide(B)))
        out["amp"] = np.stack(errs_amp, axis=1)
        out["ldpc"] = np.stack(errs_ldpc, axis=1) if errs_ldpc else np.zeros((B, 0), dtype=np.int64)
        out["bp_iters"] = np.stack(bp_iters, axis=1) if bp_iters else np.zeros((B, 0), dtype=np.int64)
        return out

    def _threshold_rounds(self, B, idx, Pl, soft_iter, threshold, errs_amp, errs_ldpc, bp_iters, unit_cancel=False):
        """The information-exchange rounds of soft_amp_ldpc_hardinit
        (sparc_ldpc.py:960-1041) for the batch; the first AMP has run on self.op."""
        op, T, L, logm, l0, ns = self.op, self.T, self.L, self.logm, self.l0, self.ns
        LLR = op.llr(B, 0, L)  # :960-970, every section
        if self._masked is None:
            self._masked = op.subset(np.arange(L))
        mk = self._masked
        mk.reserve(B, T)
        mk.stage_power(B, Pl)  # c_l of the LLR kernel
        for i in range(soft_iter):
            app, it = self.code.decode_batch(LLR[:, l0 * logm:])  # :973
            bp_iters.append(it)
            LLR[:, l0 * logm:] = app
            errs_ldpc.append(self._llr_errs(idx, LLR))  # :977
            if i == soft_iter - 1:
                break
            dec = op.threshold(B, l0, ns, app, threshold)  # :984-999 + amp_exit.py:56-105
            full = np.full((B, L), -1, dtype=np.int32)
            full[:, l0:] = dec
            undecided = full < 0
            if undecided.any():  # :1006-1032, each codeword over its own undecided sections
                if unit_cancel:
                    self._stage_unit_cancel(B, idx, full, Pl, mk)
                else:
                    op.cancel(full, mk)  # y - A beta(decided)
                mk.stage_power_batch(B, np.where(undecided, np.asarray(Pl, np.float64)[None, :], 0.0))
                mk.run(B, T)
                mk.wait()
                llr = mk.llr(B, 0, L).reshape(B, L, logm)
                LLR.reshape(B, L, logm)[undecided] = llr[undecided]
            errs_amp.append(self._llr_errs(idx, LLR))  # :1038

    def _stage_unit_cancel(self, B, idx, full, Pl, mk):
        """Stage y - A beta_1(decided) into mk, beta_1 one-hot with amplitude 1."""
        L, M = self.L, self.M
        c = np.sqrt(self.n * np.asarray(Pl, dtype=np.float64))
        rows = np.arange(B)[:, None]
        b0 = np.zeros((B, L * M))
        b0[rows, np.arange(L)[None, :] * M + idx] = c[None, :]
        y = self.op.Ab_batch(b0) + self._noise[:B]
        b1 = np.zeros((B, L * M))
        r, l = np.nonzero(full >= 0)
        b1[r, l * M + full[r, l]] = 1.0
        mk.stage(y - self.op.Ab_batch(b1), Pl)

    def _llr_errs(self, idx, LLR):
        """Bit errors of the hard decisions of LLR against the section indices
        (ber_from_LLRs, sparc_ldpc.py:343-356, times the bit count)."""
        B = idx.shape[0]
        bits = (np.asarray(LLR) < 0.0).astype(np.int64).reshape(B, self.L, self.logm)
        hat = (bits * (1 << np.arange(self.logm - 1, -1, -1))).sum(axis=2)
        return self._errs(idx, hat)

    def _errs(self, a, b):
        from .harness import _popcount
        return _popcount(np.bitwise_xor(np.asarray(a, np.int64), np.asarray(b, np.int64))).sum(axis=1)


class JointPipeline:
    """A batch of the joint decoder cut into `parts` consecutive slices, each
    decoded by its own JointDecoder (its own operator context, sharing the first slice's
    device tables (SparcOperator.twin), and HIP stream,
    its own LDPC context and stream) from its own host thread, so that one
    slice's belief-propagation tail (a few words on a few CUs for up to
    MAX_ITCOUNT iterations, c_ldpc.c:7) runs beside another slice's AMP
    kernels instead of in front of them.  The library calls release the GIL;
    every slice's steps stay in the reference's order on its own streams, and
    a codeword's decode does not depend on the batch it is in, so the per-rep
    results are those of one JointDecoder over the whole batch
    (tests/test_gpu_joint.py)."""

    def __init__(self, jd: JointDecoder, parts=2):
        from concurrent.futures import ThreadPoolExecutor
        self.jd = jd
        self.parts = [jd]
        op, code = jd.op, jd.code
        for _ in range(int(parts) - 1):
            c2 = _ldpc.code(code.standard, code.rate, code.z, code.ptype, device=code._device)
            # every slice decodes against jd's design (its ordering, whatever
            # seed built it): the twin's shared tables or its own copy of them
            self.parts.append(JointDecoder(jd.L, jd.M, jd.n, c2, jd.T, op.backend, op.precision, op.device,
                                           twin_of=jd if TWIN_SLICES else None, ordering=op.ordering))
        self._pool = ThreadPoolExecutor(max_workers=len(self.parts), thread_name_prefix="joint")
        self._slices = None

    def _cut(self, B):
        k = len(self.parts)
        edges = [B * i // k for i in range(k + 1)]
        return [slice(edges[i], edges[i + 1]) for i in range(k) if edges[i + 1] > edges[i]]

    def _map(self, fn):
        futs = [self._pool.submit(fn, part, sl) for part, sl in zip(self.parts, self._slices)]
        return [f.result() for f in futs]

    def stage(self, idx, noise, Pl):
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        noise = np.asarray(noise, dtype=np.float64).reshape(idx.shape[0], -1)
        self._slices = self._cut(idx.shape[0])
        self._map(lambda part, sl: part.stage(idx[sl], noise[sl], Pl))

    def decode_staged(self, idx, Pl, mode="soft", soft_iter=2, threshold=0.5, unit_cancel=False):
        """The slices start staggered: slice i + 1 starts when slice i's first
        AMP decode has finished, so that slice i's first BP (and every later
        stage) falls beside slice i + 1's AMP instead of beside its own twin."""
        import threading
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        assert self._slices is not None and self._slices[-1].stop == idx.shape[0], "stage the batch first"
        go = [threading.Event() for _ in self.parts]
        go[0].set()

        def one(part, sl):
            i = self.parts.index(part)
            go[i].wait()
            nxt = go[i + 1] if i + 1 < len(go) else None
            part._after_first_amp = nxt.set if nxt is not None else None
            try:
                return part.decode_staged(idx[sl], Pl, mode, soft_iter, threshold, unit_cancel)
            finally:
                part._after_first_amp = None
                if nxt is not None:
                    nxt.set()  # never leave the next slice waiting (an error, or a mode without that AMP)

        outs = self._map(one)
        return {k: np.concatenate([o[k] for o in outs], axis=0) for k in outs[0]}

    def run(self, idx, noise, Pl, mode="soft", soft_iter=2, threshold=0.5, unit_cancel=False):
        self.stage(idx, noise, Pl)
        return self.decode_staged(idx, Pl, mode, soft_iter, threshold, unit_cancel)

    def wait(self):
        for part in self.parts:
            part.op.wait()

    def close(self):
        self._pool.shutdown(wait=True)


_JD_CACHE: "OrderedDict[tuple, JointDecoder]" = OrderedDict()

# batches of at least this many codewords are decoded as two concurrent halves
PIPELINE_MIN_BATCH = 64
# the pipeline's extra slices share the first slice's operator tables
TWIN_SLICES = True


def joint_pipeline(jd: JointDecoder, parts=2) -> JointPipeline:
    """The JointPipeline over jd, cached on jd itself (the extra slices' tables
    and contexts built once, released with jd)."""
    jp = jd._pipeline
    if jp is None or len(jp.parts) != parts:
        if jp is not None:
            jp.close()
        jp = JointPipeline(jd, parts)
        jd._pipeline = jp
    return jp


def _evict(jd: JointDecoder):
    """A decoder leaving _JD_CACHE: its pipeline's thread pool and slices go too."""
    if jd._pipeline is not None:
        jd._pipeline.close()
        jd._pipeline.parts = [jd]
        jd._pipeline = None


def joint_decoder(L, M, n, ldpcparams: LDPCParams, T, backend=None, precision=None, device=None):
    """Cached JointDecoder (the operator tables and the LDPC graph are built once).

    AMP runs in binary64 unless told otherwise: in fp32 the softmax of the
    denoiser underflows below e^-87 (fp64: e^-745), so confident sections
    give p in {0, 1} exactly and the LLRs saturate at +-DBL_MAX, including
    for wrong decisions that BP could otherwise revise (measured: the fp32
    soft waterfall's BER_ldpc stalls near 0.4 above 7 dB, the fp64 one
    overlays the reference's published curve)."""
    precision = precision or "fp64"
    key = (L, M, n, ldpcparams.standard, ldpcparams.r_ldpc, ldpcparams.z, ldpcparams.ptype, T,
           backend, precision, device)
    jd = _JD_CACHE.get(key)
    if jd is None:
        code = _ldpc.code(ldpcparams.standard, ldpcparams.r_ldpc, ldpcparams.z, ldpcparams.ptype, device=device)
        jd = JointDecoder(L, M, n, code, T, backend, precision, device)
        _JD_CACHE[key] = jd
        while len(_JD_CACHE) > 4:
            _evict(_JD_CACHE.popitem(last=False)[1])
    else:
        _JD_CACHE.move_to_end(key)
    return jd


def _setup(sparcparams: SPARCParams, ldpcparams: LDPCParams, uniform_only=False, **kw):
    L, M, P = sparcparams.L, sparcparams.M, sparcparams.p
    n = int(L * np.log2(M) / sparcparams.r)
    if uniform_only or sparcparams.a is None:
        Pl = P / L * np.ones(L)
    else:
        Pl = pa_parameterised(L, sparcparams.C, P, sparcparams.a, sparcparams.f)
    jd = joint_decoder(L, M, n, ldpcparams, sparcparams.t, **kw)
    return jd, Pl


def amp_ldpc_sim_ldpc(sparcparams: SPARCParams, ldpcparams: LDPCParams, backend=None, precision=None):
    """LDPC branch of amp_ldpc_sim (sparc_ldpc.py:359-545): one rep from the
    global np.random stream.  Returns (ber_amp, ber_ldpc, ber_ldpc_amp | None, R)."""
    jd, Pl = _setup(sparcparams, ldpcparams, backend=backend, precision=precision)
    idx, noise = jd.draw(np.random, 1, sparcparams.sigma)
    r = jd.run(idx, noise, Pl, "originalHard")
    tb = jd.total_bits
    ber_ldpc_amp = float(r["ldpc_amp"][0]) / tb if "ldpc_amp" in r else None
    return float(r["amp"][0, 0]) / tb, float(r["ldpc"][0, 0]) / tb, ber_ldpc_amp, jd.R


def soft_amp_ldpc_sim(sparcparams: SPARCParams, ldpcparams: LDPCParams, soft_iter, a=None, f=None, C=None,
                      backend=None, precision=None):
    """sparc_ldpc.py:547-712: (ber_amp list (soft_iter+1), ber_ldpc list (soft_iter), R)."""
    jd, Pl = _setup(sparcparams, ldpcparams, backend=backend, precision=precision)
    idx, noise = jd.draw(np.random, 1, sparcparams.sigma)
    r = jd.run(idx, noise, Pl, "soft", soft_iter)
    tb = jd.total_bits
    return [float(e) / tb for e in r["amp"][0]], [float(e) / tb for e in r["ldpc"][0]], jd.R


def hardinitbeta_amp_ldpc_sim(sparcparams: SPARCParams, ldpcparams: LDPCParams, backend=None, precision=None):
    """sparc_ldpc.py:715-860 (uniform power only): (ber_amp [2], ber_ldpc [1], R)."""
    jd, Pl = _setup(sparcparams, ldpcparams, uniform_only=True, backend=backend, precision=precision)
    idx, noise = jd.draw(np.random, 1, sparcparams.sigma)
    r = jd.run(idx, noise, Pl, "hard")
    tb = jd.total_bits
    return [float(e) / tb for e in r["amp"][0]], [float(e) / tb for e in r["ldpc"][0]], jd.R


def mc_joint(jd: JointDecoder, Pl, sigma, seeds, mode, soft_iter=2, batch=256, threshold=0.5, unit_cancel=False,
             pipeline=None):
    """Seeded batched reps: rep s draws from RandomState(s) in the reference's
    order.  Returns the per-rep error-count dict of JointDecoder.run, in seed
    order.  pipeline (default: batches of PIPELINE_MIN_BATCH or more in the
    soft / hard / originalHard modes on the Hadamard backend, whose slices
    share one copy of the tables): decode each batch as two concurrent halves
    (JointPipeline), with the same per-rep results."""
    seeds = list(seeds)
    parts = []
    for s0 in range(0, len(seeds), batch):
        chunk = seeds[s0:s0 + batch]
        idx, noise = jd.draw([np.random.RandomState(s) for s in chunk], len(chunk), sigma)
        pipe = pipeline if pipeline is not None else (len(chunk) >= PIPELINE_MIN_BATCH and mode != "threshold"
                                                      and jd.op.backend == "hadamard")
        runner = joint_pipeline(jd) if pipe else jd
        parts.append(runner.run(idx, noise, Pl, mode, soft_iter, threshold, unit_cancel))
    return {k: np.concatenate([p[k] for p in parts], axis=0) for k in parts[0]}


# ---- LDPC with BPSK (sim_ldpc, sparc_ldpc.py:1049-1123) ----------------------------------

_RATES = {"1/2": .5, "2/3": 0.6667, "3/4": 0.75, "5/6": 0.83333, "0.45": 0.45}


def sim_ldpc(ldpcparams: LDPCParams, sigma, MIN_ERRORS=100, MAX_BLOCKS=400000, batch=1024, seed=None):
    """BER of the LDPC code with BPSK on AWGN, the reference's stopping rule
    (MIN_ERRORS block errors or MAX_BLOCKS blocks; BER = bit errors / (blocks N)).
    Blocks are decoded ``batch`` at a time on the GPU and consumed in order.
    Draws: np.random (global) unless ``seed`` is given."""
    if ldpcparams.r_ldpc not in _RATES:
        raise NameError("Rate unsupported")
    code = _ldpc.code(ldpcparams.standard, ldpcparams.r_ldpc, ldpcparams.z, ldpcparams.ptype)
    K, N = code.K, code.N
    rng = np.random if seed is None else np.random.RandomState(seed)
    std = ldpcparams.standard in ("802.11n", "802.16")
    nbit = nblk_err = nblocks = 0
    while True:
        U = rng.randint(0, 2, (batch, K)) if std else None
        X = code.encode_batch(U) if std else np.zeros((batch, N), dtype=np.int64)
        Y = (1.0 - 2.0 * X) + sigma * rng.randn(batch, N)
        app, _ = code.decode_batch(2.0 / sigma ** 2 * Y, "sumprod2")
        be = ((app < 0.0) != X).sum(axis=1)
        for b in be:
            nbit += int(b)
            nblk_err += 1 if b else 0
            nblocks += 1
            if nblk_err >= MIN_ERRORS or nblocks >= MAX_BLOCKS:
                return nbit / (nblocks * N)


# ---- waterfall (sparc_ldpc.py:1126-1282) ----------------------------------------------------

def waterfall(sparcparams: SPARCParams, ldpcparams: LDPCParams, csv_filename=None, png_filename=None,
              init="soft", pa_param=False, datapoints=10, MIN_ERRORS=100, MAX_BLOCKS=500, bpsk=True,
              sections=512, batch=64, seed0=0, backend=None, precision=None, rank=0, world=1, allreduce=None,
              ebno_dbs=None):
    """The reference's waterfall sweep on the GPU.  Per Eb/N0 point (20 log10
    convention): blocks of the joint scheme ``init`` and of plain SPARC at the
    same overall rate, consumed in seed order until MIN_ERRORS plain block
    errors or MAX_BLOCKS blocks (:1217-1245 counts the PLAIN block errors);
    BER_bpsk from sim_ldpc.  Reps are sharded over ranks like ber_point.
    Returns the rows; writes the reference CSV schema (:1257-1264) on rank 0."""
    from .harness import mc_decode
    precision = precision or "fp64"  # see joint_decoder
    L, M = sparcparams.L, sparcparams.M
    logm = int(np.log2(M))
    p, r_sparc, T = sparcparams.p, sparcparams.r, sparcparams.t
    nl = logm * sections
    z = int(nl / 24)
    ldp = LDPCParams(ldpcparams.standard, ldpcparams.r_ldpc, z)
    n_f = L * logm / r_sparc
    R = (L * logm - nl * (1 - 5 / 6)) / n_f  # HARD CODED RATE 5/6 (:1158-1160)
    if ebno_dbs is None:
        ebno_dbs = np.linspace(3, 10, datapoints)
    n = int(L * np.log2(M) / r_sparc)
    jd = joint_decoder(L, M, n, ldp, T, backend=backend, precision=precision)
    n_plain = int(L * np.log2(M) / R)
    plain = SparcOperator(L, M, n_plain, make_ordering(L, M, n_plain, 0), backend, precision)
    total_bits = L * logm
    rows = []
    for pi, ebno_db in enumerate(ebno_dbs):
        ebno = 10 ** (ebno_db / 20)
        sigma = ebno_to_sigma(ebno_db, p, R)
        a, f = sparcparams.a, sparcparams.f
        C = 0.5 * np.log2(1 + p / sigma ** 2)
        if pa_param and a is None:
            a = f = r_sparc / C
        Pl = p / L * np.ones(L) if (a is None or init == "hard") else pa_parameterised(L, C, p, a, f)
        Pl_plain = p / L * np.ones(L) if a is None else pa_parameterised(L, C, p, a, f)
        base = seed0 + pi * 10_000_000

        def round_fn(seeds, sigma=sigma, Pl=Pl, Pl_plain=Pl_plain):
            rj = mc_joint(jd, Pl, sigma, seeds, init, 2, batch)
            be_plain, _ = mc_decode(plain, Pl_plain, sigma, T, [s + 5_000_000 for s in seeds], batch=batch)
            cols = [rj["amp"][:, 0], rj["ldpc"][:, 0] if rj["ldpc"].shape[1] else 0 * be_plain]
            if init == "originalHard":
                cols.append(rj.get("ldpc_amp", 0 * be_plain))
                cols.append(0 * be_plain)
            else:
                cols.append(rj["amp"][:, 1])
                cols.append(rj["ldpc"][:, 1] if rj["ldpc"].shape[1] > 1 else 0 * be_plain)
            return be_plain, np.stack(cols, axis=1)

        res = _ber_point_multi(round_fn, total_bits, MIN_ERRORS, MAX_BLOCKS, batch, rank, world, allreduce, base)
        bpsk_ber = 0.0
        if bpsk:
            sigma_bpsk = np.sqrt((1 / ebno) / 2)
            bpsk_ber = sim_ldpc(ldp, sigma_bpsk, MIN_ERRORS, MAX_BLOCKS, seed=base + 7_000_000)
        rows.append(dict(EbN0_dB=float(ebno_db), BER_amp_1=res["cols"][0], BER_ldpc=res["cols"][1],
                         BER_amp_2=res["cols"][2], BER_ldpc_2=res["cols"][3], BER_plain=res["BER"],
                         BER_bpsk=bpsk_ber, blocks=res["blocks"], block_errors=res["block_errors"]))
    if csv_filename and rank == 0:
        fields = ["EbN0_dB", "BER_amp_1", "BER_ldpc", "BER_amp_2", "BER_ldpc_2", "BER_plain", "BER_bpsk"]
        with open(csv_filename, "a", newline="") as fh:
            wr = csv.DictWriter(fh, fieldnames=fields)
            wr.writeheader()
            for row in rows:
                wr.writerow({k: row[k] for k in fields})
    return rows


def _ber_point_multi(round_fn, total_bits, min_errors, max_blocks, batch, rank, world, allreduce, seed_base):
    """ber_point with extra per-block columns averaged over the same blocks;
    round_fn(seeds) -> (counting bit errors (B,), extra bit errors (B, k))."""
    from .dist import shard_seeds
    cum = None
    ber_cum = 0.0
    nerr = nblocks = 0
    rnd = 0
    while nerr < min_errors:
        seeds = shard_seeds(seed_base, rnd, batch, rank, world)
        be, extra = round_fn(seeds)
        k = extra.shape[1]
        glob = np.zeros((1 + k, batch * world), dtype=np.int64)
        glob[0, rank::world] = be
        glob[1:, rank::world] = np.asarray(extra, dtype=np.int64).T
        if allreduce is not None:
            glob = allreduce(glob)
        if cum is None:
            cum = np.zeros(k)
        done = False
        for j in range(batch * world):
            if nerr >= min_errors:
                done = True
                break
            b = int(glob[0, j])
            ber_cum += b / total_bits
            cum += glob[1:, j] / total_bits
            nerr += 1 if b > 0 else 0
            nblocks += 1
            if nblocks >= max_blocks:
                done = True
                break
        if done:
            break
        rnd += 1
    return dict(BER=ber_cum / nblocks, cols=(cum / nblocks).tolist(), blocks=nblocks, block_errors=nerr)


# ---- soft_hard_plot (sparc_ldpc.py:1285-1432) ----------------------------------------------

def soft_hard_plot(soft, hard, sec, soft_iter, sparcparams: SPARCParams, ldpcparams: LDPCParams, csv_filename=None,
                   png_filename=None, datapoints=10, MIN_ERRORS=100, MAX_BLOCKS=500, batch=64, seed0=0,
                   backend=None, precision=None, rank=0, world=1, allreduce=None, sigmas=None):
    """Soft exchange vs the original hard exchange on the GPU.

    The LDPC code covers nl = log2(M) * sec bits with z = int(nl / 24)
    (802.16 rate 5/6: N = 24 z bits, i.e. N / log2 M sections); overall rate
    R = (L log2 M - nl / 6) / n (:1309-1314, the 5/6 hard-coded as there).
    Per sigma of linspace(0.8, 0.4, datapoints) (:1322): BER_sparc = mean over
    MIN_ERRORS plain-SPARC reps at rate R (:1334-1337); soft: soft_amp_ldpc_sim
    blocks until MIN_ERRORS blocks with LDPC errors after round 1 or
    MAX_BLOCKS (:1339-1353); hard: amp_ldpc_sim (LDPC branch) blocks with the
    same rule (:1354-1369).  Blocks are seeded and batched (mc_joint) and
    sharded over ranks like waterfall.  Returns rows (EbN0_dB, BER_sparc,
    BER_ldpc_soft [soft_iter], BER_amp_soft [soft_iter + 1], BER_ldpc_hard,
    BER_amp_hard [2], blocks); rank 0 appends the reference's two CSV blocks
    (:1397-1413).  No plots."""
    from .harness import mc_decode
    from .dist import shard_seeds
    precision = precision or "fp64"
    L, M, p, r_sparc, T = sparcparams.L, sparcparams.M, sparcparams.p, sparcparams.r, sparcparams.t
    logm = int(np.log2(M))
    nl = logm * sec
    z = int(nl / 24)
    ldp = LDPCParams(ldpcparams.standard, ldpcparams.r_ldpc, z, ldpcparams.ptype)
    n_f = L * logm / r_sparc
    R = (L * logm - nl * (1 - 5 / 6)) / n_f
    n = int(L * np.log2(M) / r_sparc)
    n_plain = int(L * np.log2(M) / R)
    total_bits = L * logm
    Pl = p / L * np.ones(L)
    jd = joint_decoder(L, M, n, ldp, T, backend=backend, precision=precision)
    plain = SparcOperator(L, M, n_plain, make_ordering(L, M, n_plain, 0), backend, precision)
    SIGMA = np.linspace(0.8, 0.4, datapoints) if sigmas is None else np.asarray(sigmas, dtype=np.float64)
    rows = []
    for pi, sigma in enumerate(SIGMA):
        sigma = float(sigma)
        base = seed0 + pi * 10_000_000
        seeds = [s for s in range(base + 5_000_000, base + 5_000_000 + MIN_ERRORS) if s % world == rank]
        be_plain, _ = mc_decode(plain, Pl, sigma, T, seeds, batch=batch)
        tot = np.array([int(be_plain.sum())], dtype=np.int64)
        if allreduce is not None:
            tot = allreduce(tot)
        row = dict(EbN0_dB=float(20 * np.log10(1 / (2 * R) * (p / sigma ** 2))), sigma=sigma,
                   BER_sparc=float(tot[0]) / (MIN_ERRORS * total_bits))
        for mode, on in (("soft", soft), ("originalHard", hard)):
            if not on:
                continue

            def round_fn(sds, mode=mode, sigma=sigma):
                rj = mc_joint(jd, Pl, sigma, sds, mode, soft_iter, batch)
                if mode == "soft":
                    return rj["ldpc"][:, 0], np.concatenate([rj["ldpc"], rj["amp"]], axis=1)
                cols = [rj["ldpc"][:, 0], rj["amp"][:, 0], rj.get("ldpc_amp", 0 * rj["amp"][:, 0])]
                return rj["ldpc"][:, 0], np.stack(cols, axis=1)

            res = _ber_point_multi(round_fn, total_bits, MIN_ERRORS, MAX_BLOCKS, batch, rank, world, allreduce,
                                   base + (0 if mode == "soft" else 2_500_000))
            c = res["cols"]
            if mode == "soft":
                row.update(BER_ldpc_soft=c[:soft_iter], BER_amp_soft=c[soft_iter:], blocks_soft=res["blocks"])
            else:
                row.update(BER_ldpc_hard=c[0], BER_amp_hard=[c[1], c[2]], blocks_hard=res["blocks"])
        rows.append(row)
    if csv_filename and rank == 0:
        for mode, fields in (("soft", ["EbN0_dB", "BER_sparc", "BER_ldpc_soft", "BER_amp_soft"]),
                             ("hard", ["EbN0_dB", "BER_sparc", "BER_ldpc_hard", "BER_amp_hard"])):
            if not (soft if mode == "soft" else hard):
                continue
            with open(csv_filename, "a", newline="") as fh:
                wr = csv.DictWriter(fh, fieldnames=fields)
                wr.writeheader()
                for row in rows:
                    wr.writerow({k: (np.array(row[k]) if isinstance(row[k], list) else row[k]) for k in fields})
    return rows
