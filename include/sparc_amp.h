/*
 * sparc_amp.h — C ABI of the MI355X (gfx950) SPARC AMP decoder.
 *
 * Library: sparc_ldpc_amd/libsparc_amp.so (hipcc --offload-arch=gfx950).
 *
 * The reference (Spimp/sparc_ldpc) has no native boundary on this path: the
 * whole AMP decoder is Python/NumPy.  These entry points replace the Python
 * functions named on each declaration, with the reference's own native
 * boundary conventions (ldpc/py/ldpc.py:859-929 -> ldpc/src/c_ldpc.c:32-113):
 * plain pointers and sizes, caller-allocated outputs, int status returns,
 * no Python objects across the ABI.  fp64 at the ABI (the reference computes
 * in fp64); fp32 or fp64 on the device (precision argument of sa_create).
 *
 * Status codes: 0 = OK, < 0 = error (sa_last_error() describes the last one
 * raised on the calling thread).  A context is bound to one device and one
 * HIP stream; it is not thread-safe, but contexts on different devices may be
 * driven concurrently from different threads.
 */
#ifndef SPARC_AMP_H
#define SPARC_AMP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sa_ctx sa_ctx;

enum {
  SA_OK = 0,
  SA_ERR_ARG = -1,          /* bad size / shape / pointer (reference: AssertionError) */
  SA_ERR_HIP = -2,          /* HIP runtime failure */
  SA_ERR_NOMEM = -3,        /* device allocation failed (reference: c_ldpc.c:40-42 -> -1) */
  SA_ERR_ORDERING = -4,     /* ordering row not distinct / out of [1, w) */
  SA_ERR_UNSUPPORTED = -5,  /* configuration outside this backend's limits */
  SA_ERR_NO_DEVICE = -6     /* no HIP device visible */
};

enum {
  SA_BACKEND_HADAMARD = 0,  /* matrix-free sub-sampled Walsh-Hadamard operator (default) */
  SA_BACKEND_DENSE = 1,     /* materialised n x (L*M) design matrix: fp32 GEMVs for B < 4
                               codewords, int8 matrix-core GEMMs on exact +-1 entries with
                               three-digit fixed-point vectors for B >= 4 */
  SA_BACKEND_HOST = 2,      /* no device operator: the caller's own Ab / Az (any operator, as the
                               reference's amp() accepts any callables) applied on the host, the
                               loop's tau, denoiser and residual on the device (sa_host_*) */
  SA_BACKEND_MATRIX = 3     /* a caller's own dense n x (L*M) design matrix (e.g. i.i.d. Gaussian;
                               sa_create_matrix) held on the device in the context precision:
                               GEMVs for B < 4 codewords, f32 / f64 MFMA GEMMs for B >= 4 */
};

enum { SA_PREC_F32 = 0, SA_PREC_F64 = 1 };

/* sa_amp / sa_run flags */
enum {
  SA_FLAG_NO_EARLY_STOP = 1, /* run exactly T iterations (ignore the tau == last_tau stop) */
  SA_FLAG_BETA0 = 0x100,     /* sa_run: start from the beta0 staged by sa_stage */
  SA_PTR_DEVICE = 0x200      /* sa_llr / sa_soft_beta0 / sa_hard_cancel: llr / app are device pointers */
};

/* Replaces sparc_transforms(L, M, n, seed) / block_sub_fht(n, M, L, ordering)
 * (ldpc/sparc_ldpc.py:140-147, :81-136): builds the design operator of L
 * sections of M columns over n rows from `ordering` (L x n, row-major,
 * values in [1, w), w = 2^ceil(log2(max(M+1, n+1))), distinct per row) on
 * `device`.  The ordering itself is generated on the host by the caller with
 * the reference's RandomState algorithm (sparc_ldpc.py:107-117). */
int sa_create(sa_ctx** out, int L, int M, int n, const uint32_t* ordering,
              int backend, int precision, int device);

/* sa_create with plan options: which kernels and layouts a decode uses is
 * normally chosen by built-in rules from (L, M, n, precision, batch, CUs)
 * (sa_plan reports the choice); these bits override a rule, e.g. to test a
 * kernel on shapes where the rule would not pick it.  Every option keeps the
 * results within the same parity bounds; SA_PLAN_NO_PT, SA_PLAN_EAGER and
 * SA_PLAN_ONE_PASS are bit-identical to the default plan.  `sa_subset` contexts
 * inherit their parent's options. */
enum {
  SA_PLAN_DEFAULT = 0,
  SA_PLAN_SEC3 = 1 << 0,      /* one codeword: three sections per workgroup (k_sec43) where it fits */
  SA_PLAN_NO_SEC3 = 1 << 1,   /* one codeword: never k_sec43 (pairs, k_sec4) */
  SA_PLAN_ROW16 = 1 << 2,     /* one codeword: 16-row k_row2 blocks where they fit */
  SA_PLAN_NO_ROW16 = 1 << 3,  /* one codeword: 32-row k_row2 blocks */
  SA_PLAN_NO_PT = 1 << 4,     /* Ab partials [G][n] instead of row-block major (bit-identical) */
  SA_PLAN_ZIL = 1 << 5,       /* batched: z / Ab partials codeword-interleaved (the default since round 4) */
  SA_PLAN_NO_ZIL = 1 << 6,    /* batched: z / Ab partials [B][n] (binary32 too) */
  SA_PLAN_WB8 = 1 << 7,       /* batched: 8 sections per workgroup */
  SA_PLAN_WB16 = 1 << 8,      /* batched: 16 sections per workgroup */
  SA_PLAN_NO_BANKS = 1 << 9,  /* batched: bucket slots summed in h order (no bank-aware slot order) */
  SA_PLAN_EAGER = 1 << 10,    /* sa_run launches eagerly instead of replaying a captured hipGraph */
  SA_PLAN_ONE_PASS = 1 << 11, /* batched: every section group of an XCD in one pass of the work order */
  SA_PLAN_ALL = (1 << 12) - 1
};
int sa_create_ex(sa_ctx** out, int L, int M, int n, const uint32_t* ordering,
                 int backend, int precision, int device, int plan);

/* A caller's own dense design (the reference's amp() with any pair of
 * callables, sparc_ldpc.py:189,213,220, e.g. Ab = lambda b: A @ b,
 * Az = lambda z: A.T @ z for an i.i.d. Gaussian A): A is n x (L*M) row-major
 * binary64, copied to the device in `precision`; the context's sa_Ab / sa_Az
 * compute A beta / A^T z (no 1/sqrt(n): the matrix is used as given) and
 * sa_amp / sa_run run the whole loop on the device.  Section sizes M need not
 * be powers of two.  sa_encode / sa_cancel / sa_subset need an ordering
 * (SA_ERR_UNSUPPORTED here). */
int sa_create_matrix(sa_ctx** out, int L, int M, int n, const double* A,
                     int precision, int device);

/* The same backend with an i.i.d. N(0, scale^2) design generated on the
 * device (e.g. scale = 1/sqrt(n): unit-norm columns on average) for
 * simulations that never need the matrix on the host: Philox4x32-10 keyed by
 * `seed`, counter = row-major element index / 4, Box-Muller; reproducible per
 * (seed, element), not NumPy's stream. */
int sa_create_matrix_random(sa_ctx** out, int L, int M, int n, uint64_t seed, double scale,
                            int precision, int device);

/* Replaces sparc_transforms_shorter(L, M, n, ordering[sections])
 * (ldpc/sparc_ldpc.py:154-168; called with a fancy-indexed subset at
 * ldpc/amp_exit.py:113-116): a new context over the given parent sections. */
int sa_subset(const sa_ctx* parent, const int64_t* sections, int Ls, sa_ctx** out);

/* A second context over src's operator (the same L, M, n, ordering, backend,
 * precision, device and plan) that shares src's device tables, read-only,
 * and has its own stream, workspace and power allocation: concurrent decodes
 * of one operator (joint.JointPipeline's slices) read one copy of the tables
 * from L2.  src must outlive the twin.  Hadamard backend only. */
int sa_create_twin(sa_ctx* src, sa_ctx** out);

void sa_destroy(sa_ctx* ctx);

/* Replaces the Ab closure, sparc_ldpc.py:143-144 (-> block_sub_fht.Ax
 * :120-126): out[b] = A beta[b] for B codewords.  beta: B x (L*M), out: B x n. */
int sa_Ab(sa_ctx* ctx, int B, const double* beta, double* out);

/* Replaces the Az closure, sparc_ldpc.py:145-146 (-> block_sub_fht.Ay
 * :128-134): out[b] = A^T z[b].  z: B x n, out: B x (L*M). */
int sa_Az(sa_ctx* ctx, int B, const double* z, double* out);

/* Replaces amp(y, sigma_n, Pl, L, M, T, Ab, Az, beta) (sparc_ldpc.py:189-222)
 * and amp_test (ldpc/amp_test.py:14-50) for B independent codewords sharing
 * the operator: y: B x n; Pl: L section powers; beta0: B x (L*M) or NULL for
 * the zero start; beta_out: B x (L*M); iters_out (may be NULL): per codeword
 * the loop index at which the exact tau == last_tau stop fired, or T when
 * the loop ran to completion.  sigma_n is not an argument: the reference
 * never reads it. */
int sa_amp(sa_ctx* ctx, int B, const double* y, const double* Pl, int T,
           const double* beta0, double* beta_out, int* iters_out, int flags);

/* ---- device-resident path (bench / Monte-Carlo harness) ----------------
 * sa_reserve sizes the device workspace for B codewords and T iterations
 * (it discards staged data when it has to grow) and builds the tables a
 * decode of B codewords needs that are built lazily (the batched kernel's
 * bank-aware tables, once per operator); sa_stage copies y (and Pl, and optionally beta0) into the context's device
 * buffers; sa_run decodes the staged batch asynchronously on the context's
 * stream (replayed hipGraph); sa_wait blocks until it is done; sa_fetch
 * copies the results back.  sa_run_event_ms returns the device time of the
 * last sa_run measured with HIP events on the context's stream. */
int sa_reserve(sa_ctx* ctx, int B, int T);
int sa_stage(sa_ctx* ctx, int B, const double* y, const double* Pl, const double* beta0);
/* Per-codeword power allocations Pl [B][L] (Hadamard backend) for the next
 * sa_run of up to B codewords: c_{b,l} = sqrt(n Pl_{b,l}), P_b = sum_l Pl_{b,l}
 * (sparc_ldpc.py:190,214).  Sections with Pl = 0 keep beta = 0 and drop out
 * of A beta, so this is the reference's shortened-operator decode
 * (sparc_transforms_shorter, amp_exit.py:113-116) as a per-codeword section
 * mask.  The binary64 glue kernels (sa_llr, ...) keep the c_l of the last
 * sa_stage Pl; a later sa_stage with Pl returns to one allocation. */
int sa_stage_power_batch(sa_ctx* ctx, int B, const double* Pl);
int sa_run(sa_ctx* ctx, int B, int T, int flags);
int sa_wait(sa_ctx* ctx);
int sa_fetch(sa_ctx* ctx, int B, double* beta_out, int* iters_out);
/* The residual z of the last decode's final iteration, B x n (diagnostics). */
int sa_fetch_z(sa_ctx* ctx, int B, double* z_out);
double sa_run_event_ms(sa_ctx* ctx);

/* Per-kernel device time of one EAGER decode of the staged batch (every
 * launch bracketed by HIP events on the context's stream).  out[13]:
 * {mean ms, launches} for kernel kinds 0 section (k_sec), 1 row (k_row),
 * 2 dense A^T z (fp32 GEMV; int8 MFMA GEMM for B >= 4), 3 dense denoiser,
 * 4 dense A beta (GEMV; int8 MFMA GEMM for B >= 4), 5 int8 digit-plane
 * quantisation of z / beta0; out[12] = total ms of the sequence.  Leaves the
 * decode's results in place like sa_run. */
int sa_profile(sa_ctx* ctx, int B, int T, int flags, double* out);
/* Number of kernel kinds K of sa_profile / sa_profile_rep: `out` holds 2 K + 1
 * doubles (K = 6 since SA_VERSION 0.2: size buffers from this, not a constant). */
int sa_profile_kinds(void);
/* The same with every bracketed launch issued `rep` (1..1024) times back to
 * back between its events: mean = elapsed / rep, i.e. the launch's duration
 * plus the same-stream kernel boundary, without the event packets' dispatch
 * overhead.  The results left in place are then those of repeated
 * launches (not a decode); re-run sa_run before fetching. */
int sa_profile_rep(sa_ctx* ctx, int B, int T, int flags, int rep, double* out);
/* The same eager decode with every loop kernel launched once through
 * hipExtLaunchKernel with a start / stop event pair bound to the kernel's own
 * dispatch: {mean ms, launches} per kind is the kernels' execution time in
 * the decode's order (what a rocprofv3 kernel trace records), with no marker
 * packets between the launches.  Leaves the decode's results in place. */
int sa_profile_dispatch(sa_ctx* ctx, int B, int T, int flags, double* out);

/* Per-codeword section decisions (sparc_ldpc.py:452-455: argmax per
 * section, first index on ties) of the last sa_run / sa_amp, computed on
 * device: idx_out is B x L. */
int sa_decide(sa_ctx* ctx, int B, int32_t* idx_out);

/* The same decision, pipelined: sa_decide_async enqueues the argmax and the
 * copy of its B x L indices into slot `slot` (0 .. SA_DECIDE_SLOTS-1) of a
 * context-owned pinned host ring behind the work already on the stream and
 * returns at once; sa_decide_collect waits for that slot's copy only and
 * hands its indices to the caller (idx_out: B x L).  A decoder loop queues
 * decode k + 1 before it collects the decisions of decode k, so the device
 * never waits on the host. */
enum { SA_DECIDE_SLOTS = 4 };
int sa_decide_async(sa_ctx* ctx, int B, int slot);
int sa_decide_collect(sa_ctx* ctx, int B, int slot, int32_t* idx_out);

/* ---- SPARC <-> LDPC glue of the joint decoder (sparc_ldpc.py:359-712) ---
 * Binary64 kernels on the staged batch; llr / app arrays are [B][ns*log2 M]
 * (the LDPC bits of sections l0 .. l0+ns-1, MSB first) and may be device
 * pointers shared with libldpc_bp.so (flag SA_PTR_DEVICE). */

/* Encoder (sparc_ldpc.py:436-446): y[b] = A beta(idx[b]) + noise[b] staged as
 * the decode input, beta(idx) one-hot with c_l = sqrt(n Pl_l) at column
 * idx[b][l] of section l.  idx: B x L; noise: B x n or NULL.  Needs Pl staged
 * (sa_stage(ctx, B, NULL, Pl, NULL)). */
int sa_encode(sa_ctx* ctx, int B, const int32_t* idx, const double* noise);

/* Hard re-initialisation (sparc_ldpc.py:831-838): stage the one-hot beta0
 * with c_l at idx[b][l] (B x L) for the next sa_run(..., SA_FLAG_BETA0). */
int sa_stage_onehot(sa_ctx* ctx, int B, const int32_t* idx);

/* The same with amplitude scale * c_l, idx -1 = an all-zero section: the 0/1
 * start beta_0 = beta / sqrt(n P / L) with its first L_zero sections zeroed of
 * the amp_test.py reps loop (amp_test.py:202-204; scale = 1 / sqrt(n P / L)). */
int sa_stage_onehot_scaled(sa_ctx* ctx, int B, const int32_t* idx, double scale);

/* sp2bp + LLR (sparc_ldpc.py:470-479, :257-281) of sections [l0, l0+ns) of
 * the current beta: llr = nan_to_num(log(1-p) - log(p)), p the bitwise
 * posterior of beta_l / c_l. */
int sa_llr(sa_ctx* ctx, int B, int l0, int ns, double* llr, int flags);

/* Soft exchange (sparc_ldpc.py:683-698): beta0 := beta with sections
 * [l0, l0+ns) replaced by c_l * bp2sp(1/(1+exp(app))), staged for the next
 * sa_run(..., SA_FLAG_BETA0); the staged y is kept. */
int sa_soft_beta0(sa_ctx* ctx, int B, int l0, int ns, const double* app, int flags);

/* Hard exchange (sparc_ldpc.py:486-524): idx = bits2indices(app < 0) for
 * sections [l0, l0+ns) (idx_out: B x ns, may be NULL); if dst is given (a
 * context over the same n, e.g. sa_subset of the kept sections), stages
 * y - A beta_hard(idx) as dst's input y. */
int sa_hard_cancel(sa_ctx* ctx, int B, int l0, int ns, const double* app, int flags, sa_ctx* dst,
                   int32_t* idx_out);

/* Threshold decisions (amp_exit.py:56-105): for sections [l0, l0+ns) the
 * bp2sp of the LLRs `app` ([B][ns*log2 M]); idx_out[b][s] = the entry whose
 * normalised probability exceeds `threshold` if exactly one does, else -1. */
int sa_threshold(sa_ctx* ctx, int B, int l0, int ns, const double* app, int flags, double threshold,
                 int32_t* idx_out);

/* Hard cancellation of decided sections (amp_exit.py:107-109): stages
 * y - A beta(idx) as dst's input y, idx [B][L] with -1 for sections that are
 * not cancelled; dst is a context over the same n (e.g. sa_subset of the
 * undecided sections). */
int sa_cancel(sa_ctx* ctx, int B, const int32_t* idx, sa_ctx* dst);

/* The same with beta(idx) at amplitude scale * c_l: y - Ab(beta_0) of the
 * amp_test.py reps loop's hard initialisation (amp_test.py:207-210), where
 * beta_0 carries 1 = c_l / sqrt(n P / L) at the decided sections. */
int sa_cancel_scaled(sa_ctx* ctx, int B, const int32_t* idx, double scale, sa_ctx* dst);

/* ---- host-operator AMP (SA_BACKEND_HOST context; sa_create with ordering
 * NULL) ------------------------------------------------------------------
 * The reference's amp() takes ANY pair of callables (sparc_ldpc.py:189,196,
 * 213,220).  For operators that are not this library's, the caller applies
 * Ab / Az itself and the loop's other steps run on the device:
 *   sa_host_init(B, T, y, Pl, beta0, Ab(beta0))  z = y - Ab(beta0) (:192-200; both NULL: zero start)
 *   for t < T:
 *     sa_host_tau(t, stopped)        tau_t = sqrt(sum z^2 / n), stopped[b] = (tau_t == tau_{t-1}) (:203-209)
 *     if every codeword stopped: done
 *     sa_fetch_z -> the caller computes Az(z)
 *     sa_host_eta(t, Az(z))          beta = eta(beta + Az(z)) (:213-219)
 *     sa_fetch -> the caller computes Ab(beta)
 *     sa_host_residual(t, Ab(beta))  z = y - Ab(beta) + z / tau^2 (P - sum beta^2 / n) (:220)
 * Stopped codewords keep beta and z.  flags: SA_FLAG_NO_EARLY_STOP. */
int sa_host_init(sa_ctx* ctx, int B, int T, const double* y, const double* Pl, const double* beta0,
                 const double* ab0);
int sa_host_tau(sa_ctx* ctx, int B, int t, int flags, int* stopped);
int sa_host_eta(sa_ctx* ctx, int B, int t, int flags, const double* az);
int sa_host_residual(sa_ctx* ctx, int B, int t, int flags, const double* ab);

/* Monte-Carlo rep stream (BASELINE configs[3]: amp_test.py:183-246, the BER
 * sweeps of sparc_ldpc.py:1217-1245 / 1318-1323).
 *
 * sa_draw_reps: on the host cores, rep i drawn as NumPy's
 * RandomState(seeds[i]).randint(0, M, L) (idx_out [count][L]) followed by
 * .randn(n) * sigma (noise_out [count][n]), bit for bit NumPy's legacy
 * generator (MT19937, masked bounded integers, polar Gaussian); threads <= 0:
 * every hardware thread.
 *
 * sa_mc_stage copies `nreps` reps (section indices [nreps][L], noise
 * [nreps][n], fp64) to the device.  sa_mc_run decodes them through B slots
 * (4 <= B <= 1024) of the batched decode with per-slot refill: each slot runs
 * its own iteration index, and when its exact-tau stop fires or T iterations
 * are done its section decisions go to dec_out [nreps][L] and its stop index
 * (T when the loop ran out) to iters_out [nreps], and the next rep is encoded
 * into the slot (y = A beta(idx) + noise) on the device; errs_out [nreps]
 * receives each rep's bit errors (the popcounts of decision ^ index summed
 * over its sections, sparc_ldpc.py:462); any output may be NULL.  Every rep's
 * decisions and stop index equal those of sa_encode + sa_run(early stop) +
 * sa_decide on any batch holding it.  Needs one staged power allocation
 * (sa_stage Pl) and the batched codeword-interleaved Hadamard decode
 * (sa_plan: k_secb + k_rowc), else SA_ERR_UNSUPPORTED; ms_out: the device
 * time of the whole stream (events), or NULL. */
int sa_draw_reps(const uint32_t* seeds, int count, int L, int M, int n, double sigma, int32_t* idx_out,
                 double* noise_out, int threads);
int sa_mc_stage(sa_ctx* ctx, int nreps, const int32_t* idx, const double* noise);
int sa_mc_run(sa_ctx* ctx, int B, int T, int flags, int32_t* dec_out, int32_t* iters_out, int32_t* errs_out,
              double* ms_out);
/* The design's row sub-sampling table (sparc_ldpc.py:107-117): NumPy's
 * RandomState(seed) shuffling arange(1, w) once per section, cumulatively,
 * the first n of each kept, w = 2^ceil(log2(max(M+1, n+1))); out [L][n]. */
int sa_make_ordering(int L, int M, int n, uint32_t seed, uint32_t* out);

/* Introspection. */
/* The kernels a decode of B codewords runs: out8 = {section kernel (0 k_sec,
 * 1 k_sec2, 2 k_secb, 3 dense fp32 GEMVs, 4 k_sec4, 5 k_sec43, 6 dense int8
 * MFMA GEMMs, 7 caller-matrix f32 / f64 MFMA GEMMs, 8 k_secg: z from global
 * memory, 32-bit bucket entries, for n past the LDS image or >= 65535), Ab partials per codeword, row splits,
 * codewords per batched workgroup, z^2 partials, w, row kernel (1 k_row2,
 * 2 k_rowv 16-byte rows, 3 k_rowv 8-byte rows, 0 k_row, 4 k_row2 16-row
 * blocks, 5 k_rowc), number of CUs}. */
int sa_plan(sa_ctx* ctx, int B, int64_t* out8);
/* The batched section kernel's work order for B codewords (k_secb, B >= 4):
 * out4 = {section groups, sections per workgroup, section groups per XCD per
 * pass, passes per XCD}; SA_ERR_ARG when a decode of B does not run k_secb. */
int sa_plan_batched(sa_ctx* ctx, int B, int64_t* out4);
int sa_info(const sa_ctx* ctx, int64_t* out8); /* L, M, n, w, backend, precision, device, bytes */
int sa_device_count(void);
const char* sa_last_error(void);
const char* sa_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SPARC_AMP_H */
