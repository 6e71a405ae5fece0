/* ldpc_bp.h — C ABI of the MI355X (gfx950) LDPC belief-propagation decoder.
 *
 * Replaces the reference's native LDPC decoder ldpc/src/c_ldpc.c, bound by
 * ctypes in ldpc/py/ldpc.py:855-930 (code.decode).  Two layers:
 *
 *  1. Reference-signature entry points (sumprod, sumprod2, minsum, Lxor,
 *     Lxfb): same names, argument lists and meaning as c_ldpc.c:32, 138, 339,
 *     234, 294, so `ct.CDLL(".../libldpc_bp.so")` can stand in for
 *     `ct.CDLL('./bin/c_ldpc.so')` (ldpc.py:859) unchanged.  They decode one
 *     word on the GPU (the graph is uploaded once and cached by content).
 *     Return: iteration count (0..200) as the reference, or a negative
 *     LB_ERR_* code (the reference returns -1 when calloc fails, c_ldpc.c:40-42).
 *
 *  2. A context API for batches of B words sharing one graph (Monte-Carlo),
 *     with device-resident buffers for the joint SPARC/LDPC pipeline.
 *
 * All arithmetic is IEEE binary64 in the reference's per-node operation order.
 * Graph arrays follow ldpc.py:694-786: vdeg[Nv], cdeg[Nc], intrlv[Nmsg]
 * (message index, in check-node order, of each variable-node port).
 */
#ifndef LDPC_BP_H
#define LDPC_BP_H

#ifdef __cplusplus
extern "C" {
#endif

enum {
  LB_OK = 0,
  LB_ERR_ARG = -1,         /* bad argument (reference: NameError / assert) */
  LB_ERR_HIP = -2,         /* HIP runtime failure */
  LB_ERR_NOMEM = -3,       /* device allocation failed (c_ldpc.c:40-42 returns -1) */
  LB_ERR_GRAPH = -4,       /* degrees do not sum to Nmsg, or intrlv is not a permutation */
  LB_ERR_UNSUPPORTED = -5, /* check degree > 32 or variable degree > 255 */
  LB_ERR_NO_DEVICE = -6    /* no HIP device: there is no CPU fallback */
};

enum { LB_SUMPROD2 = 0, LB_SUMPROD = 1, LB_MINSUM = 2 };

#define LB_MAX_ITCOUNT 200 /* c_ldpc.c:7 */

typedef struct lb_ctx lb_ctx;

/* ---- reference-signature drop-ins (c_ldpc.c) ---------------------------- */
int sumprod(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg,
            double* app);                                      /* c_ldpc.c:32  */
int sumprod2(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg,
             double* app);                                     /* c_ldpc.c:138 */
int minsum(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg,
           double* app, double correction_factor);             /* c_ldpc.c:339 */
double Lxor(double L1, double L2, int corr_flag);              /* c_ldpc.c:234; NaN on failure */
double Lxfb(double* L, long dc, int corr_flag);                /* c_ldpc.c:294; NaN on failure */

/* ---- batched context API ---------------------------------------------------- */
/* Upload a graph (host arrays as above) to `device`. */
int lb_create(lb_ctx** out, const long* vdeg, const long* cdeg, const long* intrlv, int Nv, int Nc,
              int Nmsg, int device);
void lb_destroy(lb_ctx* ctx);

/* Decode B words: ch[B][Nv] channel LLRs -> app[B][Nv] a-posteriori LLRs and
 * iters[B] (the reference's return value per word).  Host pointers; blocking. */
int lb_decode(lb_ctx* ctx, int B, const double* ch, double* app, int* iters, int algo,
              double corr_factor, int max_iter);

/* Device-resident form: d_ch / d_app / d_iters are device pointers on the
 * context's device; queued on the context's stream, returns without waiting
 * (the tail is sized on the device, see lb_set_tail). */
int lb_decode_device(lb_ctx* ctx, int B, const double* d_ch, double* d_app, int* d_iters, int algo,
                     double corr_factor, int max_iter);

/* Device buffers of the context sized for B words (ch, app: B x Nv doubles;
 * iters: B ints), for handing LLRs to / from other device code (the SPARC
 * glue of libsparc_amp.so) without a host round trip.  lb_run / lb_fetch
 * operate on them. */
int lb_buffers(lb_ctx* ctx, int B, double** d_ch, double** d_app, int** d_iters);

/* Measurement helpers: stage B words into the context's device buffers, run
 * (asynchronously), wait, fetch; lb_run_event_ms = device time of the last run. */
int lb_stage(lb_ctx* ctx, int B, const double* ch);
int lb_run(lb_ctx* ctx, int B, int algo, double corr_factor, int max_iter);
int lb_wait(lb_ctx* ctx);
int lb_fetch(lb_ctx* ctx, int B, double* app, int* iters);
double lb_run_event_ms(lb_ctx* ctx);

/* out[0..9] = Nv, Nc, Nmsg, max vdeg, max cdeg, messages in LDS (1/0),
 *             threads per workgroup, device, the check degree of the
 *             straight-line check kernel of a check-regular code (0: the
 *             general kernel), and the first tail iteration (0: off) */
int lb_info(lb_ctx* ctx, long long* out);

/* Tail launches: a decode runs its first `tail_at` iterations one workgroup
 * per word; the words still running after that are spread over several
 * workgroups each, two launches per iteration (bit-identical results).
 * lb_decode (blocking) reads back the number of words left once and sizes
 * the tail for them, issuing iterations until a read-back shows every word
 * done; lb_run / lb_decode_device never wait: every iteration up to
 * max_iter is queued, sized from the previous tail's word count, and a
 * launch past the last running word returns at once.  tail_at < 0: the
 * default chosen at lb_create (8, or the environment's LDPC_BP_TAIL); 0: off.
 * Needs variable degrees <= 12 (LB_ERR_UNSUPPORTED otherwise). */
int lb_set_tail(lb_ctx* ctx, int tail_at);
int lb_device_count(void);
const char* lb_last_error(void);
const char* lb_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_BP_H */
