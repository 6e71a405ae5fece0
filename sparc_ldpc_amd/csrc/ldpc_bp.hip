// ldpc_bp.hip — MI355X (gfx950) LDPC belief-propagation decoder + C ABI.
//
// Replaces ldpc/src/c_ldpc.c (sumprod2 :138-206 with Lxfb :294-314 and Lxor
// :234-251; sumprod :32-113; minsum :339-381), bound by code.decode in
// ldpc/py/ldpc.py:855-930.
//
// Flooding schedule, one workgroup per codeword.  The message array (one
// binary64 per edge, in check-node order as the reference lays it out) lives
// in LDS when it fits (802.16 rate 5/6 z=192: 15360 edges = 120 KB of the
// 160 KB per CU), otherwise in a per-codeword HBM slice.  Per iteration:
//   variable phase: thread per variable node, sum channel + incoming edges
//     in port order (c_ldpc.c:171-178), write extrinsics and app;
//   check phase: thread per check node, forward/backward Lxor pass over its
//     contiguous edges (c_ldpc.c:294-314) with the forward values in
//     registers and the backward value carried, outputs written in place;
//   stop when every check's full XOR LLR b[0] is > 0 (c_ldpc.c:191-197).
// Every node performs the reference's operations in the reference's order,
// so results differ from the reference C build only through last-ulp
// differences between ROCm's and glibc's exp/log.  The path is bound by fp64
// transcendental throughput (3(dc-2)+... Lxor per check, 2 exp + 2 log each),
// not by memory: the only HBM traffic per iteration is ch and app.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "ldpc_bp.h"

#pragma clang fp contract(off)

#define LB_VERSION "ldpc_bp 0.1 gfx950"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                            \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess)                                                        \
      return fail(LB_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

constexpr int kMaxThreads = 1024;
constexpr size_t kLdsBytes = 160 * 1024;

// ---------------------------------------------------------------------------
// Node rules
// ---------------------------------------------------------------------------
// Lxor (c_ldpc.c:234-251): sign product times min |.|, plus the two
// log(1+exp(-|.|)) corrections for the exact sum-product rule.  Symmetric in
// its arguments, bit for bit.
//
// The logarithm's argument is 1 + exp(-|x|), in [1, 2]: log12 evaluates it in
// the structure of fdlibm's e_log.c (u = 2^k m, m in [sqrt(2)/2, sqrt(2)],
// f = m - 1 exact, s = f / (2 + f), log(1 + f) = f - hfsq + s (hfsq + R(s^2)),
// |error| < 1 ulp) instead of ROCm's general log, whose double-double steps
// cost 46 of the 224 instructions of an Lxor: the check kernels are bound by
// this arithmetic.  Against glibc's log on the arguments Lxor produces (u = 1
// + exp(-x), x in [0, 40], 2e7 samples) 0.51 % of the results differ, by one
// ulp, never more (the reference's own build differs from ROCm's log by last
// ulps as well).  -DLB_OCML_LOG restores ROCm's log.
__host__ __device__ __forceinline__ double log12(double u) {
#ifdef LB_OCML_LOG
  return log(u);
#else
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  // branch-free: k = 0 gives 0 - ((hfsq - (s (hfsq + R) + 0)) - f), which is
  // e_log.c's f - (hfsq - s (hfsq + R)) bit for bit (f = m - 1 is never -0)
  const double k = u > 1.41421356237309504880 ? 1.0 : 0.0;
  const double m = u * (1.0 - 0.5 * k);
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return k * ln2_hi - ((hfsq - (s * (hfsq + R) + k * ln2_lo)) - f);
#endif
}

template <bool CORR>
__device__ __forceinline__ double lxor(double a, double b) {
  double L = (signbit(a) == signbit(b)) ? 1.0 : -1.0;
  L *= fmin(fabs(a), fabs(b));
  if (CORR) {
    L += log12(1.0 + exp(-fabs(a + b)));
    L -= log12(1.0 + exp(-fabs(a - b)));
  }
  return L;
}

// Lxfb (c_ldpc.c:294-314) in place on one check node's dc messages:
// f[k] = Lxor(f[k-1], L[k]); b[k] = Lxor(b[k+1], L[k]);
// out[0] = b[1], out[dc-1] = f[dc-2], out[k] = Lxor(f[k-1], b[k+1]).
// f stays in registers (unrolled to DCMAX with guards); b is carried down.
// Returns b[0], the LLR of the XOR of all inputs (stopping rule).
template <int DCMAX, bool CORR, typename P>
__device__ __forceinline__ double lxfb(P L, int dc) {
  double f[DCMAX];
  f[0] = L[0];
#pragma unroll
  for (int k = 1; k < DCMAX; ++k)
    if (k < dc) f[k] = lxor<CORR>(f[k - 1], L[k]);
  double b = 0.0;
#pragma unroll
  for (int k = DCMAX - 1; k >= 1; --k) {
    if (k == dc - 1) {
      b = L[k];
      L[k] = f[k - 1];
    } else if (k < dc - 1) {
      const double lk = L[k];
      L[k] = lxor<CORR>(f[k - 1], b);
      b = lxor<CORR>(b, lk);
    }
  }
  const double l0 = L[0];
  L[0] = b;
  return lxor<CORR>(b, l0);
}

// Lxfb for checks of exactly DC edges (a check-regular code, e.g. 802.16
// rate 5/6: dc = 20 everywhere), in the reference's own loop structure
// (c_ldpc.c:294-314): the forward chain f[k] = Lxor(f[k-1], L[k]) and the
// backward chain b[k] = Lxor(b[k+1], L[k]) run side by side, then every
// output Lxor(f[k-1], b[k+1]) at once.  Straight-line code (no degree
// guards), so the two dependent chains interleave: the critical path is
// dc - 1 Lxor latencies plus one, against 2 (dc - 2) in lxfb's
// forward-then-backward form.  The same operations on the same operands:
// bit-identical to lxfb.
template <int DC, bool CORR>
__device__ __forceinline__ double lxfb_fixed_regs(const double (&l)[DC], double (&o)[DC]) {
  static_assert(DC >= 3, "fixed-degree checks");
  double f[DC - 1], b[DC];
  f[0] = l[0];
  b[DC - 1] = l[DC - 1];
#pragma unroll
  for (int k = 1; k < DC; ++k) {
    if (k < DC - 1) f[k] = lxor<CORR>(f[k - 1], l[k]);  // f[DC-1] is never used
    b[DC - 1 - k] = lxor<CORR>(b[DC - k], l[DC - 1 - k]);
  }
  o[0] = b[1];
  o[DC - 1] = f[DC - 2];
#pragma unroll
  for (int k = 1; k < DC - 1; ++k) o[k] = lxor<CORR>(f[k - 1], b[k + 1]);
  return b[0];  // = Lxor(b[1], L[0]), lxfb's return value
}

template <int DC, bool CORR>
__device__ __forceinline__ double lxfb_fixed(double* L) {
  double l[DC], o[DC];
#pragma unroll
  for (int k = 0; k < DC; ++k) l[k] = L[k];
  const double r = lxfb_fixed_regs<DC, CORR>(l, o);
#pragma unroll
  for (int k = 0; k < DC; ++k) L[k] = o[k];
  return r;
}

// One check node's rule on its dc messages at L (in place): the reference's
// three decoders.  Returns whether the check is unsatisfied (the stopping rule).
template <int ALGO, int DCMAX, int DCFIX, typename P>
__device__ __forceinline__ bool check_rule(P L, int dc, double corr) {
  bool bad;
  if (ALGO == LB_SUMPROD) {  // c_ldpc.c:76-102
    double aggr = 1.0;
    for (int k = 0; k < dc; ++k) {
      const double t = tanh(L[k] / 2.0);
      L[k] = t;
      aggr *= t;
    }
    bad = 2.0 * atanh(aggr) <= 0.0;
    for (int k = 0; k < dc; ++k) L[k] = 2.0 * atanh(aggr / L[k]);
  } else if (ALGO == LB_SUMPROD2) {  // c_ldpc.c:183-194
    if constexpr (DCFIX > 0) bad = lxfb_fixed<DCFIX, true>(L) <= 0.0;
    else bad = lxfb<DCMAX, true>(L, dc) <= 0.0;
  } else {  // minsum, c_ldpc.c:364-372 with node-aligned offsets
    if constexpr (DCFIX > 0) bad = lxfb_fixed<DCFIX, false>(L) <= 0.0;
    else bad = lxfb<DCMAX, false>(L, dc) <= 0.0;
    for (int k = 0; k < dc; ++k) L[k] *= corr;
  }
  return bad;
}

struct BpArgs {
  const double* ch;    // [B][Nv]
  double* app;         // [B][Nv]
  int* iters;          // [B]
  double* gmsg;        // [B][Nmsg] when the messages do not fit in LDS
  const int* vedge;    // [maxdv][Nv] message index of port k of variable node j
  const uint8_t* vdeg; // [Nv]
  const int* cstart;   // [Nc+1] first message of each check node
  int Nv, Nc, Nmsg, maxit;
  double corr;
  // hand-off to the tail kernels (tail != 0): a word not converged after
  // maxit iterations leaves its messages in gmsg and its index in active[]
  int tail;
  int* active;   // [B]
  int* nactive;  // [1]
  int* done;     // [B]
  int* lastbad;  // [2][B]: iteration stamp of the last unsatisfied check, by parity
  int B;
};

// DCFIX > 0: every check node has exactly DCFIX edges (lxfb_fixed; launched
// with at most kFixThreads threads, so a thread may hold the two chains in
// registers: 3 waves per SIMD)
constexpr int kFixThreads = 768;
template <int ALGO, int DCMAX, bool LDSM, int DCFIX = 0>
__global__ void __launch_bounds__(DCFIX > 0 ? kFixThreads : kMaxThreads) k_bp(BpArgs a) {
  extern __shared__ double lds_msg[];
  __shared__ int unsat[2];
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* msg = LDSM ? lds_msg : a.gmsg + (size_t)b * a.Nmsg;
  const double* ch = a.ch + (size_t)b * a.Nv;
  double* app = a.app + (size_t)b * a.Nv;
  const int Nv = a.Nv, Nc = a.Nc;

  for (int i = tid; i < a.Nmsg; i += nt) msg[i] = 0.0;  // calloc (c_ldpc.c:164)
  if (tid < 2) unsat[tid] = 0;
  __syncthreads();

  int it = 0;
  for (; it < a.maxit; ++it) {
    // variable nodes (c_ldpc.c:171-178)
    for (int j = tid; j < Nv; j += nt) {
      const int d = a.vdeg[j];
      double aggr = ch[j];
      for (int k = 0; k < d; ++k) aggr += msg[a.vedge[(size_t)k * Nv + j]];
      for (int k = 0; k < d; ++k) {
        const int e = a.vedge[(size_t)k * Nv + j];
        msg[e] = aggr - msg[e];
      }
      app[j] = aggr;
    }
    // unsat[it & 1] was last read in iteration it-2; the barriers of it-1 order that read first
    if (tid == 0) unsat[it & 1] = 0;
    __syncthreads();
    // check nodes
    for (int c = tid; c < Nc; c += nt) {
      const int s = a.cstart[c], dc = a.cstart[c + 1] - s;
      const bool bad = check_rule<ALGO, DCMAX, DCFIX>(msg + s, dc, a.corr);
      if (bad) unsat[it & 1] = 1;
    }
    __syncthreads();
    if (!unsat[it & 1]) break;  // c_ldpc.c:196-197
  }
  if (a.tail && it == a.maxit) {
    // not converged in the first maxit iterations: the messages go to the
    // word's slice of gmsg (already there without LDS) for k_bp_tail
    if (LDSM) {
      double* g = a.gmsg + (size_t)b * a.Nmsg;
      for (int i = tid; i < a.Nmsg; i += nt) g[i] = msg[i];
    }
    if (tid == 0) {
      a.active[atomicAdd(a.nactive, 1)] = b;
      a.done[b] = 0;
      a.lastbad[((it - 1) & 1) * a.B + b] = it - 1;  // iteration it-1 left a check unsatisfied
      a.lastbad[(it & 1) * a.B + b] = -1;            // no stale stamp from an earlier decode
    }
  } else if (tid == 0) {
    a.iters[b] = it;
  }
}

// ---------------------------------------------------------------------------
// Tail: the iterations after the first `tail_at`, for the words still running
// ---------------------------------------------------------------------------
// One workgroup holds one word's whole decode above, so the words that do not
// converge (at the joint simulator's operating point a fifth of them run to
// max_iter) leave most of the chip idle while the launch waits for them: each
// iteration is a fixed ~75 us of one CU's binary64 VALU.  From iteration
// tail_at on, the words still running are spread over the chip, two launches
// per iteration, messages in HBM in two slots (read r_{t-1}, write r_t):
//   k_bp_tail_var: thread per variable node, ch + incoming messages in port
//     order (c_ldpc.c:171-178) -> app[v] (the aggregate itself);
//   k_bp_tail_chk: S workgroups per word, thread per check node, input
//     app[v(e)] - r_{t-1}[e] (the reference's extrinsic, the same subtraction)
//     and the check rule of k_bp.
// Bit-identical to running the whole decode in k_bp.
//
// Two ways to size the tail.  Sized on the host (lb_decode, which blocks
// anyway): one 4-byte read-back gives the number n of words still running
// after tail_at iterations, the grids cover exactly those words, and the host
// stops issuing iterations once a read-back shows every word done.  Sized on
// the device (lb_run / lb_decode_device, which must not block the caller):
// every iteration up to max_iter is queued behind the first phase with grids
// sized from an estimate of n; each kernel reads n and the done count from
// device memory, strides over the words the estimate did not cover, and
// returns at once when every word is done.  Same kernels, same arithmetic in
// the same order: the two are bit-identical.
struct TailArgs {
  const double* ch;      // [B][Nv]
  double* app;           // [B][Nv]
  int* iters;            // [B]
  const double* rold;    // [B][Nmsg] check-to-variable messages of iteration it-1
  double* rnew;          // [B][Nmsg] ... of iteration it
  const int* vedge;      // [maxdv][Nv]
  const uint8_t* vdeg;   // [Nv]
  const int* evar;       // [Nmsg] variable node of each edge
  const int* cstart;     // [Nc+1]
  const int* active;     // [n] words still running
  int* done;             // [B]
  int* ndone;            // [1] words detected as done in the tail (the stop test)
  const int* nactive;    // [1] words entering the tail (device-sized mode)
  int* lastbad;          // [2][B]
  int Nv, Nc, Nmsg, B, n, S, it;
  int dyn;               // 1: n and the stop test from device memory
  double corr;
};

// words still running in this tail launch; 0 when every word is done
__device__ __forceinline__ int tail_words(const TailArgs& a) {
  if (!a.dyn) return a.n;
  const int n = *a.nactive;
  return *a.ndone >= n ? 0 : n;
}

// DV >= the largest variable degree (4, 8 or 12): every port's table entry
// and message loaded at once, summed in port order with exact selects
template <int DV>
__global__ void __launch_bounds__(256) k_bp_tail_var(TailArgs a) {
  const int n = tail_words(a);
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  for (int wi = blockIdx.y; wi < n; wi += gridDim.y) {
    const int w = a.active[wi];
    if (a.done[w]) continue;  // converged in an earlier iteration
    if (a.lastbad[((a.it - 1) & 1) * a.B + w] != a.it - 1) {
      // iteration it-1 satisfied every check (c_ldpc.c:196-197): it is the word's last
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.iters[w] = a.it - 1;
        a.done[w] = 1;
        atomicAdd(a.ndone, 1);
      }
      continue;
    }
    if (j >= a.Nv) continue;
    const double* rold = a.rold + (size_t)w * a.Nmsg;
    const int d = a.vdeg[j];
    int e[DV];
#pragma unroll
    for (int k = 0; k < DV; ++k) e[k] = a.vedge[(size_t)(k < d ? k : 0) * a.Nv + j];
    double x[DV];
#pragma unroll
    for (int k = 0; k < DV; ++k) x[k] = rold[e[k]];
    double aggr = a.ch[(size_t)w * a.Nv + j];
#pragma unroll
    for (int k = 0; k < DV; ++k)
      if (k < d) aggr += x[k];
    a.app[(size_t)w * a.Nv + j] = aggr;
  }
}

// the value of the other lane of an even/odd lane pair (DPP quad_perm [1,0,3,2])
__device__ __forceinline__ double swap_pair(double x) {
  const unsigned long long u = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, 0xB1, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), 0xB1, 0xF, 0xF, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

constexpr int kTailFixThreads = 256, kTailThreads = 128;
template <int ALGO, int DCMAX, int DCFIX>
__global__ void __launch_bounds__(DCFIX > 0 ? kTailFixThreads : kTailThreads) k_bp_tail_chk(TailArgs a) {
  constexpr int ROW = DCMAX + 1;
  __shared__ double rows[DCFIX > 0 ? 1 : kTailThreads * ROW];
  const int n = tail_words(a);
  const int cpw = (a.Nc + a.S - 1) / a.S;
  for (int item = blockIdx.x; item < n * a.S; item += gridDim.x) {
    const int wi = item / a.S, slice = item % a.S;
    const int w = a.active[wi];
    if (a.done[w]) continue;
    const double* rold = a.rold + (size_t)w * a.Nmsg;
    double* rnew = a.rnew + (size_t)w * a.Nmsg;
    const double* app = a.app + (size_t)w * a.Nv;
    const int c0 = slice * cpw, c1 = min(a.Nc, c0 + cpw);
    bool anybad = false;
    if constexpr (DCFIX > 0) {
      // two lanes per check: lane p = 0 runs the forward chain f, lane p = 1
      // the backward chain b (its inputs in reverse order), in one instruction
      // stream; then each takes half of the outputs Lxor(f[k-1], b[k+1]) with
      // the partner's chain values swapped in (DPP).  The same Lxor calls on
      // the same operands in the same order as lxfb_fixed_regs: bit-identical.
      static_assert(DCFIX == 20, "the output split below is written for dc = 20");
      const int p = threadIdx.x & 1;
      for (int c = c0 + ((int)threadIdx.x >> 1); c < c1; c += blockDim.x >> 1) {
        const int s = c * DCFIX;  // check-regular: cstart[c] = c * DCFIX
        int ev[DCFIX];
        double r[DCFIX], l[DCFIX];
#pragma unroll
        for (int k = 0; k < DCFIX; ++k) {
          const int e = s + (p ? DCFIX - 1 - k : k);
          ev[k] = a.evar[e];
          r[k] = rold[e];
        }
#pragma unroll
        for (int k = 0; k < DCFIX; ++k) l[k] = app[ev[k]] - r[k];  // lane 1: l in reverse order
        constexpr bool CORR = ALGO == LB_SUMPROD2;
        double g[DCFIX];  // lane 0: g[i] = f[i]; lane 1: g[i] = b[DC-1-i]
        g[0] = l[0];
#pragma unroll
        for (int i = 1; i < DCFIX; ++i) g[i] = lxor<CORR>(g[i - 1], l[i]);
        double pg[9];  // the partner's g[9..17]
#pragma unroll
        for (int i = 0; i < 9; ++i) pg[i] = swap_pair(g[9 + i]);
        double o[10];
        o[0] = g[18];  // lane 0: o[19] = f[18]; lane 1: o[0] = b[1]
#pragma unroll
        for (int i = 0; i < 9; ++i) {
          // lane 0: k = 1 + i, f[k-1] = g[i], b[k+1] = partner g[17-i]
          // lane 1: k = 10 + i, f[k-1] = partner g[9+i], b[k+1] = g[8-i]
          const double fa = p ? pg[i] : g[i];
          const double bb = p ? g[8 - i] : pg[8 - i];
          o[1 + i] = lxor<CORR>(fa, bb);
        }
        if (ALGO != LB_SUMPROD2) {
#pragma unroll
          for (int i = 0; i < 10; ++i) o[i] *= a.corr;
        }
        rnew[s + (p ? 0 : DCFIX - 1)] = o[0];
#pragma unroll
        for (int i = 0; i < 9; ++i) rnew[s + (p ? 10 : 1) + i] = o[1 + i];
        anybad |= p && g[DCFIX - 1] <= 0.0;  // b[0]: lxfb's return value
      }
    } else {
      for (int c = c0 + (int)threadIdx.x; c < c1; c += blockDim.x) {
        const int s = a.cstart[c], dc = a.cstart[c + 1] - s;
        double* L = rows + threadIdx.x * ROW;
        for (int k = 0; k < dc; ++k) L[k] = app[a.evar[s + k]] - rold[s + k];
        anybad |= check_rule<ALGO, DCMAX, 0>(L, dc, a.corr);
        for (int k = 0; k < dc; ++k) rnew[s + k] = L[k];
      }
    }
    if (anybad) a.lastbad[(a.it & 1) * a.B + w] = a.it;
  }
}

// after the last tail iteration: the iteration count of the words that ran to
// the end (max_iter, or max_iter - 1 when the last iteration converged)
__global__ void k_bp_tail_end(int* iters, const int* active, const int* nactive, const int* done,
                              const int* lastbad, int B, int maxit) {
  const int n = *nactive;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int w = active[i];
    if (!done[w]) iters[w] = lastbad[((maxit - 1) & 1) * B + w] == maxit - 1 ? maxit : maxit - 1;
  }
}

__global__ void k_lxor(double a, double b, int corr, double* out) {
  out[0] = corr ? lxor<true>(a, b) : lxor<false>(a, b);
}

__global__ void k_lxfb(double* L, int dc, int corr, double* out) {
  out[0] = corr ? lxfb<32, true>(L, dc) : lxfb<32, false>(L, dc);
}

using KernelFn = void (*)(BpArgs);

template <int ALGO, bool LDSM>
KernelFn pick_dc(int maxdc) {
  if (maxdc <= 8) return k_bp<ALGO, 8, LDSM>;
  if (maxdc <= 16) return k_bp<ALGO, 16, LDSM>;
  return k_bp<ALGO, 32, LDSM>;
}

// check-regular codes whose degree has a straight-line instance (lxfb_fixed)
bool fixed_dc(int mindc, int maxdc, int nt) { return mindc == maxdc && maxdc == 20 && nt <= kFixThreads; }

KernelFn pick_kernel(int algo, int maxdc, bool lds, bool fixed = false) {
  if (fixed && algo == LB_SUMPROD2) return lds ? k_bp<LB_SUMPROD2, 32, true, 20> : k_bp<LB_SUMPROD2, 32, false, 20>;
  if (fixed && algo == LB_MINSUM) return lds ? k_bp<LB_MINSUM, 32, true, 20> : k_bp<LB_MINSUM, 32, false, 20>;
  // sumprod does not use the register-resident forward values: one instance suffices
  switch (algo) {
    case LB_SUMPROD2: return lds ? pick_dc<LB_SUMPROD2, true>(maxdc) : pick_dc<LB_SUMPROD2, false>(maxdc);
    case LB_SUMPROD: return lds ? k_bp<LB_SUMPROD, 8, true> : k_bp<LB_SUMPROD, 8, false>;
    default: return lds ? pick_dc<LB_MINSUM, true>(maxdc) : pick_dc<LB_MINSUM, false>(maxdc);
  }
}

using TailFn = void (*)(TailArgs);

template <int ALGO>
TailFn pick_tail_dc(int maxdc) {
  if (maxdc <= 8) return k_bp_tail_chk<ALGO, 8, 0>;
  if (maxdc <= 16) return k_bp_tail_chk<ALGO, 16, 0>;
  return k_bp_tail_chk<ALGO, 32, 0>;
}

TailFn pick_tail(int algo, int maxdc, bool fixed) {
  if (fixed && algo == LB_SUMPROD2) return k_bp_tail_chk<LB_SUMPROD2, 32, 20>;
  if (fixed && algo == LB_MINSUM) return k_bp_tail_chk<LB_MINSUM, 32, 20>;
  switch (algo) {
    case LB_SUMPROD2: return pick_tail_dc<LB_SUMPROD2>(maxdc);
    case LB_SUMPROD: return pick_tail_dc<LB_SUMPROD>(maxdc);
    default: return pick_tail_dc<LB_MINSUM>(maxdc);
  }
}

TailFn pick_tail_var(int nq) {
  return nq == 1 ? k_bp_tail_var<4> : (nq == 2 ? k_bp_tail_var<8> : k_bp_tail_var<12>);
}

// first iteration of the tail launches (0: off); LDPC_BP_TAIL overrides
constexpr int kTailAt = 8;
constexpr int kTailChunk = 8;  // tail iterations per stop test

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int default_device() {
  const char* e = getenv("LDPC_BP_DEVICE");
  if (!e || !*e) e = getenv("LOCAL_RANK");
  return (e && *e) ? atoi(e) : 0;
}

}  // namespace

struct lb_ctx {
  int dev = 0, Nv = 0, Nc = 0, Nmsg = 0, maxdv = 0, maxdc = 0, mindc = 0, nt = 0;
  bool fixed = false;  // check-regular with a straight-line check kernel (lxfb_fixed)
  bool lds = false;
  // tail launches (k_bp_tail): edge tables, per-word state, first tail iteration
  int tail_at = 0, nq = 0, ncu = 256;
  int* d_evar = nullptr;
  int *d_active = nullptr, *d_nact = nullptr, *d_done = nullptr, *d_lastbad = nullptr;
  int* h_nact = nullptr;  // pinned: [0] words entering the tail, [1..2] done counts of the last chunks,
                        // [3] the last device-sized tail's words
  hipEvent_t evc[2] = {nullptr, nullptr};
  hipEvent_t evn = nullptr;   // device-sized tails: its word count has landed in h_nact[0]
  bool est_pending = false;   // a device-sized tail's word count is in flight
  int est_n = 0, est_B = 0, est_Bq = 0;  // the last landed count and its batch; the batch in flight
  int capTailB = 0;
  int tail_default = 0;       // tail_at chosen at lb_create (kTailAt or LDPC_BP_TAIL)
  int* d_vedge = nullptr;
  uint8_t* d_vdeg = nullptr;
  int* d_cstart = nullptr;
  double *d_ch = nullptr, *d_app = nullptr, *d_msg = nullptr;
  int* d_it = nullptr;
  int capB = 0, capMsgB = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool attrs_set = false;
};

namespace {

void release(lb_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  (void)hipFree(c->d_vedge);
  (void)hipFree(c->d_vdeg);
  (void)hipFree(c->d_cstart);
  (void)hipFree(c->d_ch);
  (void)hipFree(c->d_app);
  (void)hipFree(c->d_msg);
  (void)hipFree(c->d_it);
  (void)hipFree(c->d_evar);
  (void)hipFree(c->d_active);
  (void)hipFree(c->d_nact);
  (void)hipFree(c->d_done);
  (void)hipFree(c->d_lastbad);
  if (c->h_nact) (void)hipHostFree(c->h_nact);
  for (hipEvent_t e : c->evc)
    if (e) (void)hipEventDestroy(e);
  if (c->evn) (void)hipEventDestroy(c->evn);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int dev_alloc(void** p, size_t bytes) {
  if (hipMalloc(p, bytes) != hipSuccess) {
    *p = nullptr;
    return fail(LB_ERR_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
  }
  return LB_OK;
}

int ensure_io(lb_ctx* c, int B) {
  if (B <= c->capB) return LB_OK;
  (void)hipFree(c->d_ch);
  (void)hipFree(c->d_app);
  (void)hipFree(c->d_it);
  c->d_ch = c->d_app = nullptr;
  c->d_it = nullptr;
  c->capB = 0;
  int rc;
  if ((rc = dev_alloc((void**)&c->d_ch, (size_t)B * c->Nv * sizeof(double)))) return rc;
  if ((rc = dev_alloc((void**)&c->d_app, (size_t)B * c->Nv * sizeof(double)))) return rc;
  if ((rc = dev_alloc((void**)&c->d_it, (size_t)B * sizeof(int)))) return rc;
  c->capB = B;
  return LB_OK;
}

// message slices: one per word without LDS, two per word (r_{t-1}, r_t)
// for the tail launches; capMsgB counts word slices
int ensure_msg(lb_ctx* c, int B, bool tail) {
  const int need = tail ? 2 * B : (c->lds ? 0 : B);
  if (need <= c->capMsgB) return LB_OK;
  (void)hipFree(c->d_msg);
  c->d_msg = nullptr;
  c->capMsgB = 0;
  int rc;
  if ((rc = dev_alloc((void**)&c->d_msg, (size_t)need * c->Nmsg * sizeof(double)))) return rc;
  c->capMsgB = need;
  return LB_OK;
}

int ensure_tail(lb_ctx* c, int B) {
  if (B <= c->capTailB) return LB_OK;
  (void)hipFree(c->d_active);
  (void)hipFree(c->d_done);
  (void)hipFree(c->d_lastbad);
  c->d_active = c->d_done = c->d_lastbad = nullptr;
  c->capTailB = 0;
  int rc;
  if ((rc = dev_alloc((void**)&c->d_active, (size_t)B * sizeof(int)))) return rc;
  if ((rc = dev_alloc((void**)&c->d_done, (size_t)B * sizeof(int)))) return rc;
  if ((rc = dev_alloc((void**)&c->d_lastbad, (size_t)2 * B * sizeof(int)))) return rc;
  if (!c->d_nact && (rc = dev_alloc((void**)&c->d_nact, 2 * sizeof(int)))) return rc;
  for (hipEvent_t* e : {&c->evc[0], &c->evc[1], &c->evn})
    if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
      *e = nullptr;
      return fail(LB_ERR_HIP, "hipEventCreate failed");
    }
  if (!c->h_nact && hipHostMalloc((void**)&c->h_nact, 4 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
    c->h_nact = nullptr;
    return fail(LB_ERR_NOMEM, "hipHostMalloc failed");
  }
  c->capTailB = B;
  return LB_OK;
}

int set_attrs(lb_ctx* c) {
  if (c->attrs_set || !c->lds) return LB_OK;
  const size_t bytes = (size_t)c->Nmsg * sizeof(double);
  for (int algo = 0; algo < 3; ++algo)
    HIP_TRY(hipFuncSetAttribute((const void*)pick_kernel(algo, c->maxdc, true, c->fixed),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  c->attrs_set = true;
  return LB_OK;
}

// sized_on_host: the tail's shape from the number of words still running
// (one read-back; the caller blocks anyway), else sized on the device and
// queued without waiting (see TailArgs)
int launch(lb_ctx* c, int B, const double* d_ch, double* d_app, int* d_it, int algo, double corr,
           int max_iter, bool sized_on_host) {
  if (algo < LB_SUMPROD2 || algo > LB_MINSUM) return fail(LB_ERR_ARG, "unknown decoder type");
  if (max_iter < 0) return fail(LB_ERR_ARG, "max_iter < 0");
  if (B == 0) return LB_OK;
  // the tail's variable kernel puts the words on the grid's y dimension (<= 65535)
  const bool tail = c->tail_at > 0 && max_iter > c->tail_at && B <= 65535;
  int rc;
  if ((rc = ensure_msg(c, B, tail))) return rc;
  if ((rc = set_attrs(c))) return rc;
  if (tail && (rc = ensure_tail(c, B))) return rc;
  BpArgs a;
  a.ch = d_ch;
  a.app = d_app;
  a.iters = d_it;
  a.gmsg = c->d_msg;
  a.vedge = c->d_vedge;
  a.vdeg = c->d_vdeg;
  a.cstart = c->d_cstart;
  a.Nv = c->Nv;
  a.Nc = c->Nc;
  a.Nmsg = c->Nmsg;
  a.maxit = tail ? c->tail_at : max_iter;
  a.corr = corr;
  a.tail = tail ? 1 : 0;
  a.active = c->d_active;
  a.nactive = c->d_nact;
  a.done = c->d_done;
  a.lastbad = c->d_lastbad;
  a.B = B;
  // the previous device-sized tail's word count, if it has landed: the estimate
  // the next device-sized tail's grids are sized for
  if (c->est_pending && hipEventQuery(c->evn) == hipSuccess) {
    c->est_n = c->h_nact[3];
    c->est_B = c->est_Bq;
    c->est_pending = false;
  }
  if (tail) HIP_TRY(hipMemsetAsync(c->d_nact, 0, 2 * sizeof(int), c->stream));  // nactive, ndone
  const size_t shm = c->lds ? (size_t)c->Nmsg * sizeof(double) : 0;
  hipLaunchKernelGGL(pick_kernel(algo, c->maxdc, c->lds, c->fixed), dim3(B), dim3(c->nt), shm, c->stream, a);
  HIP_TRY(hipGetLastError());
  if (!tail) return LB_OK;

  int n = B;
  if (sized_on_host) {
    // how many words are left decides the tail's shape (one 4-byte read-back)
    HIP_TRY(hipMemcpyAsync(c->h_nact, c->d_nact, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    n = *c->h_nact;
    if (n < 0 || n > B) return fail(LB_ERR_HIP, "tail word count out of range");
    if (n == 0) return LB_OK;
  }
  // the words the grids are sized for: exact, or the last device-sized tail's
  // share of its batch applied to this one (a quarter before any), with slack
  int nsz = n;
  if (!sized_on_host) {
    const double share = c->est_B > 0 ? (double)c->est_n / c->est_B : 0.25;
    nsz = std::min(B, std::max(8, (int)std::ceil(share * B * 1.25)));
  }
  // m waves per workgroup so that the words' waves (one thread per check)
  // cover the SIMDs once: S = ceil(Nc / 64m) workgroups per word
  // the straight-line check rule runs on lane pairs (32 checks per wave)
  const bool split = c->fixed && algo != LB_SUMPROD;
  const long waves = (long)nsz * ((c->Nc + (split ? 31 : 63)) / (split ? 32 : 64));
  const int mmax = c->fixed && algo != LB_SUMPROD ? kTailFixThreads / 64 : kTailThreads / 64;
  int m = (int)((waves + 4L * c->ncu - 1) / (4L * c->ncu));
  m = m < 1 ? 1 : (m > mmax ? mmax : m);
  const int cpt = split ? 32 : 64;  // checks per wave
  const int S = (c->Nc + cpt * m - 1) / (cpt * m);
  TailArgs t;
  t.ch = d_ch;
  t.app = d_app;
  t.iters = d_it;
  t.vedge = c->d_vedge;
  t.vdeg = c->d_vdeg;
  t.evar = c->d_evar;
  t.cstart = c->d_cstart;
  t.active = c->d_active;
  t.done = c->d_done;
  t.ndone = c->d_nact + 1;
  t.nactive = c->d_nact;
  t.lastbad = c->d_lastbad;
  t.Nv = c->Nv;
  t.Nc = c->Nc;
  t.Nmsg = c->Nmsg;
  t.B = B;
  t.n = n;
  t.S = S;
  t.dyn = sized_on_host ? 0 : 1;
  t.corr = corr;
  double* slot[2] = {c->d_msg, c->d_msg + (size_t)B * c->Nmsg};
  const TailFn chk = pick_tail(algo, c->maxdc, split);
  const TailFn var = pick_tail_var(c->nq);
  const dim3 vgrid((c->Nv + 255) / 256, nsz);
  const dim3 cgrid((unsigned)nsz * S);
  if (!sized_on_host) {
    // every iteration queued; a launch past the last running word returns at once
    for (int it = c->tail_at; it < max_iter; ++it) {
      t.rold = slot[(it - c->tail_at) & 1];
      t.rnew = slot[(it - c->tail_at + 1) & 1];
      t.it = it;
      hipLaunchKernelGGL(var, vgrid, dim3(256), 0, c->stream, t);
      hipLaunchKernelGGL(chk, cgrid, dim3(64 * m), 0, c->stream, t);
    }
    // this tail's word count, for the next one's estimate (read when it has landed)
    HIP_TRY(hipMemcpyAsync(c->h_nact + 3, c->d_nact, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->evn, c->stream));
    c->est_pending = true;
    c->est_Bq = B;
  } else {
    // chunks of kTailChunk iterations; after each, the count of words found
    // done is copied back, and the host stops issuing chunks once the copy of
    // two chunks ago shows every word done (the GPU keeps the latest chunk
    // meanwhile: no stall while words run, no empty launches to max_iter after)
    for (int it0 = c->tail_at, k = 0; it0 < max_iter; it0 += kTailChunk, ++k) {
      if (k >= 2) {
        HIP_TRY(hipEventSynchronize(c->evc[k & 1]));
        if (c->h_nact[1 + (k & 1)] >= n) break;
      }
      for (int it = it0; it < std::min(max_iter, it0 + kTailChunk); ++it) {
        t.rold = slot[(it - c->tail_at) & 1];
        t.rnew = slot[(it - c->tail_at + 1) & 1];
        t.it = it;
        hipLaunchKernelGGL(var, vgrid, dim3(256), 0, c->stream, t);
        hipLaunchKernelGGL(chk, cgrid, dim3(64 * m), 0, c->stream, t);
      }
      HIP_TRY(hipMemcpyAsync(c->h_nact + 1 + (k & 1), c->d_nact + 1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipEventRecord(c->evc[k & 1], c->stream));
    }
  }
  hipLaunchKernelGGL(k_bp_tail_end, dim3((nsz + 255) / 256), dim3(256), 0, c->stream, d_it, c->d_active, c->d_nact,
                     c->d_done, c->d_lastbad, B, max_iter);
  HIP_TRY(hipGetLastError());
  return LB_OK;
}

// Graph cache for the reference-signature entry points (one decode per call,
// the graph identical across calls in the reference's harness).
struct CacheKey {
  int Nv, Nc, Nmsg, dev;
  uint64_t h;
  bool operator<(const CacheKey& o) const {
    return std::tie(Nv, Nc, Nmsg, dev, h) < std::tie(o.Nv, o.Nc, o.Nmsg, o.dev, o.h);
  }
};
std::mutex g_cache_mu;
std::map<CacheKey, lb_ctx*> g_cache;

uint64_t fnv(uint64_t h, const long* p, int n) {
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)p[i];
    h *= 1099511628211ull;
  }
  return h;
}

int cached_ctx(long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg, lb_ctx** out) {
  if (!vdeg || !cdeg || !intrlv || Nv <= 0 || Nc <= 0 || Nmsg <= 0) return fail(LB_ERR_ARG, "null graph");
  const int dev = default_device();
  uint64_t h = 1469598103934665603ull;
  h = fnv(h, vdeg, Nv);
  h = fnv(h, cdeg, Nc);
  h = fnv(h, intrlv, Nmsg);
  const CacheKey k{Nv, Nc, Nmsg, dev, h};
  std::lock_guard<std::mutex> g(g_cache_mu);
  auto it = g_cache.find(k);
  if (it != g_cache.end()) {
    *out = it->second;
    return LB_OK;
  }
  if (g_cache.size() >= 16) {  // bounded: drop everything (a harness uses one or two codes)
    for (auto& kv : g_cache) release(kv.second);
    g_cache.clear();
  }
  lb_ctx* c = nullptr;
  const int rc = lb_create(&c, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, dev);
  if (rc) return rc;
  g_cache[k] = c;
  *out = c;
  return LB_OK;
}

int ref_decode(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg, double* app,
               int algo, double corr) {
  if (!ch || !app) return fail(LB_ERR_ARG, "null ch/app");
  lb_ctx* c = nullptr;
  int rc = cached_ctx(vdeg, cdeg, intrlv, Nv, Nc, Nmsg, &c);
  if (rc) return rc;
  int it = 0;
  rc = lb_decode(c, 1, ch, app, &it, algo, corr, LB_MAX_ITCOUNT);
  return rc ? rc : it;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* lb_last_error(void) { return g_err.c_str(); }
const char* lb_version(void) { return LB_VERSION; }
int lb_device_count(void) { return device_count(); }

int lb_create(lb_ctx** out, const long* vdeg, const long* cdeg, const long* intrlv, int Nv, int Nc,
              int Nmsg, int device) {
  if (!out) return fail(LB_ERR_ARG, "out is null");
  *out = nullptr;
  if (!vdeg || !cdeg || !intrlv || Nv <= 0 || Nc <= 0 || Nmsg <= 0)
    return fail(LB_ERR_ARG, "empty or null graph");
  // host-side validation (the reference trusts its own prepare_decoder)
  long sv = 0, sc = 0;
  int maxdv = 0, maxdc = 0, mindc = 1 << 30;
  for (int j = 0; j < Nv; ++j) {
    if (vdeg[j] < 0) return fail(LB_ERR_GRAPH, "negative variable degree");
    sv += vdeg[j];
    maxdv = vdeg[j] > maxdv ? (int)vdeg[j] : maxdv;
  }
  for (int j = 0; j < Nc; ++j) {
    if (cdeg[j] < 1) return fail(LB_ERR_GRAPH, "check node of degree < 1");
    sc += cdeg[j];
    maxdc = cdeg[j] > maxdc ? (int)cdeg[j] : maxdc;
    mindc = cdeg[j] < mindc ? (int)cdeg[j] : mindc;
  }
  if (sv != Nmsg || sc != Nmsg) return fail(LB_ERR_GRAPH, "sum(vdeg) and sum(cdeg) must equal Nmsg");
  if (maxdc > 32) return fail(LB_ERR_UNSUPPORTED, "check degree > 32");
  if (maxdv > 255) return fail(LB_ERR_UNSUPPORTED, "variable degree > 255");
  std::vector<char> seen(Nmsg, 0);
  for (int i = 0; i < Nmsg; ++i) {
    if (intrlv[i] < 0 || intrlv[i] >= Nmsg || seen[intrlv[i]]) return fail(LB_ERR_GRAPH, "intrlv is not a permutation");
    seen[intrlv[i]] = 1;
  }
  const int ndev = device_count();
  if (ndev == 0) return fail(LB_ERR_NO_DEVICE, "no HIP device visible (there is no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(LB_ERR_ARG, "device index out of range");

  std::vector<int> vedge((size_t)std::max(maxdv, 1) * Nv, 0);
  std::vector<uint8_t> vd(Nv);
  std::vector<int> cs(Nc + 1);
  long p = 0;
  for (int j = 0; j < Nv; ++j) {
    vd[j] = (uint8_t)vdeg[j];
    for (int k = 0; k < vdeg[j]; ++k) vedge[(size_t)k * Nv + j] = (int)intrlv[p++];
  }
  cs[0] = 0;
  for (int j = 0; j < Nc; ++j) cs[j + 1] = cs[j] + (int)cdeg[j];
  // tail edge table: the variable node of each edge
  const int nq = maxdv <= 12 ? std::max(1, (maxdv + 3) / 4) : 0;
  std::vector<int> evar;
  if (nq) {
    evar.resize(Nmsg);
    long q = 0;
    for (int j = 0; j < Nv; ++j)
      for (int k = 0; k < vdeg[j]; ++k) evar[intrlv[q++]] = j;
  }

  lb_ctx* c = new lb_ctx;
  c->dev = device;
  c->Nv = Nv;
  c->Nc = Nc;
  c->Nmsg = Nmsg;
  c->maxdv = maxdv;
  c->maxdc = maxdc;
  c->lds = (size_t)Nmsg * sizeof(double) <= kLdsBytes - 64;
  // one thread per check node when possible (the check phase dominates)
  c->nt = std::min(kMaxThreads, std::max(256, (Nc + 63) / 64 * 64));
  c->mindc = mindc;
  c->fixed = fixed_dc(mindc, maxdc, c->nt);
  c->nq = nq;
  c->tail_at = 0;
  if (c->nq) {
    const char* e = getenv("LDPC_BP_TAIL");
    c->tail_at = (e && *e) ? std::max(0, atoi(e)) : kTailAt;
  }
  c->tail_default = c->tail_at;
  int rc = LB_OK;
  auto bail = [&](int r) { release(c); return r; };
  if (hipSetDevice(device) != hipSuccess) return bail(fail(LB_ERR_HIP, "hipSetDevice failed"));
  if ((rc = dev_alloc((void**)&c->d_vedge, vedge.size() * sizeof(int)))) return bail(rc);
  if ((rc = dev_alloc((void**)&c->d_vdeg, (size_t)Nv))) return bail(rc);
  if ((rc = dev_alloc((void**)&c->d_cstart, (size_t)(Nc + 1) * sizeof(int)))) return bail(rc);
  if (c->nq && (rc = dev_alloc((void**)&c->d_evar, evar.size() * sizeof(int)))) return bail(rc);
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) c->ncu = ncu;
  }
  // (the stream at the device's highest priority, and the tail's waves at the
  // highest issue priority, measured slower / neutral beside a pipelined joint
  // batch's AMP stream, rounds 4-5: default priorities)
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess)
    return bail(fail(LB_ERR_HIP, "stream/event creation failed"));
  // uploads on the context's non-blocking stream, waited for (a pageable
  // hipMemcpy may return before its DMA lands, unordered with this stream)
  if (hipMemcpyAsync(c->d_vedge, vedge.data(), vedge.size() * sizeof(int), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(c->d_vdeg, vd.data(), (size_t)Nv, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(c->d_cstart, cs.data(), (size_t)(Nc + 1) * sizeof(int), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      (c->nq && hipMemcpyAsync(c->d_evar, evar.data(), evar.size() * sizeof(int), hipMemcpyHostToDevice, c->stream) != hipSuccess) ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return bail(fail(LB_ERR_HIP, "graph upload failed"));
  *out = c;
  return LB_OK;
}

void lb_destroy(lb_ctx* ctx) { release(ctx); }

int lb_decode(lb_ctx* c, int B, const double* ch, double* app, int* iters, int algo, double corr_factor,
              int max_iter) {
  if (!c) return fail(LB_ERR_ARG, "null context");
  if (B < 0 || (B > 0 && (!ch || !app || !iters))) return fail(LB_ERR_ARG, "bad batch arguments");
  if (B == 0) return LB_OK;
  HIP_TRY(hipSetDevice(c->dev));
  int rc;
  if ((rc = ensure_io(c, B))) return rc;
  const size_t bytes = (size_t)B * c->Nv * sizeof(double);
  HIP_TRY(hipMemcpyAsync(c->d_ch, ch, bytes, hipMemcpyHostToDevice, c->stream));
  if ((rc = launch(c, B, c->d_ch, c->d_app, c->d_it, algo, corr_factor, max_iter, true))) return rc;
  HIP_TRY(hipMemcpyAsync(app, c->d_app, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(iters, c->d_it, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LB_OK;
}

int lb_decode_device(lb_ctx* c, int B, const double* d_ch, double* d_app, int* d_iters, int algo,
                     double corr_factor, int max_iter) {
  if (!c) return fail(LB_ERR_ARG, "null context");
  if (B < 0 || (B > 0 && (!d_ch || !d_app || !d_iters))) return fail(LB_ERR_ARG, "bad batch arguments");
  HIP_TRY(hipSetDevice(c->dev));
  return launch(c, B, d_ch, d_app, d_iters, algo, corr_factor, max_iter, false);
}

int lb_buffers(lb_ctx* c, int B, double** d_ch, double** d_app, int** d_iters) {
  if (!c || B <= 0) return fail(LB_ERR_ARG, "bad buffer request");
  HIP_TRY(hipSetDevice(c->dev));
  int rc;
  if ((rc = ensure_io(c, B))) return rc;
  if (d_ch) *d_ch = c->d_ch;
  if (d_app) *d_app = c->d_app;
  if (d_iters) *d_iters = c->d_it;
  return LB_OK;
}

int lb_stage(lb_ctx* c, int B, const double* ch) {
  if (!c || B <= 0 || !ch) return fail(LB_ERR_ARG, "bad stage arguments");
  HIP_TRY(hipSetDevice(c->dev));
  int rc;
  if ((rc = ensure_io(c, B))) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_ch, ch, (size_t)B * c->Nv * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LB_OK;
}

int lb_run(lb_ctx* c, int B, int algo, double corr_factor, int max_iter) {
  if (!c || B <= 0 || B > c->capB) return fail(LB_ERR_ARG, "run before stage, or B larger than staged");
  HIP_TRY(hipSetDevice(c->dev));
  HIP_TRY(hipEventRecord(c->ev0, c->stream));
  int rc = launch(c, B, c->d_ch, c->d_app, c->d_it, algo, corr_factor, max_iter, false);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->ev1, c->stream));
  return LB_OK;
}

int lb_wait(lb_ctx* c) {
  if (!c) return fail(LB_ERR_ARG, "null context");
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LB_OK;
}

int lb_fetch(lb_ctx* c, int B, double* app, int* iters) {
  if (!c || B <= 0 || B > c->capB) return fail(LB_ERR_ARG, "bad fetch arguments");
  HIP_TRY(hipSetDevice(c->dev));
  if (app) HIP_TRY(hipMemcpyAsync(app, c->d_app, (size_t)B * c->Nv * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (iters) HIP_TRY(hipMemcpyAsync(iters, c->d_it, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LB_OK;
}

double lb_run_event_ms(lb_ctx* c) {
  if (!c) return -1.0;
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.0;
  return ms;
}

int lb_info(lb_ctx* c, long long* out) {
  if (!c || !out) return fail(LB_ERR_ARG, "null argument");
  out[0] = c->Nv;
  out[1] = c->Nc;
  out[2] = c->Nmsg;
  out[3] = c->maxdv;
  out[4] = c->maxdc;
  out[5] = c->lds ? 1 : 0;
  out[6] = c->nt;
  out[7] = c->dev;
  out[8] = c->fixed ? c->maxdc : 0;
  out[9] = c->tail_at;
  return LB_OK;
}

int lb_set_tail(lb_ctx* c, int tail_at) {
  if (!c) return fail(LB_ERR_ARG, "null context");
  if (tail_at > 0 && !c->nq) return fail(LB_ERR_UNSUPPORTED, "tail launches need variable degrees <= 12");
  c->tail_at = tail_at < 0 ? c->tail_default : tail_at;
  return LB_OK;
}

int sumprod(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg, double* app) {
  return ref_decode(ch, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, app, LB_SUMPROD, 0.0);
}

int sumprod2(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg, double* app) {
  return ref_decode(ch, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, app, LB_SUMPROD2, 0.0);
}

int minsum(double* ch, long* vdeg, long* cdeg, long* intrlv, int Nv, int Nc, int Nmsg, double* app,
           double correction_factor) {
  return ref_decode(ch, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, app, LB_MINSUM, correction_factor);
}

static double scalar_kernel(int which, double a, double b, double* L, long dc, int corr) {
  const double nan = std::nan("");
  if (device_count() == 0) {
    fail(LB_ERR_NO_DEVICE, "no HIP device visible (there is no CPU fallback)");
    return nan;
  }
  if (which == 1 && (!L || dc < 1 || dc > 32)) {
    fail(LB_ERR_ARG, "Lxfb needs 1 <= dc <= 32");
    return nan;
  }
  if (hipSetDevice(default_device()) != hipSuccess) return nan;
  double* d = nullptr;
  if (hipMalloc((void**)&d, (33 + (size_t)(which == 1 ? dc : 0)) * sizeof(double)) != hipSuccess) {
    fail(LB_ERR_NOMEM, "hipMalloc failed");
    return nan;
  }
  double r = nan;
  bool ok = true;
  if (which == 0) {
    hipLaunchKernelGGL(k_lxor, dim3(1), dim3(1), 0, 0, a, b, corr, d);
  } else {
    ok = hipMemcpy(d + 1, L, (size_t)dc * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    if (ok) hipLaunchKernelGGL(k_lxfb, dim3(1), dim3(1), 0, 0, d + 1, (int)dc, corr, d);
  }
  ok = ok && hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
       hipMemcpy(&r, d, sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
  if (ok && which == 1) ok = hipMemcpy(L, d + 1, (size_t)dc * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  if (!ok) {
    fail(LB_ERR_HIP, "scalar kernel failed");
    return nan;
  }
  return r;
}

double Lxor(double L1, double L2, int corr_flag) { return scalar_kernel(0, L1, L2, nullptr, 0, corr_flag); }

double Lxfb(double* L, long dc, int corr_flag) { return scalar_kernel(1, 0, 0, L, dc, corr_flag); }

}  // extern "C"
