// sa_mc.hip — the Monte-Carlo rep stream of BASELINE configs[3] (the reps
// loop of amp_test.py:183-246 and the BER sweeps of sparc_ldpc.py:1217-1245,
// 1318-1323) on one device:
//
//  * sa_draw_reps: the seeded synthetic reps of harness._draw_reps on the host
//    cores — rep s draws RandomState(s).randint(0, M, L) then .randn(n) —
//    restated natively (MT19937 with its integer seeding, the masked bounded
//    integers and the polar Gaussian of NumPy's legacy RandomState), bit for
//    bit the same values, over several threads;
//  * sa_mc_stage / sa_mc_run: the staged reps decoded through a batch of B
//    slots with per-slot refill.  Every slot carries its own iteration index
//    (SecArgs::tb / RowArgs::tb); when a slot's exact-tau stop fires
//    (sparc_ldpc.py:204) or its T iterations are done, its section decisions
//    are taken and the next rep is encoded into it (y = A beta(idx) + noise,
//    beta = 0, z = y) inside the same captured iteration, so the batch stays
//    full instead of running until its slowest codeword stops.  A codeword's
//    decode does not depend on its slot or its neighbours, so every rep's
//    decisions and stop index equal those of the batched decode (sa_run).
#include "sa_host.h"

#include <thread>

namespace sa {

// ---- NumPy legacy RandomState, restated ------------------------------------
// (numpy/random: mt19937_seed, mt19937_next32 / next_double,
// buffered_bounded_masked_uint32, legacy_gauss; the published MT19937 of
// Matsumoto & Nishimura.)  Plain IEEE binary64 operations in NumPy's order
// and the C library's log / sqrt, no contraction: the same bits.
struct LegacyMT {
  uint32_t key[624];
  int pos = 624;
  bool has_gauss = false;
  double gauss = 0.0;

  explicit LegacyMT(uint32_t seed) {
    key[0] = seed;
    for (int i = 1; i < 624; ++i) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + (uint32_t)i;
  }
  void twist() {
    constexpr uint32_t U = 0x80000000u, Lo = 0x7fffffffu, A = 0x9908b0dfu;
    int i = 0;
    for (; i < 624 - 397; ++i) {
      const uint32_t y = (key[i] & U) | (key[i + 1] & Lo);
      key[i] = key[i + 397] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    for (; i < 623; ++i) {
      const uint32_t y = (key[i] & U) | (key[i + 1] & Lo);
      key[i] = key[i + 397 - 624] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    const uint32_t y = (key[623] & U) | (key[0] & Lo);
    key[623] = key[396] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    pos = 0;
  }
  uint32_t next32() {
    if (pos == 624) twist();
    uint32_t y = key[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double next_double() {
#pragma clang fp contract(off)
    const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
  // randint(0, M) of the legacy generator: the smallest all-ones mask over
  // M - 1, rejection of the masked 32-bit draws above M - 1
  int32_t bounded(uint32_t rng) {
    if (rng == 0) return 0;  // no draw
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = next32() & mask) > rng) {
    }
    return (int32_t)v;
  }
  double gaussian() {  // legacy_gauss: the polar method, the second value kept
#pragma clang fp contract(off)
    if (has_gauss) {
      has_gauss = false;
      const double t = gauss;
      gauss = 0.0;
      return t;
    }
    double x1, x2, r2;
    do {
      x1 = 2.0 * next_double() - 1.0;
      x2 = 2.0 * next_double() - 1.0;
      r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    gauss = f * x1;
    has_gauss = true;
    return f * x2;
  }
};

// ---- device side --------------------------------------------------------------

// the slot arrays of the refilled batch (sa_ctx::d_slots, slot_cap entries each)
struct McArgs {
  int* rep;    // rep decoded in the slot, -1: empty
  int* tb;     // the slot's iteration index t_b (SecArgs::tb), -1: empty
  int* done;   // rep whose decode finished in this iteration (its decisions are due), -1: none
  int* fresh;  // 1: the slot took a new rep in this iteration (beta = 0, y, z = y, z^2 partials)
  int* fin_list;    // the slots that finished in this iteration, in slot order (ctl[3] of them)
  int* fresh_list;  // the slots that took a new rep, in slot order (ctl[4] of them; the first of fin_list)
  int* ctl;    // {next rep, live slots, reps, finished, refilled}
  int* iters;  // [B] stop index of the slot's decode (k_secb), -1 running
  int32_t* dec;          // [reps][L] decisions
  int32_t* its;          // [reps] stop index, T when the loop ran out
  int32_t* errs;         // [reps] bit errors: sum over sections of popcount(decision ^ index)
  const int32_t* idx;    // [reps][L] section indices
  const double* noise;   // [reps][n]
  int B, T, L, M, n, NZ;
};

constexpr int kMcStepThreads = 1024;  // slots of one k_mc_step workgroup

// After an iteration's section and row kernels: every slot whose stop fired
// (iters >= 0) or whose T iterations are done finishes (its stop index goes
// to its rep's slot in `its`), the others move to t_b + 1; the finished slots
// take the next reps in slot order (a workgroup-wide exclusive scan) or empty.
__global__ void __launch_bounds__(kMcStepThreads) k_mc_step(McArgs a) {
  __shared__ int sc[kMcStepThreads];
  __shared__ int s_next;
  const int b = threadIdx.x;
  if (b == 0) s_next = a.ctl[0];
  int fin = 0, rep = -1;
  if (b < a.B) {
    rep = a.rep[b];
    if (rep >= 0) {
      const int it = a.iters[b], t = a.tb[b];
      if (it >= 0 || t + 1 >= a.T) {
        fin = 1;
        a.its[rep] = it >= 0 ? it : a.T;
      } else {
        a.tb[b] = t + 1;
      }
    }
    a.done[b] = fin ? rep : -1;
  }
  sc[b] = fin;
  __syncthreads();
  for (int off = 1; off < kMcStepThreads; off <<= 1) {  // inclusive scan
    const int v = b >= off ? sc[b - off] : 0;
    __syncthreads();
    sc[b] += v;
    __syncthreads();
  }
  const int next = s_next, total = sc[kMcStepThreads - 1], nreps = a.ctl[2];
  int live = 0;
  if (b < a.B) {
    int fr = 0;
    if (fin) {
      const int r = next + sc[b] - 1;
      if (r < nreps) {
        a.rep[b] = r;
        a.tb[b] = 0;
        a.iters[b] = -1;
        fr = 1;
      } else {
        a.rep[b] = -1;
        a.tb[b] = -1;
      }
    }
    a.fresh[b] = fr;
    if (fin) a.fin_list[sc[b] - 1] = b;
    if (fr) a.fresh_list[sc[b] - 1] = b;  // the refilled are the first nreps - next finished
    live = (fin ? fr : rep >= 0) ? 1 : 0;
  }
  __syncthreads();  // every thread has read s_next / sc
  sc[b] = live;
  __syncthreads();
  for (int off = kMcStepThreads / 2; off > 0; off >>= 1) {
    if (b < off) sc[b] += sc[b + off];
    __syncthreads();
  }
  if (b == 0) {
    const int nf = next + total < nreps ? total : nreps - next;
    a.ctl[0] = next + nf;
    a.ctl[1] = sc[0];
    a.ctl[3] = total;
    a.ctl[4] = nf;
  }
}

// One wave per (section, finished slot), grid-stride over the slots that
// finished in this iteration: the section decision (k_decide's argmax) into
// the rep's row of dec and its bit errors against the sent index (popcount of
// the xor, sparc_ldpc.py:462) added to the rep's count; then, where the slot
// took a new rep, the section zeroed (beta = 0, the zero start of
// sparc_ldpc.py:193-200).
template <typename real, int E>
__device__ __forceinline__ void mc_turnover_blocks(const McArgs& a, real* beta, int blk, int nblk) {
  const int lane = threadIdx.x & 63;
  const int nfin = a.ctl[3], G4 = (a.L + 3) / 4;
  for (int item = blk; item < nfin * G4; item += nblk) {
    const int b = a.fin_list[item / G4], l = (item % G4) * 4 + (threadIdx.x >> 6);
    if (l >= a.L) continue;
    const int done = a.done[b];
    real* bl = beta + ((size_t)b * a.L + l) * a.M;
    const int bi = section_argmax<real, E>(bl, lane, a.M);
    if (lane == 0) {
      a.dec[(size_t)done * a.L + l] = bi;
      const int e = __popc((unsigned)(bi ^ a.idx[(size_t)done * a.L + l]));
      if (e) atomicAdd(a.errs + done, e);
    }
    if (a.fresh[b]) {
#pragma unroll
      for (int i = 0; i < E; ++i) {
        const int e = elem_index<E>(lane, i);
        if (e < a.M) bl[e] = (real)0;
      }
    }
  }
}

// Every staged rep's channel output and start, before the stream runs (the
// whole batch of encodes fills the chip; inside the stream's iterations a few
// refills at a time did not).  Workgroup = one 128-row block of k_rowc x
// kFillSlots reps, one wave per 64-row half, a lane per row carrying the
// kFillSlots reps' sums side by side (one Ab-table read serves all of them;
// the reps' section indices are workgroup-uniform scalar loads):
// y = A beta(idx) + noise with sa_encode's arithmetic (k_colsum: the binary64
// sum of +-c_l over the sections in order, / sqrt(n), + noise, one rounding to
// `real`) and the block's z^2 partial exactly as k_rowc's zero start forms it
// (y0 y0 + y1 y1 for rows lane and 64 + lane, then the wave sum).  A refilled
// slot copies them (k_mc_turnover's refill blocks): its state then equals a fresh batched
// decode's after its ROW_INIT0 step.
constexpr int kFillSlots = 4;

template <typename real>
__global__ void __launch_bounds__(128) k_mc_encode(McArgs a, int nreps, const ushort4* __restrict__ fwd,
                                                   const double* __restrict__ cd, double sqrt_n,
                                                   real* __restrict__ y_all, real* __restrict__ zzp_all) {
  __shared__ real yh[kFillSlots][64];  // the second half's y, for the first half's z^2 partial
  const int j0 = blockIdx.y * kFillSlots;
  const int cnt = nreps - j0 < kFillSlots ? nreps - j0 : kFillSlots;
  const int lane = threadIdx.x & 63, half = threadIdx.x >> 6, n = a.n, L = a.L;
  const int r = blockIdx.x * 128 + half * 64 + lane;
  // the kFillSlots reps' section indices: uniform over the workgroup (scalar loads)
  const int32_t* ib = a.idx + (size_t)j0 * L;
  real yv[kFillSlots];
#pragma unroll
  for (int j = 0; j < kFillSlots; ++j) yv[j] = 0;
  if (r < n) {
    // kFillSlots independent sums per lane (one per rep), each in section order
    double acc[kFillSlots];
#pragma unroll
    for (int j = 0; j < kFillSlots; ++j) acc[j] = 0.0;
    const int G4 = (L + kSpw - 1) / kSpw;
    // the row's Ab-table entries kFillAhead groups at a time, the next block's
    // loads in flight while this block's sums run
    constexpr int kFillAhead = 16;
    const ushort4* fr = fwd + r;
    ushort4 cur[kFillAhead], nxt[kFillAhead];
#pragma unroll
    for (int u = 0; u < kFillAhead; ++u) cur[u] = fr[(size_t)(u < G4 ? u : 0) * n];
    // per rep, its row of section indices (uniform: scalar loads at constant
    // offsets from a base advanced once per block)
    const int32_t* rows[kFillSlots];
#pragma unroll
    for (int j = 0; j < kFillSlots; ++j) rows[j] = ib + (size_t)(j < cnt ? j : 0) * L;
    for (int g0 = 0; g0 < G4; g0 += kFillAhead) {
#pragma unroll
      for (int u = 0; u < kFillAhead; ++u) {
        const int gn = g0 + kFillAhead + u;
        nxt[u] = fr[(size_t)(gn < G4 ? gn : 0) * n];
      }
      const double* cb = cd + (size_t)g0 * kSpw;
      const int32_t* rb[kFillSlots];
#pragma unroll
      for (int j = 0; j < kFillSlots; ++j) rb[j] = rows[j] + (size_t)g0 * kSpw;
#pragma unroll
      for (int u = 0; u < kFillAhead; ++u) {
        const unsigned short fq[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int o = u * kSpw + q;
          if ((g0 * kSpw) + o < L) {  // (uniform; no early exit, so that the block stays unrolled)
            const unsigned kk = fq[q] & 0x7fffu;
            // +-c_l as its bits: the row's sign (sg) folded into the high word once,
            // each rep's parity bit xored into it (exactly -c or c, as a select would give)
            const unsigned long long cbits = (unsigned long long)__double_as_longlong(cb[o]);
            const unsigned chi = (unsigned)(cbits >> 32) ^ ((unsigned)(fq[q] >> 15) << 31);
            const unsigned clo = (unsigned)cbits;
#pragma unroll
            for (int j = 0; j < kFillSlots; ++j) {
              const unsigned par = (unsigned)__popc(kk & (unsigned)rb[j][o]) << 31;
              acc[j] += __longlong_as_double((long long)(((unsigned long long)(chi ^ par) << 32) | clo));
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kFillAhead; ++u) cur[u] = nxt[u];
    }
#pragma unroll
    for (int j = 0; j < kFillSlots; ++j) {
      if (j < cnt) {
        const double x = acc[j] / sqrt_n;
        yv[j] = (real)(x + a.noise[(size_t)(j0 + j) * n + r]);
        y_all[(size_t)(j0 + j) * n + r] = yv[j];
      }
    }
  }
  if (half == 1) {
#pragma unroll
    for (int j = 0; j < kFillSlots; ++j) yh[j][lane] = yv[j];
  }
  __syncthreads();
  if (half == 0) {
#pragma unroll
    for (int j = 0; j < kFillSlots; ++j) {
      if (j >= cnt) break;
      // k_rowc: q = 0; q += z0 z0 (row lane); q += z1 z1 (row 64 + lane), rows past n skipped
      real q = 0;
      if (r < n) q += yv[j] * yv[j];
      const real y1 = yh[j][lane];
      if (r + 64 < n) q += y1 * y1;
      const real sz = wave_sum(q);
      if (lane == 0) zzp_all[(size_t)(j0 + j) * a.NZ + blockIdx.x] = sz;
    }
  }
}

// A refilled slot takes its rep's encoded y and z^2 partials (k_mc_encode):
// y, z = y in the codeword-interleaved layout, the partials; grid-stride over
// the refilled slots' rows.
template <typename real, int CB>
__device__ __forceinline__ void mc_fill_blocks(const McArgs& a, const real* __restrict__ y_all,
                                               const real* __restrict__ zzp_all, real* __restrict__ y,
                                               real* __restrict__ z, real* __restrict__ zzp, int blk, int nblk) {
  const int nf = a.ctl[4], n = a.n, NZ = a.NZ;
  const long long tot = (long long)nf * n;
  for (long long i = blk * 256LL + threadIdx.x; i < tot; i += (long long)nblk * 256) {
    const int slot = a.fresh_list[i / n], r = (int)(i % n);
    const int rep = a.rep[slot];
    const real yv = y_all[(size_t)rep * n + r];
    y[(size_t)slot * n + r] = yv;
    z[((size_t)(slot / CB) * n + r) * CB + (slot % CB)] = yv;
    if (r < NZ) zzp[(size_t)slot * NZ + r] = zzp_all[(size_t)rep * NZ + r];
  }
}

// The turnover and the refill copy in one launch (independent work behind
// k_mc_step): blocks [0, gto) run the turnover items, the rest the copy.
template <typename real, int E, int CB>
__global__ void __launch_bounds__(256) k_mc_turnover(McArgs a, real* beta, int gto, const real* __restrict__ y_all,
                                                     const real* __restrict__ zzp_all, real* __restrict__ y,
                                                     real* __restrict__ z, real* __restrict__ zzp) {
  if ((int)blockIdx.x < gto) mc_turnover_blocks<real, E>(a, beta, blockIdx.x, gto);
  else mc_fill_blocks<real, CB>(a, y_all, zzp_all, y, z, zzp, blockIdx.x - gto, gridDim.x - gto);
}

// ---- host side ------------------------------------------------------------------

namespace {

McArgs mc_args(sa_ctx* c, int B, int T) {
  McArgs a;
  const int S = c->slot_cap;
  a.rep = c->d_slots; a.tb = c->d_slots + S; a.done = c->d_slots + 2 * S; a.fresh = c->d_slots + 3 * S;
  a.fin_list = c->d_slots + 4 * S; a.fresh_list = c->d_slots + 5 * S;
  a.ctl = c->d_slots + 6 * S;
  a.iters = c->d_iters;
  a.dec = c->d_mc_dec; a.its = c->d_mc_its; a.errs = c->d_mc_its + c->mc_cap; a.idx = c->d_mc_idx;
  a.noise = c->d_mc_noise;
  a.B = B; a.T = T; a.L = c->L; a.M = c->M; a.n = c->n; a.NZ = c->NZ2;
  return a;
}

// the refill of the slots flagged fresh: decisions of the finished, beta = 0,
// y / z / z^2 partials of the new reps
template <typename real>
int mc_turnover(sa_ctx* c, const McArgs& a) {
  const int gto = std::min(2048, a.B * ((c->L + 3) / 4));
  const int gfill = std::min(4096, (a.B * c->n + 255) / 256);
  constexpr int CBz = 16 / (int)sizeof(real);
  const real* ya = (const real*)c->d_mc_y;
  const real* za = (const real*)c->d_mc_zzp;
  switch (c->E) {
#define SA_TO(EE)                                                                                             \
  case EE:                                                                                                    \
    k_mc_turnover<real, EE, CBz><<<gto + gfill, 256, 0, c->stream>>>(a, (real*)c->d_beta, gto, ya, za,        \
                                                                     (real*)c->d_y, (real*)c->d_z,            \
                                                                     (real*)c->d_zzp);                        \
    break;
    SA_TO(1) SA_TO(2) SA_TO(4) SA_TO(8) SA_TO(16)
#undef SA_TO
    default: return fail(SA_ERR_UNSUPPORTED, "sa_mc_run: M > 1024");
  }
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

// every staged rep's y and z^2 partials (k_mc_encode)
template <typename real>
int mc_encode_all(sa_ctx* c, const McArgs& a, int nreps) {
  k_mc_encode<real><<<dim3(c->NZ2, (nreps + kFillSlots - 1) / kFillSlots), 128, 0, c->stream>>>(a, nreps, (const ushort4*)c->d_fwd, c->d_cd, std::sqrt((double)c->n),
                                   (real*)c->d_mc_y, (real*)c->d_mc_zzp);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

// K iterations of the refilled batch: section kernel, row kernel, slot step,
// turnover (all on the context's stream, captured once per (B, T, K, flags))
template <typename real>
int mc_iterations(sa_ctx* c, int B, int T, int K, int es) {
  const McArgs a = mc_args(c, B, T);
  c->mc_tb = a.tb;
  int rc = SA_OK;
  for (int k = 0; k < K && !rc; ++k) {
    if ((rc = launch_secb<real>(c, B, 0, es))) break;
    if ((rc = launch_row<real>(c, B, ROW_AMP, 0, es, c->Gb, c->Gb))) break;
    k_mc_step<<<1, kMcStepThreads, 0, c->stream>>>(a);
    if ((rc = mc_turnover<real>(c, a))) break;
  }
  c->mc_tb = nullptr;
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

int mc_ensure_slots(sa_ctx* c, int B) {
  if (c->slot_cap >= B) return SA_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto& kv : c->mc_graphs) (void)hipGraphExecDestroy(kv.second);
  c->mc_graphs.clear();
  dev_free(c->d_slots);
  c->d_slots = nullptr;
  c->slot_cap = 0;
  if (int rc = dev_alloc(c, (void**)&c->d_slots, (6 * (size_t)B + 8) * sizeof(int))) return rc;
  c->slot_cap = B;
  return SA_OK;
}

}  // namespace

// (the stream's kernels use at most 64 KB of LDS: nothing to raise)
hipError_t mc_lds_attrs() { return hipSuccess; }

void mc_release(sa_ctx* c) {
  for (auto& kv : c->mc_graphs) (void)hipGraphExecDestroy(kv.second);
  c->mc_graphs.clear();
  dev_free(c->d_mc_idx); dev_free(c->d_mc_noise); dev_free(c->d_mc_dec); dev_free(c->d_mc_its);
  dev_free(c->d_mc_y); dev_free(c->d_mc_zzp);
  c->d_mc_y = c->d_mc_zzp = nullptr;
  dev_free(c->d_slots);
  c->d_mc_idx = c->d_mc_dec = c->d_mc_its = nullptr;
  c->d_mc_noise = nullptr;
  c->d_slots = nullptr;
  c->mc_cap = c->mc_nreps = c->slot_cap = 0;
  if (c->h_mc_live) (void)hipHostFree(c->h_mc_live);
  c->h_mc_live = nullptr;
  for (auto& e : c->mc_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->mc_ev) e = nullptr;
}

}  // namespace sa

using namespace sa;

extern "C" {

int sa_draw_reps(const uint32_t* seeds, int count, int L, int M, int n, double sigma, int32_t* idx_out,
                 double* noise_out, int threads) {
  if (count < 0 || L <= 0 || M <= 0 || n < 0 || (count > 0 && (!seeds || !idx_out || (n > 0 && !noise_out))))
    return fail(SA_ERR_ARG, "sa_draw_reps: bad arguments");
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min(nt, std::max(1, count)));
  auto work = [&](int t0) {
    for (int i = t0; i < count; i += nt) {
      LegacyMT mt(seeds[i]);
      int32_t* ix = idx_out + (size_t)i * L;
      for (int l = 0; l < L; ++l) ix[l] = mt.bounded((uint32_t)(M - 1));
      double* nz = noise_out + (size_t)i * n;
      for (int r = 0; r < n; ++r) nz[r] = mt.gaussian();
      for (int r = 0; r < n; ++r) nz[r] = nz[r] * sigma;  // noise *= sigma
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  return SA_OK;
}

int sa_make_ordering(int L, int M, int n, uint32_t seed, uint32_t* out) {
  // sparc_ldpc.py:107-117: RandomState(seed), one cumulative shuffle of
  // arange(1, w) per section, the first n kept.  NumPy's 1-d shuffle swaps
  // x[i] with x[random_interval(i)] for i = w - 2 .. 1 (masked 32-bit draws)
  if (L <= 0 || M <= 0 || n <= 0 || !out) return fail(SA_ERR_ARG, "sa_make_ordering: bad arguments");
  const int mx = (M + 1) > (n + 1) ? (M + 1) : (n + 1);
  const long long w = 1LL << ilog2(mx);
  if (w > (1LL << 30)) return fail(SA_ERR_UNSUPPORTED, "sa_make_ordering: w too large");
  std::vector<uint32_t> x((size_t)w - 1);
  for (long long i = 0; i < w - 1; ++i) x[i] = (uint32_t)(i + 1);
  LegacyMT mt(seed);
  for (int l = 0; l < L; ++l) {
    for (long long i = w - 2; i >= 1; --i) {
      const uint32_t j = (uint32_t)mt.bounded((uint32_t)i);
      std::swap(x[i], x[j]);
    }
    std::memcpy(out + (size_t)l * n, x.data(), (size_t)n * sizeof(uint32_t));
  }
  return SA_OK;
}

int sa_mc_stage(sa_ctx* c, int nreps, const int32_t* idx, const double* noise) {
  if (check_tables(c, "sa_mc_stage")) return SA_ERR_UNSUPPORTED;
  if (nreps <= 0 || !idx || !noise) return fail(SA_ERR_ARG, "sa_mc_stage: bad arguments");
  for (size_t i = 0; i < (size_t)nreps * c->L; ++i)
    if (idx[i] < 0 || idx[i] >= c->M) return fail(SA_ERR_ARG, "sa_mc_stage: index outside [0, M)");
  HIP_TRY(hipSetDevice(c->device));
  if (nreps > c->mc_cap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    dev_free(c->d_mc_idx); dev_free(c->d_mc_noise); dev_free(c->d_mc_dec); dev_free(c->d_mc_its);
    dev_free(c->d_mc_y); dev_free(c->d_mc_zzp);
    c->d_mc_idx = c->d_mc_dec = c->d_mc_its = nullptr;
    c->d_mc_noise = nullptr;
    c->d_mc_y = c->d_mc_zzp = nullptr;
    c->mc_cap = 0;
    for (auto& kv : c->mc_graphs) (void)hipGraphExecDestroy(kv.second);  // they hold the old pointers
    c->mc_graphs.clear();
    int rc;
    if ((rc = dev_alloc(c, (void**)&c->d_mc_idx, (size_t)nreps * c->L * sizeof(int32_t)))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_mc_dec, (size_t)nreps * c->L * sizeof(int32_t)))) return rc;
    // stop indices, then the bit errors
    if ((rc = dev_alloc(c, (void**)&c->d_mc_its, 2 * (size_t)nreps * sizeof(int32_t)))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_mc_noise, (size_t)nreps * c->n * sizeof(double)))) return rc;
    // the encoded reps (k_mc_encode): y [nreps][n] and z^2 partials [nreps][NZ2], in the context precision
    if ((rc = dev_alloc(c, &c->d_mc_y, (size_t)nreps * c->n * rsz(c)))) return rc;
    if ((rc = dev_alloc(c, &c->d_mc_zzp, (size_t)nreps * c->NZ2 * rsz(c)))) return rc;
    c->mc_cap = nreps;
  }
  HIP_TRY(hipMemcpyAsync(c->d_mc_idx, idx, (size_t)nreps * c->L * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_mc_noise, noise, (size_t)nreps * c->n * sizeof(double), hipMemcpyHostToDevice,
                         c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->mc_nreps = nreps;
  return SA_OK;
}

int sa_mc_run(sa_ctx* c, int B, int T, int flags, int32_t* dec_out, int32_t* iters_out, int32_t* errs_out,
              double* ms_out) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B < 4 || B > kMcStepThreads || T <= 0) return fail(SA_ERR_ARG, "sa_mc_run: B in [4, 1024], T > 0");
  if (c->mc_nreps <= 0) return fail(SA_ERR_ARG, "sa_mc_run: no reps staged (sa_mc_stage)");
  if (!c->shared_power || c->pb_on) return fail(SA_ERR_ARG, "sa_mc_run: one power allocation must be staged");
  if (c->backend != SA_BACKEND_HADAMARD || !c->pow2 || c->big || !zil_for(c, B))
    return fail(SA_ERR_UNSUPPORTED, "sa_mc_run: needs the batched codeword-interleaved Hadamard decode "
                                    "(k_secb + k_rowc)");
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_workspace(c, B, T))) return rc;
  if ((rc = ensure_invb(c))) return rc;
  if ((rc = mc_ensure_slots(c, B))) return rc;
  if (!c->h_mc_live) {
    HIP_TRY(hipHostMalloc((void**)&c->h_mc_live, 4 * sizeof(int), hipHostMallocDefault));
    for (auto& e : c->mc_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const int es = (flags & SA_FLAG_NO_EARLY_STOP) ? 0 : 1;
  const bool f64 = c->prec == SA_PREC_F64;
  const int nreps = c->mc_nreps;
  pick_row(c, B);
  c->zil_last = true;
  // the slots' start: the first min(B, reps) reps in slots 0.., the rest
  // empty; every slot's estimate zero (the turnover zeroes a refilled slot's
  // later), the first reps' y / z / z^2 partials by the fill kernel
  {
    const int S = c->slot_cap, n0 = std::min(B, nreps);
    std::vector<int> h(6 * (size_t)S + 8, -1);
    for (int b = 0; b < S; ++b) {
      const bool on = b < n0;
      h[b] = on ? b : -1;                 // rep
      h[S + b] = on ? 0 : -1;             // t_b
      h[2 * (size_t)S + b] = -1;          // done
      h[3 * (size_t)S + b] = on ? 1 : 0;  // fresh
      h[5 * (size_t)S + b] = b;           // fresh_list (the first n0 entries)
    }
    int* ctl = h.data() + 6 * (size_t)S;
    ctl[0] = n0;      // next rep
    ctl[1] = n0;      // live slots
    ctl[2] = nreps;
    ctl[3] = 0;       // finished (none yet)
    ctl[4] = n0;      // refilled
    HIP_TRY(hipMemcpyAsync(c->d_slots, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(c->d_beta, 0, (size_t)B * c->L * c->M * rsz(c), c->stream));
    k_fill32<<<(B + 255) / 256, 256, 0, c->stream>>>((uint32_t*)c->d_iters, 0xffffffffu, (size_t)B);
    k_fill32<<<(nreps + 255) / 256, 256, 0, c->stream>>>((uint32_t*)(c->d_mc_its + c->mc_cap), 0u, (size_t)nreps);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));  // h is a host temporary
  }
  HIP_TRY(hipEventRecord(c->ev0, c->stream));
  const McArgs a = mc_args(c, B, T);
  if ((rc = f64 ? mc_encode_all<double>(c, a, nreps) : mc_encode_all<float>(c, a, nreps))) return rc;
  if ((rc = f64 ? mc_turnover<double>(c, a) : mc_turnover<float>(c, a))) return rc;
  // K iterations per graph replay: a replay's work is a few ms, the host
  // polls the live-slot count of the replay two back (no stall)
  const int K = 8;
  const auto key = std::make_tuple(B, T, K, flags & 0xff);
  auto it = c->mc_graphs.find(key);
  if (it == c->mc_graphs.end()) {
    HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    rc = f64 ? mc_iterations<double>(c, B, T, K, es) : mc_iterations<float>(c, B, T, K, es);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    hipGraphExec_t ex = nullptr;
    e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    it = c->mc_graphs.emplace(key, ex).first;
  }
  // every rep takes at most T iterations and a slot refills in the iteration
  // it finishes
  // (list scheduling: at most reps * T / B + T iterations)
  const long long max_replays = ((long long)(nreps + B - 1) / B * T + T + K - 1) / K + 2;
  int* live_dev = c->d_slots + 6 * c->slot_cap + 1;
  long long r = 0;
  for (; r < max_replays; ++r) {
    HIP_TRY(hipGraphLaunch(it->second, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_mc_live + (r & 3), live_dev, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->mc_ev[r & 3], c->stream));
    if (r >= 2) {
      HIP_TRY(hipEventSynchronize(c->mc_ev[(r - 2) & 3]));
      if (c->h_mc_live[(r - 2) & 3] == 0) break;
    }
  }
  HIP_TRY(hipEventRecord(c->ev1, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  int ctl[2] = {0, 0};
  HIP_TRY(hipMemcpy(ctl, c->d_slots + 6 * c->slot_cap, sizeof(ctl), hipMemcpyDeviceToHost));
  if (ctl[1] != 0 || ctl[0] != nreps) return fail(SA_ERR_HIP, "sa_mc_run: the stream did not drain");
  if (ms_out) {
    float ms = -1.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *ms_out = ms;
  }
  if (dec_out)
    HIP_TRY(hipMemcpyAsync(dec_out, c->d_mc_dec, (size_t)nreps * c->L * sizeof(int32_t), hipMemcpyDeviceToHost,
                           c->stream));
  if (iters_out)
    HIP_TRY(hipMemcpyAsync(iters_out, c->d_mc_its, (size_t)nreps * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  if (errs_out)
    HIP_TRY(hipMemcpyAsync(errs_out, c->d_mc_its + c->mc_cap, (size_t)nreps * sizeof(int32_t), hipMemcpyDeviceToHost,
                           c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->last_B = B;
  c->last_T = T;
  return SA_OK;
}

}  // extern "C"
