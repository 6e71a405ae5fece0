// sa_glue.hip — SPARC <-> LDPC glue of the joint decoder on the device
// (encoding, LLRs, bp2sp, hard / threshold decisions, cancellation).
#include "sa_host.h"

// ---------------------------------------------------------------------------
// SPARC <-> LDPC glue of the joint decoder (sparc_ldpc.py:257-314, 359-712)
// ---------------------------------------------------------------------------
// All of it runs on the device in binary64 on the B codewords of the batch;
// the LLR / app arrays are handed to and from the LDPC decoder
// (libldpc_bp.so) as device pointers, so a joint round never leaves HBM.
namespace sa {

// Columns of one-hot beta summed per row: for row r of codeword b,
//   acc = sum_{l in [l0, l0+ns)} c_l * sgn(o_lr) * H_M[k_lr, idx[b][l-l0]]
// (A[r, l*M + i] = sgn(o_lr) (-1)^popcount(k_lr & i) / sqrt(n), the same
// factorisation as the section kernels).  out = base - acc/sqrt(n) (hard
// cancellation, sparc_ldpc.py:508-518) or acc/sqrt(n) + add (encoding,
// sparc_ldpc.py:436-446).  One thread per row, idx staged in LDS.
template <typename real>
__global__ void __launch_bounds__(256) k_colsum(const ushort4* __restrict__ fwd, const double* __restrict__ cd,
                                                const int32_t* __restrict__ idx, int ldi, int l0, int ns,
                                                const real* __restrict__ base, const double* __restrict__ add,
                                                real* __restrict__ out, int n, double sqrt_n, double amp) {
  extern __shared__ int32_t sidx[];
  const int b = blockIdx.y, r = blockIdx.x * 256 + threadIdx.x;
  for (int i = threadIdx.x; i < ns; i += 256) sidx[i] = idx[(size_t)b * ldi + i];
  __syncthreads();
  if (r >= n) return;
  double acc = 0.0;
  const int g0 = l0 / kSpw, g1 = (l0 + ns + kSpw - 1) / kSpw;
  for (int g = g0; g < g1; ++g) {
    const ushort4 f = fwd[(size_t)g * n + r];
    const unsigned short fq[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int l = g * kSpw + q;
      if (l < l0 || l >= l0 + ns || sidx[l - l0] < 0) continue;  // idx < 0: section not decided
      const unsigned k = fq[q] & 0x7fffu;
      const unsigned neg = (fq[q] >> 15) ^ (__popc(k & (unsigned)sidx[l - l0]) & 1u);
      acc += neg ? -cd[l] : cd[l];
    }
  }
  const double x = (amp == 1.0 ? acc : acc * amp) / sqrt_n;
  const size_t o = (size_t)b * n + r;
  out[o] = base ? (real)((double)base[o] - x) : (real)(x + (add ? add[o] : 0.0));
}

// Sequential ascending sum of cnt LDS values v[idx(i)], i = 0..cnt-1, with
// the loads issued 16 ahead of the dependent additions (the reference's
// order; a one-lane chain otherwise waits on every LDS read).
template <typename F>
__device__ __forceinline__ double lds_seq_sum(const double* v, int cnt, F idx) {
  double s = 0.0;
  int i = 0;
  for (; i + 16 <= cnt; i += 16) {
    double r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) r[u] = v[idx(i + u)];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += r[u];
  }
  for (; i < cnt; ++i) s += v[idx(i)];
  return s;
}

// sp2bp + LLR (sparc_ldpc.py:470-479 -> :257-281): one wavefront per
// (codeword, LDPC section).  The section's posterior beta_j / c_l is read once
// (coalesced) into LDS; lane t < log2 M then forms p_t, the sum over the
// entries j whose bit (logM-1-t) is set, in ascending j (the reference's
// order); llr = nan_to_num(log(1 - p) - log(p)).
template <typename real>
__global__ void __launch_bounds__(64) k_llr(const real* __restrict__ beta, const double* __restrict__ cd, int L,
                                            int M, int lgM, int l0, int ns, double* __restrict__ llr) {
  extern __shared__ double post[];
  const size_t bl = blockIdx.x;  // b * ns + lp
  const int l = l0 + (int)(bl % ns);
  const real* bs = beta + ((bl / ns) * L + l) * M;
  const double c = cd[l];
  for (int j = threadIdx.x; j < M; j += 64) post[j] = (double)bs[j] / c;
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= lgM) return;
  const int sh = lgM - 1 - t, lo = (1 << sh) - 1;
  // i-th entry (ascending) whose bit sh is set
  const double p = lds_seq_sum(post, M >> 1, [=](int i) { return ((i >> sh) << (sh + 1)) | (lo + 1) | (i & lo); });
  double v = log(1.0 - p) - log(p);
  if (v != v) v = 0.0;                                 // nan_to_num: NaN -> 0
  else if (isinf(v)) v = v > 0 ? DBL_MAX : -DBL_MAX;  // +-inf -> +-max
  llr[bl * lgM + t] = v;
}

// bp2sp of the LDPC a-posteriori LLRs into beta0 (sparc_ldpc.py:683-696 ->
// :283-314), one wavefront per (codeword, LDPC section): bp_t = 1/(1+exp(app_t));
// sp_m = prod_t (bit_t(m) ? bp_t : 1 - bp_t), MSB first, in LDS; the
// reference's sequential normaliser S (builtin sum, :313); beta0_m = (sp_m / S) c_l.
template <typename real>
__global__ void __launch_bounds__(64) k_soft_sec(const double* __restrict__ app, const double* __restrict__ cd,
                                                 int L, int M, int lgM, int l0, int ns, real* __restrict__ beta) {
  extern __shared__ double sp[];
  __shared__ double bpv[32];
  __shared__ double S;
  const size_t bl = blockIdx.x;  // b * ns + lp
  const int l = l0 + (int)(bl % ns);
  if (threadIdx.x < lgM) bpv[threadIdx.x] = 1.0 / (1.0 + exp(app[bl * lgM + threadIdx.x]));
  __syncthreads();
  for (int m = threadIdx.x; m < M; m += 64) {
    double prod = 1.0;
    for (int t = 0; t < lgM; ++t) {
      const double bp = bpv[t];
      prod *= ((m >> (lgM - 1 - t)) & 1) ? bp : 1.0 - bp;
    }
    sp[m] = prod;
  }
  __syncthreads();
  if (threadIdx.x == 0) S = lds_seq_sum(sp, M, [](int i) { return i; });
  __syncthreads();
  const double c = cd[l], tot = S;
  real* o = beta + ((bl / ns) * L + l) * M;
  for (int m = threadIdx.x; m < M; m += 64) o[m] = (real)((sp[m] / tot) * c);
}

// beta0 of the sections AMP keeps (:657, :691, :696): (beta / c) * c.
template <typename real>
__global__ void k_rescale(real* __restrict__ beta, const double* __restrict__ cd, int L, int M, int l0, int ns,
                          int B) {
  const size_t tot = (size_t)B * L * M;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    const int l = (int)((i / M) % L);
    if (l >= l0 && l < l0 + ns) continue;
    const double c = cd[l];
    beta[i] = (real)(((double)beta[i] / c) * c);
  }
}

// Hard decisions of the LDPC output (:486-490): bits = app < 0, MSB first.
__global__ void k_app_idx(const double* __restrict__ app, int lgM, int ns, int B, int32_t* __restrict__ idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * ns) return;
  const double* a = app + (size_t)i * lgM;
  int32_t v = 0;
  for (int t = 0; t < lgM; ++t) v = (v << 1) | (a[t] < 0.0 ? 1 : 0);
  idx[i] = v;
}

// One-hot beta0 (sparc_ldpc.py:832-835): beta[b][l*M + idx[b][l]] = c_l, 0 elsewhere.
template <typename real>
__global__ void k_onehot(const int32_t* __restrict__ idx, const double* __restrict__ cd, int L, int M, int B,
                         double scale, real* __restrict__ beta) {
  const size_t tot = (size_t)B * L * M;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
    const size_t bl = i / M;
    const int m = (int)(i % M), l = (int)(bl % L);
    beta[i] = m == idx[bl] ? (real)(scale == 1.0 ? cd[l] : cd[l] * scale) : (real)0;  // idx < 0: all zero
  }
}

// Threshold decisions of the LDPC soft output (amp_exit.py:56-105 on the
// bp2sp of sparc_ldpc.py:987-994): per (codeword, section) the normalised
// product of bit marginals sp_m / S; the section is decided (index m) iff
// exactly one entry exceeds the threshold, else -1.  One workgroup per
// section: products in LDS, the reference's sequential normaliser, counts.
__global__ void __launch_bounds__(256) k_threshold(const double* __restrict__ app, int M, int lgM, int ns,
                                                   double thr, int32_t* __restrict__ idx) {
  extern __shared__ double sp[];
  __shared__ int cnt, pick;
  __shared__ double S, bpv[32];
  const size_t bl = blockIdx.x;  // b * ns + section
  if (threadIdx.x < lgM) bpv[threadIdx.x] = 1.0 / (1.0 + exp(app[bl * lgM + threadIdx.x]));
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (int m = threadIdx.x; m < M; m += 256) {
    double prod = 1.0;
    for (int t = 0; t < lgM; ++t) {
      const double bp = bpv[t];
      prod *= ((m >> (lgM - 1 - t)) & 1) ? bp : 1.0 - bp;
    }
    sp[m] = prod;
  }
  __syncthreads();
  if (threadIdx.x == 0) S = lds_seq_sum(sp, M, [](int i) { return i; });
  __syncthreads();
  for (int m = threadIdx.x; m < M; m += 256)
    if (sp[m] / S > thr) {
      atomicAdd(&cnt, 1);
      pick = m;  // only read when cnt == 1
    }
  __syncthreads();
  if (threadIdx.x == 0) idx[bl] = cnt == 1 ? pick : -1;
}

int grid_of(size_t tot) {
  const size_t g = (tot + 255) / 256;
  return (int)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

constexpr int kGlueMaxM = 8192;  // a section of fp64 in the 64 KiB of dynamic LDS

int check_glue(sa_ctx* c, int B, int l0, int ns) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || B > c->Bcap) return fail(SA_ERR_ARG, "batch larger than the context's workspace");
  if (l0 < 0 || ns <= 0 || l0 + ns > c->L) return fail(SA_ERR_ARG, "section range outside [0, L)");
  if (!c->power_set) return fail(SA_ERR_ARG, "power allocation not staged");
  if (c->M < 2) return fail(SA_ERR_UNSUPPORTED, "M < 2 carries no bits");
  if (!c->pow2) return fail(SA_ERR_UNSUPPORTED, "bit-level glue needs M a power of two (bits2indices, sparc_ldpc.py:317)");
  if (c->M > kGlueMaxM) return fail(SA_ERR_UNSUPPORTED, "SPARC<->LDPC glue stages a section in LDS: M <= 8192");
  return SA_OK;
}

// Host-or-device fp64 array of `count` values on the context's device:
// returns a device pointer (copying host data into the staging buffer).
int dev_in(sa_ctx* c, const double* p, size_t count, int flags, const double** out) {
  if (flags & SA_PTR_DEVICE) {
    *out = p;
    return SA_OK;
  }
  int rc = ensure_stage(c, count);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, p, count * 8, hipMemcpyHostToDevice, c->stream));
  *out = c->d_stage;
  return SA_OK;
}

template <typename real>
int launch_colsum(sa_ctx* c, const int32_t* d_idx, int ldi, int l0, int ns, const real* base, const double* add,
                  real* out, int B, double amp = 1.0) {
  dim3 grid((c->n + 255) / 256, B);
  k_colsum<real><<<grid, 256, (size_t)ns * sizeof(int32_t), c->stream>>>(
      (const ushort4*)c->d_fwd, c->d_cd, d_idx, ldi, l0, ns, base, add, out, c->n, std::sqrt((double)c->n), amp);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

}  // namespace sa

using namespace sa;

extern "C" {

int sa_encode(sa_ctx* c, int B, const int32_t* idx, const double* noise) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || !idx) return fail(SA_ERR_ARG, "sa_encode: bad arguments");
  if (!c->power_set) return fail(SA_ERR_ARG, "sa_encode: power allocation not staged");
  if (int rc0 = check_tables(c, "sa_encode")) return rc0;
  if (!c->pow2) return fail(SA_ERR_UNSUPPORTED, "sa_encode: the row-parallel encoder needs M a power of two");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, c->Tcap > 0 ? c->Tcap : 1);
  if (rc) return rc;
  for (size_t i = 0; i < (size_t)B * c->L; ++i)
    if (idx[i] < 0 || idx[i] >= c->M) return fail(SA_ERR_ARG, "sa_encode: index outside [0, M)");
  HIP_TRY(hipMemcpyAsync(c->d_idx, idx, (size_t)B * c->L * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  const double* d_noise = nullptr;
  if (noise && (rc = dev_in(c, noise, (size_t)B * c->n, 0, &d_noise))) return rc;
  rc = c->prec == SA_PREC_F64
           ? launch_colsum<double>(c, c->d_idx, c->L, 0, c->L, nullptr, d_noise, (double*)c->d_y, B)
           : launch_colsum<float>(c, c->d_idx, c->L, 0, c->L, nullptr, d_noise, (float*)c->d_y, B);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

namespace {
int stage_onehot_impl(sa_ctx* c, int B, const int32_t* idx, double scale, bool allow_empty) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || B > c->Bcap || !idx) return fail(SA_ERR_ARG, "sa_stage_onehot: bad arguments");
  if (!c->power_set) return fail(SA_ERR_ARG, "sa_stage_onehot: power allocation not staged");
  if (!std::isfinite(scale)) return fail(SA_ERR_ARG, "sa_stage_onehot: scale must be finite");
  if (c->dead) return fail(SA_ERR_UNSUPPORTED, "sa_stage_onehot: M must be a power of two (bits2indices)");
  for (size_t i = 0; i < (size_t)B * c->L; ++i)
    if (idx[i] >= c->M || (idx[i] < 0 && !(allow_empty && idx[i] == -1)))
      return fail(SA_ERR_ARG, "sa_stage_onehot: index outside [0, M)");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(c->d_idx, idx, (size_t)B * c->L * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  const size_t tot = (size_t)B * c->L * c->M;
  if (c->prec == SA_PREC_F64)
    k_onehot<double><<<grid_of(tot), 256, 0, c->stream>>>(c->d_idx, c->d_cd, c->L, c->M, B, scale, (double*)c->d_beta);
  else
    k_onehot<float><<<grid_of(tot), 256, 0, c->stream>>>(c->d_idx, c->d_cd, c->L, c->M, B, scale, (float*)c->d_beta);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}
}  // namespace

int sa_stage_onehot(sa_ctx* c, int B, const int32_t* idx) { return stage_onehot_impl(c, B, idx, 1.0, false); }

int sa_stage_onehot_scaled(sa_ctx* c, int B, const int32_t* idx, double scale) {
  return stage_onehot_impl(c, B, idx, scale, true);
}

int sa_llr(sa_ctx* c, int B, int l0, int ns, double* llr, int flags) {
  int rc = check_glue(c, B, l0, ns);
  if (rc) return rc;
  if (!llr) return fail(SA_ERR_ARG, "sa_llr: llr is NULL");
  HIP_TRY(hipSetDevice(c->device));
  const int lgM = ilog2(c->M);
  const size_t cnt = (size_t)B * ns * lgM;
  double* d_out = llr;
  if (!(flags & SA_PTR_DEVICE)) {
    if ((rc = ensure_stage(c, cnt))) return rc;
    d_out = c->d_stage;
  }
  const size_t lds = (size_t)c->M * sizeof(double);
  if (c->prec == SA_PREC_F64)
    k_llr<double><<<B * ns, 64, lds, c->stream>>>((const double*)c->d_beta, c->d_cd, c->L, c->M, lgM, l0, ns, d_out);
  else
    k_llr<float><<<B * ns, 64, lds, c->stream>>>((const float*)c->d_beta, c->d_cd, c->L, c->M, lgM, l0, ns, d_out);
  HIP_TRY(hipGetLastError());
  if (!(flags & SA_PTR_DEVICE)) HIP_TRY(hipMemcpyAsync(llr, d_out, cnt * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_soft_beta0(sa_ctx* c, int B, int l0, int ns, const double* app, int flags) {
  int rc = check_glue(c, B, l0, ns);
  if (rc) return rc;
  if (!app) return fail(SA_ERR_ARG, "sa_soft_beta0: app is NULL");
  HIP_TRY(hipSetDevice(c->device));
  const int lgM = ilog2(c->M);
  const size_t na = (size_t)B * ns * lgM;
  const double* d_app = app;
  if (!(flags & SA_PTR_DEVICE)) {
    if ((rc = ensure_stage(c, na))) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_stage, app, na * 8, hipMemcpyHostToDevice, c->stream));
    d_app = c->d_stage;
  }
  const size_t tot = (size_t)B * c->L * c->M, lds = (size_t)c->M * sizeof(double);
  if (c->prec == SA_PREC_F64) {
    if (ns < c->L) k_rescale<double><<<grid_of(tot), 256, 0, c->stream>>>((double*)c->d_beta, c->d_cd, c->L, c->M, l0, ns, B);
    k_soft_sec<double><<<B * ns, 64, lds, c->stream>>>(d_app, c->d_cd, c->L, c->M, lgM, l0, ns, (double*)c->d_beta);
  } else {
    if (ns < c->L) k_rescale<float><<<grid_of(tot), 256, 0, c->stream>>>((float*)c->d_beta, c->d_cd, c->L, c->M, l0, ns, B);
    k_soft_sec<float><<<B * ns, 64, lds, c->stream>>>(d_app, c->d_cd, c->L, c->M, lgM, l0, ns, (float*)c->d_beta);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_hard_cancel(sa_ctx* c, int B, int l0, int ns, const double* app, int flags, sa_ctx* dst, int32_t* idx_out) {
  if (dst && check_tables(c, "sa_hard_cancel")) return SA_ERR_UNSUPPORTED;
  int rc = check_glue(c, B, l0, ns);
  if (rc) return rc;
  if (!app) return fail(SA_ERR_ARG, "sa_hard_cancel: app is NULL");
  if (dst && (dst->n != c->n || dst->prec != c->prec || dst->device != c->device))
    return fail(SA_ERR_ARG, "sa_hard_cancel: dst must share n, precision and device");
  HIP_TRY(hipSetDevice(c->device));
  if (dst && (rc = ensure_workspace(dst, B, dst->Tcap > 0 ? dst->Tcap : 1))) return rc;
  const int lgM = ilog2(c->M);
  const double* d_app = nullptr;
  if ((rc = dev_in(c, app, (size_t)B * ns * lgM, flags, &d_app))) return rc;
  k_app_idx<<<(B * ns + 255) / 256, 256, 0, c->stream>>>(d_app, lgM, ns, B, c->d_idx);
  HIP_TRY(hipGetLastError());
  if (dst) {
    rc = c->prec == SA_PREC_F64
             ? launch_colsum<double>(c, c->d_idx, ns, l0, ns, (const double*)c->d_y, nullptr, (double*)dst->d_y, B)
             : launch_colsum<float>(c, c->d_idx, ns, l0, ns, (const float*)c->d_y, nullptr, (float*)dst->d_y, B);
    if (rc) return rc;
  }
  if (idx_out)
    HIP_TRY(hipMemcpyAsync(idx_out, c->d_idx, (size_t)B * ns * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_threshold(sa_ctx* c, int B, int l0, int ns, const double* app, int flags, double threshold,
                 int32_t* idx_out) {
  int rc = check_glue(c, B, l0, ns);
  if (rc) return rc;
  if (!app || !idx_out) return fail(SA_ERR_ARG, "sa_threshold: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const int lgM = ilog2(c->M);
  const double* d_app = nullptr;
  if ((rc = dev_in(c, app, (size_t)B * ns * lgM, flags, &d_app))) return rc;
  k_threshold<<<B * ns, 256, (size_t)c->M * sizeof(double), c->stream>>>(d_app, c->M, lgM, ns, threshold, c->d_idx);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(idx_out, c->d_idx, (size_t)B * ns * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_cancel_scaled(sa_ctx* c, int B, const int32_t* idx, double scale, sa_ctx* dst) {
  if (check_ctx(c) || check_ctx(dst)) return SA_ERR_ARG;
  if (int rc0 = check_tables(c, "sa_cancel")) return rc0;
  if (!c->pow2) return fail(SA_ERR_UNSUPPORTED, "sa_cancel: needs M a power of two");
  if (B <= 0 || B > c->Bcap || !idx) return fail(SA_ERR_ARG, "sa_cancel: bad arguments");
  if (!c->power_set) return fail(SA_ERR_ARG, "sa_cancel: power allocation not staged");
  if (dst->n != c->n || dst->prec != c->prec || dst->device != c->device)
    return fail(SA_ERR_ARG, "sa_cancel: dst must share n, precision and device");
  for (size_t i = 0; i < (size_t)B * c->L; ++i)
    if (idx[i] >= c->M) return fail(SA_ERR_ARG, "sa_cancel: index >= M");
  if (!std::isfinite(scale)) return fail(SA_ERR_ARG, "sa_cancel: scale must be finite");
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_workspace(dst, B, dst->Tcap > 0 ? dst->Tcap : 1))) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_idx, idx, (size_t)B * c->L * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  rc = c->prec == SA_PREC_F64
           ? launch_colsum<double>(c, c->d_idx, c->L, 0, c->L, (const double*)c->d_y, nullptr, (double*)dst->d_y, B, scale)
           : launch_colsum<float>(c, c->d_idx, c->L, 0, c->L, (const float*)c->d_y, nullptr, (float*)dst->d_y, B, scale);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_cancel(sa_ctx* c, int B, const int32_t* idx, sa_ctx* dst) { return sa_cancel_scaled(c, B, idx, 1.0, dst); }

}  // extern "C"
