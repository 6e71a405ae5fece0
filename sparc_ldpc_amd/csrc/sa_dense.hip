// sa_dense.hip — the materialised-matrix backends: the Hadamard design as an
// fp32 matrix (GEMVs; int8 MFMA GEMMs from 4 codewords, dense_i8.hip), a
// caller's dense design (SA_BACKEND_MATRIX: GEMVs; f32 / f64 MFMA GEMMs,
// dense_mfma.hip), the dense denoiser, and the host-operator loop's kernels.
#include "sa_host.h"

namespace sa {

// ---------------------------------------------------------------------------
// Dense backend (fp32 A, HBM-streamed GEMV pair)
// ---------------------------------------------------------------------------

// A[r][j] = (-1)^popcount(ordering[l][r] & (w - M + c)) / sqrt(n), j = l*M + c
// (sparc_ldpc.py:65-77 with the 1/sqrt(n) of :143-146); columns >= L*M are 0.
__global__ void k_dense_build(const uint32_t* ord, float* A, int L, int M, int n, int w,
                              size_t lda, float s) {
  const size_t total = (size_t)n * lda;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const size_t r = idx / lda, j = idx % lda;
    float v = 0.f;
    if (j < (size_t)L * M) {
      const int l = (int)(j / M), c = (int)(j % M);
      const uint32_t o = ord[(size_t)l * n + r];
      v = (__popc(o & (uint32_t)(w - M + c)) & 1) ? -s : s;
    }
    A[idx] = v;
  }
}

// 16-byte vectors of the dense kernels: 4 binary32 or 2 binary64 elements
template <typename real> struct V16;
template <> struct V16<float> { using t = f4; static constexpr int N = 4; };
template <> struct V16<double> { using t = double __attribute__((ext_vector_type(2))); static constexpr int N = 2; };

// Streaming (non-temporal) 16-B load of the design matrix: read once per pass.
template <typename real>
__device__ __forceinline__ typename V16<real>::t ld_stream_v(const real* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const typename V16<real>::t*>(p));
}

template <typename real>
struct DenseArgs {
  const real* A;      // [n][lda]
  const real* z;      // [B][n]
  real* azp;          // [B][RS][lda]    Az partials (A carries any 1/sqrt(n))
  const real* beta;   // [B][L*M]
  real* abp;          // [B][KS][n]      Ab partials
  const real* zzp;    // [B][NZ]
  const real* tau;    // [B][T1]
  int L, M, n, NZ, T1, t, early_stop, RS, KS, mode;  // mode: 0 = AMP stop test, 1 = none
  size_t lda;
};

template <typename real>
__device__ __forceinline__ bool dense_stopped(const DenseArgs<real>& a, int b) {
  if (a.mode != 0 || !a.early_stop) return false;
  const real tau = tau_from_parts(a.zzp + (size_t)b * a.NZ, a.NZ, a.n);
  const real last = a.t > 0 ? a.tau[(size_t)b * a.T1 + a.t - 1] : (real)0;
  return tau == last;
}

// Az partials: azp[b][rs][j] = sum_{r in split rs} A[r][j] z[b][r].
// 256 threads x one 16-B column vector (4 binary32 / 2 binary64 columns) per
// workgroup; rows split RS ways; row order within a split.
template <typename real>
__global__ void __launch_bounds__(256) k_dense_az(DenseArgs<real> a) {
  constexpr int N = V16<real>::N;
  __shared__ real zsh[2048];
  const int b = blockIdx.z, rs = blockIdx.y;
  if (dense_stopped(a, b)) return;
  const int rows_per = (a.n + a.RS - 1) / a.RS;
  const int r0 = rs * rows_per, r1 = min(a.n, r0 + rows_per);
  const size_t j = ((size_t)blockIdx.x * 256 + threadIdx.x) * N;
  real acc[N];
#pragma unroll
  for (int q = 0; q < N; ++q) acc[q] = 0;
  for (int rb = r0; rb < r1; rb += 2048) {
    const int cnt = min(2048, r1 - rb);
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += 256) zsh[i] = a.z[(size_t)b * a.n + rb + i];
    __syncthreads();
    if (j < a.lda) {
      const real* Ap = a.A + (size_t)rb * a.lda + j;
      int i = 0;
      for (; i + 8 <= cnt; i += 8) {
        typename V16<real>::t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld_stream_v<real>(Ap + (size_t)(i + u) * a.lda);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const real zz = zsh[i + u];
#pragma unroll
          for (int q = 0; q < N; ++q) acc[q] += v[u][q] * zz;
        }
      }
      for (; i < cnt; ++i) {
        const typename V16<real>::t v = *reinterpret_cast<const typename V16<real>::t*>(Ap + (size_t)i * a.lda);
        const real zz = zsh[i];
#pragma unroll
        for (int q = 0; q < N; ++q) acc[q] += v[q] * zz;
      }
    }
  }
  if (j < a.lda) {
    typename V16<real>::t o;
#pragma unroll
    for (int q = 0; q < N; ++q) o[q] = acc[q];
    *reinterpret_cast<typename V16<real>::t*>(a.azp + ((size_t)b * a.RS + rs) * a.lda + j) = o;
  }
}

// Ab partials: abp[b][ks][r] = sum_{j in split ks} A[r][j] beta[b][j];
// 8 rows per workgroup share each 16-B beta load.
constexpr int kDenseRows = 8;
template <typename real>
__global__ void __launch_bounds__(256) k_dense_ab(DenseArgs<real> a, const real* tau) {
  constexpr int N = V16<real>::N;
  __shared__ real red[kDenseRows][4];
  const int b = blockIdx.z, ks = blockIdx.y;
  if (a.mode == 0 && a.early_stop) {
    const real t0 = tau[(size_t)b * a.T1 + a.t];
    const real t1 = a.t > 0 ? tau[(size_t)b * a.T1 + a.t - 1] : (real)0;
    if (t0 == t1) return;
  }
  const int r0 = blockIdx.x * kDenseRows;
  const size_t LM = (size_t)a.L * a.M;
  const size_t nv = (LM + N - 1) / N;  // 16-B column vectors with data (pad columns are 0 in A)
  const size_t per = (nv + a.KS - 1) / a.KS;
  const size_t c0 = ks * per, c1 = c0 + per < nv ? c0 + per : nv;
  real acc[kDenseRows];
#pragma unroll
  for (int k = 0; k < kDenseRows; ++k) acc[k] = 0;
  const real* bb = a.beta + (size_t)b * LM;
  for (size_t c = c0 + threadIdx.x; c < c1; c += 256) {
    real bv[N];
    if (c * N + N - 1 < LM && ((LM % N) == 0)) {
      const typename V16<real>::t t = *reinterpret_cast<const typename V16<real>::t*>(bb + c * N);
#pragma unroll
      for (int q = 0; q < N; ++q) bv[q] = t[q];
    } else {
#pragma unroll
      for (int q = 0; q < N; ++q) bv[q] = c * N + q < LM ? bb[c * N + q] : (real)0;
    }
#pragma unroll
    for (int k = 0; k < kDenseRows; ++k) {
      const int r = r0 + k;
      if (r < a.n) {
        const typename V16<real>::t v = ld_stream_v<real>(a.A + (size_t)r * a.lda + c * N);
        real d = v[0] * bv[0];
#pragma unroll
        for (int q = 1; q < N; ++q) d += v[q] * bv[q];
        acc[k] += d;
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kDenseRows; ++k) {
    const real s = wave_sum(acc[k]);
    if (lane == 0) red[k][wv] = s;
  }
  __syncthreads();
  if (threadIdx.x < kDenseRows) {
    const int r = r0 + threadIdx.x;
    if (r < a.n) {
      const real s = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
      a.abp[((size_t)b * a.KS + ks) * a.n + r] = s;
    }
  }
}

// Dense Az partial reduction into d_out (B x L*M), used by sa_Az on the dense backends.
template <typename real>
__global__ void k_dense_az_reduce(const real* azp, real* out, int RS, size_t lda, size_t LM, int B) {
  const size_t total = (size_t)B * LM;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t b = i / LM, j = i % LM;
    real s = 0;
    for (int rs = 0; rs < RS; ++rs) s += azp[(b * RS + rs) * lda + j];
    out[i] = s;
  }
}

// A caller's matrix (SA_BACKEND_MATRIX): rows [r0, r0 + rows) of the fp64
// host matrix (staged, [rows][LM]) into the device matrix [np][lda] in the
// context precision, pad columns zero.
template <typename real>
__global__ void k_matrix_rows(const double* __restrict__ src, real* __restrict__ A, long long rows, long long LM,
                              size_t lda, long long r0) {
  const long long total = rows * (long long)lda;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / (long long)lda, j = i % (long long)lda;
    A[(size_t)(r0 + r) * lda + j] = j < LM ? (real)src[r * LM + j] : (real)0;
  }
}

#include "dense_i8.h"
#include "dense_mfma.h"

// Dense-path denoiser: sums the RS Az partials of one section (wave) and
// applies denoise_section; writes tau (workgroup 0) and beta^2 partials.
// On the int8 matrix-core path (bq != NULL) it also writes the new beta's
// kI8NPB base-256 digit planes at the fixed scale bfix[0] (beta_l <= c_l, so
// one power-of-two scale per decode: dense_i8.hip).
// Also the denoiser of the host-operator path (SA_BACKEND_HOST: the caller's
// A^T z uploaded as the single partial), in either precision.
template <typename real>
struct DenArgs {
  const real* azp;  // [B][RS][lda] A^T z partials (scaled: A carries 1/sqrt(n))
  const real* zzp;  // [B][NZ]
  const real* tau;  // [B][T1]
  int L, M, n, NZ, T1, t, early_stop, RS;
  size_t lda;
};

template <typename real, int E>
__global__ void __launch_bounds__(256) k_dense_den(DenArgs<real> a, const real* c, real* beta,
                                                   real* bbp, real* tau_out, int* iters, int G,
                                                   int8_t* bq, long long bq_ps, long long bq_ld,
                                                   const double* bfix) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = blockIdx.x, b = blockIdx.y;
  const int l = g * 4 + wv;
  const int M = a.M;
  const real tau = tau_from_parts(a.zzp + (size_t)b * a.NZ, a.NZ, a.n);
  const real last = a.t > 0 ? a.tau[(size_t)b * a.T1 + a.t - 1] : (real)0;
  const bool stop = a.early_stop && tau == last;
  if (g == 0 && threadIdx.x == 0) {
    tau_out[(size_t)b * a.T1 + a.t] = tau;
    if (stop && iters[b] < 0) iters[b] = a.t;
  }
  if (stop) return;
  __shared__ real bbw[4];
  real bb = 0;
  if (l < a.L) {
    real v[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = elem_index<E>(lane, i);
      real s = 0;
      if (e < M)
        for (int rs = 0; rs < a.RS; ++rs) s += a.azp[((size_t)b * a.RS + rs) * a.lda + (size_t)l * M + e];
      v[i] = s;  // already carries the 1/sqrt(n) of A
    }
    real* bl = beta + ((size_t)b * a.L + l) * M;
    real bprev[E];
    load_section_any<real, E>(bl, bprev, lane, M);
    bb = denoise_section<real, E>(v, bprev, bl, lane, M, c[l], tau * tau, (real)1, false);
    store_section_any<real, E>(bl, v, lane, M);
    if (bq) {
      const double sf = bfix[0];
      int8_t* qb = bq + (long long)b * bq_ld + (long long)l * M;
      if (E >= 4 && (M & 3) == 0) {  // 4 consecutive elements per lane: one 4-byte store per plane
#pragma unroll
        for (int i = 0; i < (E >= 4 ? E : 0); i += 4) {
          const int e = elem_index<E>(lane, i);
          if (e >= M) continue;
          int d[4][kI8NPB];
#pragma unroll
          for (int u = 0; u < 4; ++u) i8_digits<kI8NPB>((int)rint((double)v[i + u] * sf), d[u]);
#pragma unroll
          for (int p = 0; p < kI8NPB; ++p)
            *reinterpret_cast<char4*>(qb + p * bq_ps + e) = make_char4(d[0][p], d[1][p], d[2][p], d[3][p]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < E; ++i) {
          const int e = elem_index<E>(lane, i);
          if (e < M) {
            int d[kI8NPB];
            i8_digits<kI8NPB>((int)rint((double)v[i] * sf), d);
#pragma unroll
            for (int p = 0; p < kI8NPB; ++p) qb[p * bq_ps + e] = (int8_t)d[p];
          }
        }
      }
    }
  }
  if (lane == 0) bbw[wv] = bb;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ns = min(4, a.L - g * 4);
    real t = 0;
    for (int s = 0; s < ns; ++s) t += bbw[s];
    bbp[(size_t)b * G + g] = t;
  }
}

// tau_t of the host-operator loop (sparc_ldpc.py:203-209), ahead of the
// caller's A^T z: tau[b][t], the exact tau == last_tau stop and stopped[b].
template <typename real>
__global__ void __launch_bounds__(64) k_tau(const real* zzp, int NZ, int n, real* tau, int T1, int t,
                                            int early_stop, int* iters, int* stopped) {
  const int b = blockIdx.x;
  const real tv = tau_from_parts(zzp + (size_t)b * NZ, NZ, n);
  if (threadIdx.x == 0) {
    const real last = t > 0 ? tau[(size_t)b * T1 + t - 1] : (real)0;
    const bool stop = early_stop && tv == last;
    tau[(size_t)b * T1 + t] = tv;
    if (stop && iters[b] < 0) iters[b] = t;
    stopped[b] = stop ? 1 : 0;
  }
}

// ---- host side -------------------------------------------------------------
// ---- int8 matrix-core dense path (dense_i8.hip) -------------------------
int i8_bp(int B) { return (B + kI8TX - 1) / kI8TX * kI8TX; }

// K splits of the A beta GEMM for B codewords: the fewest (workgroup rounds x
// stages per workgroup), i.e. the shortest critical path on n_cus CUs
int i8_splits(const sa_ctx* c, int B) {
  const long long tiles = (long long)(c->np8 / kI8TY) * (i8_bp(B) / kI8TX);
  const int nst = (int)(c->LMp8 / kI8KS);
  int best = 1;
  long long bcost = -1;
  for (int S = 1; S <= kI8MaxS; ++S) {
    const long long rounds = (tiles * S + c->n_cus - 1) / c->n_cus;
    const long long cost = rounds * ((nst + S - 1) / S);
    if (bcost < 0 || cost < bcost) { bcost = cost; best = S; }
  }
  return best;
}

// The fixed digit scale of beta on the GEMM path: beta_l <= c_l (the softmax
// weights sum to one), so s = 2^(30 - E) with c_max (1 + 2^-10) < 2^E keeps
// |rint(beta s)| <= 2^30 (four digits); bfix = {s, 1 / (s sqrt(n))} in device
// memory (a replayed graph reads the current value).
int i8_set_bfix(sa_ctx* c) {
  int E = 0;
  if (c->cmax > 0) (void)std::frexp(c->cmax * (1.0 + 1.0 / 1024), &E);
  const double sfix = std::ldexp(1.0, i8_bits<kI8NPB>() - E);
  const double h[2] = {sfix, 1.0 / (sfix * std::sqrt((double)c->n))};
  HIP_TRY(hipMemcpyAsync(c->d_bfix, h, sizeof(h), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

// Builds A8 / AT8 on first use and sizes the digit planes for B codewords.
int ensure_i8(sa_ctx* c, int B) {
  if (!use_i8(c, B)) return SA_OK;
  int rc;
  if (!c->d_A8) {
    c->np8 = ((long long)c->n + kI8TY - 1) / kI8TY * kI8TY;
    c->LMp8 = ((long long)c->L * c->M + kI8TY - 1) / kI8TY * kI8TY;
    const size_t bytes = (size_t)c->np8 * (size_t)c->LMp8;
    if ((rc = dev_alloc(c, (void**)&c->d_A8, bytes))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_AT8, bytes))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_bfix, 2 * sizeof(double)))) return rc;
    uint32_t* d_ord = nullptr;
    HIP_TRY(hipMalloc(&d_ord, c->ordering.size() * 4));
    HIP_TRY(hipMemcpyAsync(d_ord, c->ordering.data(), c->ordering.size() * 4, hipMemcpyHostToDevice, c->stream));
    k_i8_build<<<8192, 256, 0, c->stream>>>(d_ord, c->d_A8, c->L, c->M, c->n, c->w, c->np8, c->LMp8, 0);
    k_i8_build<<<8192, 256, 0, c->stream>>>(d_ord, c->d_AT8, c->L, c->M, c->n, c->w, c->LMp8, c->np8, 1);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_ord);
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("k_i8_build: ") + hipGetErrorString(e));
    if (c->power_set && (rc = i8_set_bfix(c))) return rc;
  }
  const int Bp = i8_bp(B);
  if (Bp > c->Bp8) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    drop_graphs(c);
    dev_free(c->d_zq); dev_free(c->d_bq); dev_free(c->d_zsc); dev_free(c->d_bsc0);
    c->d_zq = c->d_bq = nullptr;
    c->d_zsc = c->d_bsc0 = nullptr;
    c->Bp8 = 0;
    const size_t zb = kI8NPZ * (size_t)Bp * (size_t)c->np8, bb = kI8NPB * (size_t)Bp * (size_t)c->LMp8;
    if ((rc = dev_alloc(c, (void**)&c->d_zq, zb))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_bq, bb))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_zsc, (size_t)Bp * sizeof(double)))) return rc;
    if ((rc = dev_alloc(c, (void**)&c->d_bsc0, (size_t)Bp * sizeof(double)))) return rc;
    HIP_TRY(hipMemsetAsync(c->d_zq, 0, zb, c->stream));  // K and codeword padding stays zero
    HIP_TRY(hipMemsetAsync(c->d_bq, 0, bb, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->Bp8 = Bp;
  }
  return SA_OK;
}

template <typename real>
DenseArgs<real> dense_args(sa_ctx* c, int t, int es, int mode) {
  DenseArgs<real> a;
  a.A = (const real*)c->d_A; a.z = (const real*)c->d_z; a.azp = (real*)c->d_azp;
  a.beta = (const real*)c->d_beta; a.abp = (real*)c->d_abp; a.zzp = (const real*)c->d_zzp;
  a.tau = (const real*)c->d_tau;
  a.L = c->L; a.M = c->M; a.n = c->n; a.NZ = c->nz_cur; a.T1 = c->Tcap + 1; a.t = t;
  a.early_stop = es; a.RS = c->RS; a.KS = c->KS; a.mode = mode; a.lda = c->lda;
  return a;
}

template <typename real>
int launch_dense_az(sa_ctx* c, int B, int t, int es, int mode) {
  DenseArgs<real> a = dense_args<real>(c, t, es, mode);
  dim3 grid((unsigned)((c->lda / V16<real>::N + 255) / 256), c->RS, B);
  if (c->prof) c->prof->begin(c->stream, K_DAZ);
  plaunch(c, k_dense_az<real>, grid, 256, 0, a);
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

template <typename real>
int launch_dense_ab(sa_ctx* c, int B, int t, int es, int mode) {
  DenseArgs<real> a = dense_args<real>(c, t, es, mode);
  dim3 grid((unsigned)((c->n + kDenseRows - 1) / kDenseRows), c->KS, B);
  if (c->prof) c->prof->begin(c->stream, K_DAB);
  plaunch(c, k_dense_ab<real>, grid, 256, 0, a, (const real*)c->d_tau);
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

template <typename real, int E>
void launch_dense_den_e(sa_ctx* c, int B, const DenArgs<real>& a, bool i8) {
  dim3 grid(c->Gd, B);
  if (c->prof) c->prof->begin(c->stream, K_DDEN);
  plaunch(c, k_dense_den<real, E>, grid, 256, 0, a, (const real*)c->d_c, (real*)c->d_beta,
                                               (real*)c->d_bbp, (real*)c->d_tau, c->d_iters, c->Gd,
                                               i8 ? c->d_bq : nullptr, (long long)c->Bp8 * c->LMp8,
                                               c->LMp8, c->d_bfix);
  if (c->prof) c->prof->end(c->stream);
}

// i8 = true: the Az of the matrix-core GEMM (one partial, d_azp[b][0][:]) and
// the beta digit planes written for the next A beta GEMM.  The host-operator
// backend's A^T z is one uploaded partial as well.
template <typename real>
int launch_dense_den(sa_ctx* c, int B, int t, int es, bool i8 = false, bool one_partial = false) {
  DenArgs<real> a;
  a.azp = (const real*)c->d_azp; a.zzp = (const real*)c->d_zzp; a.tau = (const real*)c->d_tau;
  a.L = c->L; a.M = c->M; a.n = c->n; a.NZ = c->nz_cur; a.T1 = c->Tcap + 1; a.t = t; a.early_stop = es;
  a.RS = (i8 || one_partial || c->backend == SA_BACKEND_HOST) ? 1 : c->RS;
  a.lda = c->lda;
  switch (c->E) {
    case 1: launch_dense_den_e<real, 1>(c, B, a, i8); break;
    case 2: launch_dense_den_e<real, 2>(c, B, a, i8); break;
    case 4: launch_dense_den_e<real, 4>(c, B, a, i8); break;
    case 8: launch_dense_den_e<real, 8>(c, B, a, i8); break;
    case 16: launch_dense_den_e<real, 16>(c, B, a, i8); break;
    case 32: launch_dense_den_e<real, 32>(c, B, a, i8); break;
    case 64: launch_dense_den_e<real, 64>(c, B, a, i8); break;
    default: return fail(SA_ERR_UNSUPPORTED, "bad E");
  }
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

// Digit planes of B vectors of length len (rows ld apart) -> q planes of K
// bytes per row (K = np8 for z, LMp8 for beta), scales sc[b] = 1/(s_b sqrt(n)).
template <int NP>
int launch_i8_quant(sa_ctx* c, int B, const void* src, long long ld, int len, int8_t* q, long long K, double* sc) {
  if (c->prof) c->prof->begin(c->stream, K_QNT);
  plaunch(c, k_i8_quant<NP>, B, 256, 0, (const float*)src, ld, len, q, (long long)c->Bp8 * K, K,
                                                         sc, 1.0 / std::sqrt((double)c->n));
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

// out[b][s][y] = (A v_b)_y restricted to K split s: the digit planes X
// ([NP][Bp8][K]) against the +-1 matrix Y (rows of K bytes), Ny valid rows.
template <int NP>
int launch_gemm_i8(sa_ctx* c, int B, const int8_t* X, long long K, const int8_t* Y, long long Yrows, int Ny,
                   float* out, long long ldb, long long lds, int S, const double* scale, int sst, int kind) {
  I8Args a;
  a.X = X; a.Y = Y; a.out = out; a.scale = scale;
  a.xps = (long long)c->Bp8 * K; a.K = K; a.ldb = ldb; a.lds = lds;
  a.nst = (int)(K / kI8KS);
  a.kps = (a.nst + S - 1) / S;
  a.XT = i8_bp(B) / kI8TX; a.YT = (int)(Yrows / kI8TY); a.S = S;
  a.B = B; a.Ny = Ny; a.sst = sst;
  if (i8_bp(B) > c->Bp8 || K % kI8KS || Yrows % kI8TY) return fail(SA_ERR_ARG, "k_gemm_i8: operand shapes");
  const long long grid = (long long)a.XT * a.YT * S;
  if (grid > 0x7fffffff) return fail(SA_ERR_UNSUPPORTED, "k_gemm_i8: grid too large");
  if (c->prof) c->prof->begin(c->stream, kind);
  plaunch(c, k_gemm_i8<NP>, (unsigned)grid, 512, I8Tile<NP>::Lds, a);
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

// Ab of the beta staged in d_beta on the GEMM path: S Ab partials in d_abp
// (quantised at a per-codeword scale: an arbitrary beta, e.g. beta0)
int i8_ab_any(sa_ctx* c, int B, int S) {
  const long long LM = (long long)c->L * c->M;
  int rc = launch_i8_quant<kI8NPB>(c, B, c->d_beta, LM, (int)LM, c->d_bq, c->LMp8, c->d_bsc0);
  if (rc) return rc;
  return launch_gemm_i8<kI8NPB>(c, B, c->d_bq, c->LMp8, c->d_A8, c->np8, c->n, (float*)c->d_abp, (long long)S * c->n,
                        c->n, S, c->d_bsc0, 1, K_DAB);
}

// Az of the z in d_z on the GEMM path into out[b][0 .. L*M) (rows ldb apart)
int i8_az(sa_ctx* c, int B, float* out, long long ldb) {
  int rc = launch_i8_quant<kI8NPZ>(c, B, c->d_z, c->n, c->n, c->d_zq, c->np8, c->d_zsc);
  if (rc) return rc;
  return launch_gemm_i8<kI8NPZ>(c, B, c->d_zq, c->np8, c->d_AT8, c->LMp8, c->L * c->M, out, ldb, 0, 1, c->d_zsc, 1,
                        K_DAZ);
}

// ---- caller's dense matrix on the matrix cores (dense_mfma.hip) ----------
long long f_kstage(const sa_ctx* c) { return kFKB / (long long)rsz(c); }  // K elements per stage

// K splits of the A beta GEMM: the fewest (workgroup rounds x stages per
// workgroup) on n_cus CUs at two workgroups per CU
int fgemm_splits(const sa_ctx* c, int B) {
  const long long tiles = (long long)(c->np / kFTY) * ((B + kFTX - 1) / kFTX);
  const long long nst = (long long)c->lda / f_kstage(c);
  int best = 1;
  long long bcost = -1;
  for (int S = 1; S <= kFMaxS; ++S) {
    const long long rounds = (tiles * S + 2 * c->n_cus - 1) / (2 * c->n_cus);
    const long long cost = rounds * ((nst + S - 1) / S);
    if (bcost < 0 || cost < bcost) { bcost = cost; best = S; }
  }
  return best;
}

// The transposed matrix (first batched use) and the padded GEMM vectors for B codewords.
int ensure_fgemm(sa_ctx* c, int B) {
  if (!use_fgemm(c, B)) return SA_OK;
  const size_t s = rsz(c);
  int rc;
  if (!c->d_AT) {
    if ((rc = dev_alloc(c, &c->d_AT, (size_t)c->LMy * (size_t)c->nk * s))) return rc;
    const dim3 grid((unsigned)((c->LMy + 63) / 64), (unsigned)((c->nk + 63) / 64));
    if (s == 8)
      k_transpose<double><<<grid, 256, 0, c->stream>>>((const double*)c->d_A, (long long)c->lda, c->n,
                                                       (long long)c->L * c->M, (double*)c->d_AT, c->LMy, c->nk);
    else
      k_transpose<float><<<grid, 256, 0, c->stream>>>((const float*)c->d_A, (long long)c->lda, c->n,
                                                      (long long)c->L * c->M, (float*)c->d_AT, c->LMy, c->nk);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  if (B > c->fg_cap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    drop_graphs(c);
    dev_free(c->d_xz); dev_free(c->d_xb);
    c->d_xz = c->d_xb = nullptr;
    c->fg_cap = 0;
    if ((rc = dev_alloc(c, &c->d_xz, (size_t)B * (size_t)c->nk * s))) return rc;
    if ((size_t)c->L * c->M != c->lda && (rc = dev_alloc(c, &c->d_xb, (size_t)B * c->lda * s))) return rc;
    c->fg_cap = B;
  }
  return SA_OK;
}

template <typename real>
int launch_gemm_f(sa_ctx* c, int B, const real* X, long long ldx, const real* Y, long long ldy, long long K,
                  long long Yrows, int Ny, real* out, long long ldb, long long lds, int S, int kind) {
  FArgs<real> a;
  a.X = X; a.Y = Y; a.out = out; a.ldx = ldx; a.ldy = ldy; a.ldb = ldb; a.lds = lds;
  a.nst = (int)(K / f_kstage(c));
  a.kps = (a.nst + S - 1) / S;
  a.XT = (B + kFTX - 1) / kFTX; a.YT = (int)(Yrows / kFTY); a.S = S; a.B = B; a.Ny = Ny;
  if (K % f_kstage(c) || Yrows % kFTY || ldx < K || ldy < K || B > c->fg_cap)
    return fail(SA_ERR_ARG, "k_gemm_f: operand shapes");
  const long long grid = (long long)a.XT * a.YT * S;
  if (grid > 0x7fffffff) return fail(SA_ERR_UNSUPPORTED, "k_gemm_f: grid too large");
  if (c->prof) c->prof->begin(c->stream, kind);
  if (kind == K_DAB)
    plaunch(c, k_gemm_f<real, 1>, (unsigned)grid, 512, kFLds, a);
  else
    plaunch(c, k_gemm_f<real, 0>, (unsigned)grid, 512, kFLds, a);
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

// A beta of the beta in d_beta on the GEMM path: S partials [B][S][n] in d_abp
template <typename real>
int fgemm_ab(sa_ctx* c, int B, int S) {
  const long long LM = (long long)c->L * c->M;
  const real* X = (const real*)c->d_beta;
  if (LM != (long long)c->lda) {  // L*M not a whole number of K stages: a zero-padded copy
    k_pad_rows<real><<<4096, 256, 0, c->stream>>>((const real*)c->d_beta, LM, LM, (real*)c->d_xb, (long long)c->lda,
                                                  B);
    HIP_TRY(hipGetLastError());
    X = (const real*)c->d_xb;
  }
  return launch_gemm_f<real>(c, B, X, (long long)c->lda, (const real*)c->d_A, (long long)c->lda, (long long)c->lda,
                             c->np, c->n, (real*)c->d_abp, (long long)S * c->n, c->n, S, K_DAB);
}

// A^T z of the z in d_z on the GEMM path into out[b][0 .. L*M) (rows ldb apart)
template <typename real>
int fgemm_az(sa_ctx* c, int B, real* out, long long ldb) {
  k_pad_rows<real><<<4096, 256, 0, c->stream>>>((const real*)c->d_z, (long long)c->n, (long long)c->n,
                                                (real*)c->d_xz, c->nk, B);
  HIP_TRY(hipGetLastError());
  return launch_gemm_f<real>(c, B, (const real*)c->d_xz, c->nk, (const real*)c->d_AT, c->nk, c->nk, c->LMy,
                             c->L * c->M, out, ldb, 0, 1, K_DAZ);
}

int build_dense(sa_ctx* c) {
  const int L = c->L, n = c->n, w = c->w, M = c->M;
  c->lda = ((size_t)L * M + 3) / 4 * 4;
  int rc;
  if ((rc = dev_alloc(c, (void**)&c->d_A, (size_t)n * c->lda * sizeof(float)))) return rc;
  uint32_t* d_ord = nullptr;
  HIP_TRY(hipMalloc(&d_ord, c->ordering.size() * 4));
  HIP_TRY(hipMemcpyAsync(d_ord, c->ordering.data(), c->ordering.size() * 4, hipMemcpyHostToDevice, c->stream));
  const float s = (float)(1.0 / std::sqrt((double)n));
  k_dense_build<<<8192, 256, 0, c->stream>>>(d_ord, (float*)c->d_A, L, M, n, w, c->lda, s);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_ord);
  if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("k_dense_build: ") + hipGetErrorString(e));
  return SA_OK;
}

// ---- the dense backends' steps of the AMP sequence (seq_amp / seq_ab / seq_az) ----

// Ab partials of A beta: the GEMM's K splits (B >= 4) or the GEMV's KS splits
int dense_parts(const sa_ctx* c, int B) {
  return use_i8(c, B) ? i8_splits(c, B) : (use_fgemm(c, B) ? fgemm_splits(c, B) : c->KS);
}

// the beta0 start: z = y - A beta0 from the S partials of A beta0
template <typename real>
int dense_start(sa_ctx* c, int B, int S) {
  int rc;
  if (use_i8(c, B)) {
    if ((rc = i8_ab_any(c, B, S))) return rc;
  } else if (use_fgemm(c, B)) {
    if ((rc = fgemm_ab<real>(c, B, S))) return rc;
  } else if ((rc = launch_dense_ab<real>(c, B, 0, 0, 1))) {
    return rc;
  }
  return launch_row<real>(c, B, ROW_INIT, 0, 0, S, c->Gd);
}

// One iteration's operator steps: A^T z -> denoiser -> the S partials of A beta
// (the row kernel that follows is seq_amp's)
template <typename real>
int dense_iter(sa_ctx* c, int B, int t, int es, int S) {
  int rc;
  if (use_i8(c, B)) {
    // z -> digit planes -> Az GEMM (into the dense Az buffer, one partial)
    // -> denoiser (+ beta digit planes) -> A beta GEMM (S partials)
    if ((rc = i8_az(c, B, (float*)c->d_azp, (long long)c->lda))) return rc;
    if ((rc = launch_dense_den<float>(c, B, t, es, true))) return rc;
    return launch_gemm_i8<kI8NPB>(c, B, c->d_bq, c->LMp8, c->d_A8, c->np8, c->n, (float*)c->d_abp,
                                  (long long)S * c->n, c->n, S, c->d_bfix + 1, 0, K_DAB);
  }
  if (use_fgemm(c, B)) {
    // z -> Az GEMM (one partial) -> denoiser -> A beta GEMM (S partials);
    // the GEMMs skip nothing for a stopped codeword: the row kernel keeps
    // its residual and the denoiser its estimate
    if ((rc = fgemm_az<real>(c, B, (real*)c->d_azp, (long long)c->lda))) return rc;
    if ((rc = launch_dense_den<real>(c, B, t, es, false, true))) return rc;
    return fgemm_ab<real>(c, B, S);
  }
  if ((rc = launch_dense_az<real>(c, B, t, es, 0))) return rc;
  if ((rc = launch_dense_den<real>(c, B, t, es))) return rc;
  return launch_dense_ab<real>(c, B, t, es, 0);
}

// A beta of the batch staged in d_beta -> d_out (B x n)
template <typename real>
int dense_ab(sa_ctx* c, int B) {
  int rc;
  if (use_i8(c, B)) {
    const int S = i8_splits(c, B);
    if ((rc = i8_ab_any(c, B, S))) return rc;
    return launch_row<real>(c, B, ROW_ABOUT, 0, 0, S, c->Gd);
  }
  if (use_fgemm(c, B)) {
    const int S = fgemm_splits(c, B);
    if ((rc = fgemm_ab<real>(c, B, S))) return rc;
    return launch_row<real>(c, B, ROW_ABOUT, 0, 0, S, c->Gd);
  }
  if ((rc = launch_dense_ab<real>(c, B, 0, 0, 1))) return rc;
  return launch_row<real>(c, B, ROW_ABOUT, 0, 0, c->KS, c->Gd);
}

// A^T z of the batch staged in d_z -> d_out (B x L*M)
template <typename real>
int dense_az(sa_ctx* c, int B) {
  if constexpr (sizeof(real) == 4)
    if (use_i8(c, B)) return i8_az(c, B, (float*)c->d_out, (long long)c->L * c->M);
  if (use_fgemm(c, B)) return fgemm_az<real>(c, B, (real*)c->d_out, (long long)c->L * c->M);
  int rc = launch_dense_az<real>(c, B, 0, 0, 1);
  if (rc) return rc;
  // the RS row-split partials into d_out
  k_dense_az_reduce<real><<<4096, 256, 0, c->stream>>>((const real*)c->d_azp, (real*)c->d_out, c->RS, c->lda,
                                                       (size_t)c->L * c->M, B);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

template int dense_start<float>(sa_ctx*, int, int);
template int dense_start<double>(sa_ctx*, int, int);
template int dense_iter<float>(sa_ctx*, int, int, int, int);
template int dense_iter<double>(sa_ctx*, int, int, int, int);
template int dense_ab<float>(sa_ctx*, int);
template int dense_ab<double>(sa_ctx*, int);
template int dense_az<float>(sa_ctx*, int);
template int dense_az<double>(sa_ctx*, int);

// A caller's matrix (SA_BACKEND_MATRIX, uploaded by sa_create_matrix): rows of
// whole GEMM K stages (128 B), padded to whole 256-row tiles, zero padding
int matrix_init(sa_ctx* c) {
  const size_t s = rsz(c);
  const long long ks = kFKB / (long long)s;
  c->lda = (size_t)(((long long)c->L * c->M + ks - 1) / ks * ks);
  c->np = ((long long)c->n + kFTY - 1) / kFTY * kFTY;
  c->nk = ((long long)c->n + ks - 1) / ks * ks;
  c->LMy = ((long long)c->L * c->M + kFTY - 1) / kFTY * kFTY;
  int rc = dev_alloc(c, &c->d_A, (size_t)c->np * c->lda * s);
  if (rc) return rc;
  HIP_TRY(hipMemsetAsync(c->d_A, 0, (size_t)c->np * c->lda * s, c->stream));
  return SA_OK;
}

// the MFMA GEMMs' LDS staging buffers
hipError_t dense_lds_attrs() {
  hipError_t e = hipFuncSetAttribute((const void*)k_gemm_i8<kI8NPZ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     I8Tile<kI8NPZ>::Lds);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_gemm_i8<kI8NPB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            I8Tile<kI8NPB>::Lds);
  const void* fs[] = {(const void*)k_gemm_f<float, 0>, (const void*)k_gemm_f<float, 1>,
                      (const void*)k_gemm_f<double, 0>, (const void*)k_gemm_f<double, 1>};
  for (const void* f : fs)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kFLds);
  return e;
}

}  // namespace sa

using namespace sa;

extern "C" {

int sa_create_matrix(sa_ctx** out, int L, int M, int n, const double* A, int precision, int device) {
  if (!out) return fail(SA_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (!A) return fail(SA_ERR_ARG, "A is NULL");
  sa_ctx* c = nullptr;
  int rc = create_impl(&c, L, M, n, nullptr, SA_BACKEND_MATRIX, precision, device, SA_PLAN_DEFAULT);
  if (rc) return rc;
  // the n x (L*M) row-major binary64 matrix in chunks of rows through the
  // staging buffer (at most 32 M values), converted on the device
  const long long LM = (long long)L * M;
  const long long chunk = std::max(1LL, std::min<long long>(n, (32LL << 20) / LM));
  rc = ensure_stage(c, (size_t)(chunk * LM));
  for (long long r0 = 0; !rc && r0 < n; r0 += chunk) {
    const long long rows = std::min<long long>(chunk, n - r0);
    hipError_t e = hipMemcpyAsync(c->d_stage, A + r0 * LM, (size_t)(rows * LM) * 8, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
      if (c->prec == SA_PREC_F64)
        k_matrix_rows<double><<<4096, 256, 0, c->stream>>>(c->d_stage, (double*)c->d_A, rows, LM, c->lda, r0);
      else
        k_matrix_rows<float><<<4096, 256, 0, c->stream>>>(c->d_stage, (float*)c->d_A, rows, LM, c->lda, r0);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the staging buffer is reused
    if (e != hipSuccess) rc = fail(SA_ERR_HIP, std::string("sa_create_matrix upload: ") + hipGetErrorString(e));
  }
  if (rc) {
    sa_destroy(c);
    return rc;
  }
  *out = c;
  return SA_OK;
}

int sa_create_matrix_random(sa_ctx** out, int L, int M, int n, uint64_t seed, double scale, int precision,
                            int device) {
  if (!out) return fail(SA_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (!std::isfinite(scale)) return fail(SA_ERR_ARG, "scale must be finite");
  sa_ctx* c = nullptr;
  int rc = create_impl(&c, L, M, n, nullptr, SA_BACKEND_MATRIX, precision, device, SA_PLAN_DEFAULT);
  if (rc) return rc;
  const long long LM = (long long)L * M;
  if (c->prec == SA_PREC_F64)
    k_matrix_gauss<double><<<8192, 256, 0, c->stream>>>((double*)c->d_A, n, LM, c->lda, (unsigned long long)seed,
                                                         scale);
  else
    k_matrix_gauss<float><<<8192, 256, 0, c->stream>>>((float*)c->d_A, n, LM, c->lda, (unsigned long long)seed,
                                                        scale);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    sa_destroy(c);
    return fail(SA_ERR_HIP, std::string("k_matrix_gauss: ") + hipGetErrorString(e));
  }
  *out = c;
  return SA_OK;
}

// ---- host-operator AMP (SA_BACKEND_HOST): the caller's Ab / Az ----------
extern "C++" {
namespace {
int check_host(sa_ctx* c, int B, const char* what) {
  if (!c) return fail(SA_ERR_ARG, "null context");
  if (c->backend != SA_BACKEND_HOST)
    return fail(SA_ERR_UNSUPPORTED, std::string(what) + ": needs a host-operator context (SA_BACKEND_HOST)");
  if (B <= 0 || B > c->Bcap) return fail(SA_ERR_ARG, std::string(what) + ": bad batch (sa_host_init first)");
  return SA_OK;
}

template <typename real>
int host_init_impl(sa_ctx* c, int B, const double* beta0, const double* ab0) {
  int rc;
  pick_row(c, B);
  k_fill32<<<(B + 255) / 256, 256, 0, c->stream>>>((uint32_t*)c->d_iters, 0xffffffffu, (size_t)B);
  if (beta0) {  // z = y - Ab(beta0) with the caller's Ab(beta0) (sparc_ldpc.py:196-200)
    if ((rc = upload(c, c->d_beta, beta0, (size_t)B * c->L * c->M))) return rc;
    if ((rc = upload(c, c->d_abp, ab0, (size_t)B * c->n))) return rc;
    return launch_row<real>(c, B, ROW_INIT, 0, 0, 1, c->Gd);
  }
  const size_t nw = (size_t)B * c->L * c->M * rsz(c) / 4;
  k_fill32<<<(int)std::min<size_t>((nw + 255) / 256, 8192), 256, 0, c->stream>>>((uint32_t*)c->d_beta, 0u, nw);
  return launch_row<real>(c, B, ROW_INIT0, 0, 0, 1, c->Gd);
}
}  // namespace
}  // extern "C++"

int sa_host_init(sa_ctx* c, int B, int T, const double* y, const double* Pl, const double* beta0, const double* ab0) {
  if (!c) return fail(SA_ERR_ARG, "null context");
  if (c->backend != SA_BACKEND_HOST) return fail(SA_ERR_UNSUPPORTED, "sa_host_init: needs a host-operator context");
  if (B <= 0 || T < 0 || !y || !Pl || (!beta0) != (!ab0))
    return fail(SA_ERR_ARG, "sa_host_init: bad arguments (beta0 and Ab(beta0) go together)");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, T > 0 ? T : 1);
  if (!rc) rc = set_power(c, Pl);
  if (!rc) rc = upload(c, c->d_y, y, (size_t)B * c->n);
  if (rc) return rc;
  rc = c->prec == SA_PREC_F64 ? host_init_impl<double>(c, B, beta0, ab0) : host_init_impl<float>(c, B, beta0, ab0);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

int sa_host_tau(sa_ctx* c, int B, int t, int flags, int* stopped) {
  if (int rc = check_host(c, B, "sa_host_tau")) return rc;
  if (t < 0 || t >= c->Tcap || !stopped) return fail(SA_ERR_ARG, "sa_host_tau: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  const int es = (flags & SA_FLAG_NO_EARLY_STOP) ? 0 : 1;
  if (c->prec == SA_PREC_F64)
    k_tau<double><<<B, 64, 0, c->stream>>>((const double*)c->d_zzp, c->nz_cur, c->n, (double*)c->d_tau, c->Tcap + 1,
                                            t, es, c->d_iters, c->d_stop);
  else
    k_tau<float><<<B, 64, 0, c->stream>>>((const float*)c->d_zzp, c->nz_cur, c->n, (float*)c->d_tau, c->Tcap + 1,
                                           t, es, c->d_iters, c->d_stop);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(stopped, c->d_stop, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_host_eta(sa_ctx* c, int B, int t, int flags, const double* az) {
  if (int rc = check_host(c, B, "sa_host_eta")) return rc;
  if (t < 0 || t >= c->Tcap || !az) return fail(SA_ERR_ARG, "sa_host_eta: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  const int es = (flags & SA_FLAG_NO_EARLY_STOP) ? 0 : 1;
  int rc = upload(c, c->d_azp, az, (size_t)B * c->L * c->M);
  if (!rc) rc = c->prec == SA_PREC_F64 ? launch_dense_den<double>(c, B, t, es) : launch_dense_den<float>(c, B, t, es);
  return rc;
}

int sa_host_residual(sa_ctx* c, int B, int t, int flags, const double* ab) {
  if (int rc = check_host(c, B, "sa_host_residual")) return rc;
  if (t < 0 || t >= c->Tcap || !ab) return fail(SA_ERR_ARG, "sa_host_residual: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  const int es = (flags & SA_FLAG_NO_EARLY_STOP) ? 0 : 1;
  int rc = upload(c, c->d_abp, ab, (size_t)B * c->n);
  if (!rc)
    rc = c->prec == SA_PREC_F64 ? launch_row<double>(c, B, ROW_AMP, t, es, 1, c->Gd)
                                : launch_row<float>(c, B, ROW_AMP, t, es, 1, c->Gd);
  return rc;
}

}  // extern "C"
