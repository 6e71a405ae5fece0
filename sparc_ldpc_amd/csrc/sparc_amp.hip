// sparc_amp.hip — MI355X (gfx950) SPARC AMP decoder: kernels + C ABI.
//
// Hot path of Spimp/sparc_ldpc: the amp() loop of ldpc/sparc_ldpc.py:189-222
// over the sub-sampled Walsh-Hadamard design operator of
// ldpc/sparc_ldpc.py:32-147.  See DESIGN.md for the derivation; in short, for
// M a power of two and w = 2^ceil(log2(max(M+1, n+1))) the block of section l
// factorises as
//     A_l[r, c] = sgn(o >> log2 M) * H_M[o & (M-1), c] / sqrt(n),
//     o = ordering[l, r],  sgn(h) = (-1)^popcount(h),
// because the reference keeps the LAST M columns (w-M+c, :68/:77) of the
// natural-order Hadamard H_w, whose high index bits are all ones.  So
//     Az_l = H_M v_l / sqrt(n),  v_l[k] = sum_h sgn(h) z[inv_l[h*M + k]]
//     Ab[r] = sum_l sgn(o_lr >> log2 M) (H_M beta_l)[o_lr & (M-1)] / sqrt(n)
// with inv_l the inverse of ordering row l (sentinel n -> a zero slot).
// Per section that is one M-point FWHT (in registers + cross-lane shuffles,
// one wavefront per section) plus gathers from LDS, instead of the
// reference's w-point FWHT; no n x (L*M) matrix is ever formed.
//
// A second backend materialises the fp32 n x (L*M) matrix and streams it as
// a GEMV pair (the HBM-roofline formulation of BASELINE.json's north_star).
//
// One AMP iteration = two launches (section kernel, row kernel) replayed from
// a hipGraph captured once per (B, T, flags).  All reductions are in a fixed
// order, so results are bitwise reproducible run to run.

// 0.3: sa_profile / sa_profile_rep write 2 * sa_profile_kinds() + 1 doubles (13 since 0.2)
// 0.4: sa_profile_dispatch (dispatch-bound event pairs), sa_decide_async / sa_decide_collect
#define SA_VERSION "sparc_amp 0.4 gfx950"

#include "sa_host.h"

namespace sa {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

template <typename src_t, typename dst_t>
__global__ void k_convert(const src_t* s, dst_t* d, size_t N) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = (dst_t)s[i];
}

// Word fill used inside captured sequences instead of hipMemsetAsync (keeps
// the graphs made of kernel nodes only).
__global__ void k_fill32(uint32_t* p, uint32_t v, size_t nw) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// Fused path: the final residual of a codeword lies in the buffer of parity
// iters[b] (z double-buffered); bring it home to z (one codeword).
template <typename real>
__global__ void k_beta_final(real* beta, const real* beta2, const int* it, size_t LM) {
  const int b = blockIdx.y;
  if (!(it[b] & 1)) return;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < LM; i += (size_t)gridDim.x * blockDim.x)
    beta[(size_t)b * LM + i] = beta2[(size_t)b * LM + i];
}

__global__ void k_iters_final(int* it, int B, int T) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B && it[b] < 0) it[b] = T;
}


int dev_alloc(sa_ctx* c, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(SA_ERR_NOMEM, "hipMalloc(" + std::to_string(bytes) + ") failed: " + hipGetErrorString(e));
  }
  c->bytes += bytes;
  return SA_OK;
}

void dev_free(void* p) {
  if (p) (void)hipFree(p);
}

void drop_graphs(sa_ctx* c) {
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  c->graphs.clear();
  for (auto& kv : c->mc_graphs) (void)hipGraphExecDestroy(kv.second);  // sa_mc_run's
  c->mc_graphs.clear();
}

void free_workspace(sa_ctx* c) {
  void** bufs[] = {&c->d_y, &c->d_z, &c->d_beta, &c->d_out, &c->d_abp, &c->d_bbp,
                   &c->d_zzp, &c->d_tau, &c->d_azp, &c->d_cb, &c->d_Pb};
  for (void** p : bufs) {
    dev_free(*p);
    *p = nullptr;
  }
  dev_free(c->d_iters); c->d_iters = nullptr;
  dev_free(c->d_stop); c->d_stop = nullptr;
  dev_free(c->d_idx); c->d_idx = nullptr;
  dev_free(c->d_beta2); c->d_beta2 = nullptr;
  c->beta2_cap = 0;
  c->Bcap = c->Tcap = 0;
  if (c->pb_on) {  // the per-codeword powers went with the workspace
    c->pb_on = false;
    c->power_set = c->shared_power;
  }
}


int ensure_fgemm(sa_ctx* c, int B);

int ensure_workspace(sa_ctx* c, int B, int T) {
  if (c->backend == SA_BACKEND_DENSE) {
    int rc8 = ensure_i8(c, B > c->Bcap ? B : c->Bcap);
    if (rc8) return rc8;
  }
  if (c->backend == SA_BACKEND_MATRIX) {
    int rcf = ensure_fgemm(c, B > c->Bcap ? B : c->Bcap);
    if (rcf) return rcf;
  }
  if (B <= c->Bcap && T <= c->Tcap) return SA_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  drop_graphs(c);
  const int nB = B > c->Bcap ? B : c->Bcap;
  const int nT = T > c->Tcap ? T : c->Tcap;
  free_workspace(c);
  const size_t s = rsz(c), LM = (size_t)c->L * c->M;
  int Gmax = c->G > c->KS ? c->G : c->KS;
  if (c->backend == SA_BACKEND_DENSE && Gmax < kI8MaxS) Gmax = kI8MaxS;
  if (c->backend == SA_BACKEND_MATRIX && Gmax < kFMaxS) Gmax = kFMaxS;
  if (c->Gb > Gmax) Gmax = c->Gb;
  if (c->G2 > Gmax) Gmax = c->G2;
  if (c->G3 > Gmax) Gmax = c->G3;
  int rc;
  if ((rc = dev_alloc(c, &c->d_y, nB * c->n * s))) return rc;
  const size_t nBp = (size_t)(nB + 3) / 4 * 4;  // whole chunks of the interleaved batched layout
  if ((rc = dev_alloc(c, &c->d_z, nBp * c->n * s))) return rc;
  if ((rc = dev_alloc(c, &c->d_beta, nB * LM * s))) return rc;
  if ((rc = dev_alloc(c, &c->d_out, nB * (LM > (size_t)c->n ? LM : (size_t)c->n) * s))) return rc;
  // rows padded to 32: the row-block-major layout of the pair / triple kernels (SecArgs::pt)
  if ((rc = dev_alloc(c, &c->d_abp, nBp * Gmax * ((size_t)c->NZ16 * kRow2Rows) * s))) return rc;
  if ((rc = dev_alloc(c, &c->d_bbp, (size_t)nB * Gmax * s))) return rc;
  if ((rc = dev_alloc(c, &c->d_zzp, (size_t)nB * c->NZh * s))) return rc;
  if ((rc = dev_alloc(c, &c->d_tau, (size_t)nB * (nT + 1) * s))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->d_iters, (size_t)nB * sizeof(int)))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->d_stop, (size_t)nB * sizeof(int)))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->d_idx, (size_t)nB * c->L * sizeof(int32_t)))) return rc;
  if ((rc = dev_alloc(c, &c->d_cb, (size_t)nB * c->L * s))) return rc;
  if ((rc = dev_alloc(c, &c->d_Pb, (size_t)nB * s))) return rc;
  if (is_dense(c))
    if ((rc = dev_alloc(c, &c->d_azp, (size_t)nB * c->RS * c->lda * s))) return rc;
  if (c->backend == SA_BACKEND_HOST)  // the caller's A^T z, one partial per codeword
    if ((rc = dev_alloc(c, &c->d_azp, (size_t)nB * c->lda * s))) return rc;
  c->Bcap = nB;
  c->Tcap = nT;
  return SA_OK;
}

int ensure_stage(sa_ctx* c, size_t count) {
  if (count <= c->stage_cap) return SA_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  dev_free(c->d_stage);
  c->d_stage = nullptr;
  int rc = dev_alloc(c, (void**)&c->d_stage, count * sizeof(double));
  if (rc) return rc;
  c->stage_cap = count;
  return SA_OK;
}

// Host fp64 -> device `real` buffer (through the fp64 staging buffer).
int upload(sa_ctx* c, void* dst, const double* src, size_t count) {
  if (c->prec == SA_PREC_F64) {
    HIP_TRY(hipMemcpyAsync(dst, src, count * 8, hipMemcpyHostToDevice, c->stream));
    return SA_OK;
  }
  int rc = ensure_stage(c, count);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, src, count * 8, hipMemcpyHostToDevice, c->stream));
  const int blocks = (int)((count + 255) / 256 < 4096 ? (count + 255) / 256 : 4096);
  k_convert<double, float><<<blocks > 0 ? blocks : 1, 256, 0, c->stream>>>(c->d_stage, (float*)dst, count);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

int download(sa_ctx* c, double* dst, const void* src, size_t count) {
  if (c->prec == SA_PREC_F64) {
    HIP_TRY(hipMemcpyAsync(dst, src, count * 8, hipMemcpyDeviceToHost, c->stream));
    return SA_OK;
  }
  int rc = ensure_stage(c, count);
  if (rc) return rc;
  const int blocks = (int)((count + 255) / 256 < 4096 ? (count + 255) / 256 : 4096);
  k_convert<float, double><<<blocks > 0 ? blocks : 1, 256, 0, c->stream>>>((const float*)src, c->d_stage, count);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(dst, c->d_stage, count * 8, hipMemcpyDeviceToHost, c->stream));
  return SA_OK;
}



// ---- composite sequences (all asynchronous on c->stream) ----------------

// Ab of the batch staged in d_beta -> d_out  (B x n)
template <typename real>
int seq_ab(sa_ctx* c, int B) {
  if (is_dense(c)) return dense_ab<real>(c, B);
  int rc;
  if ((rc = launch_sec<real>(c, B, SEC_AB, 0, 0))) return rc;
  return launch_row<real>(c, B, ROW_ABOUT, 0, 0, c->G, c->G);
}

// Az of the batch staged in d_z -> d_out  (B x L*M)
template <typename real>
int seq_az(sa_ctx* c, int B) {
  if (is_dense(c)) return dense_az<real>(c, B);
  return launch_sec<real>(c, B, SEC_AZ, 0, 0);
}

// Whole AMP decode of the staged batch: y in d_y, beta0 in d_beta if has_b0.
template <typename real>
int seq_amp(sa_ctx* c, int B, int T, int flags, int has_b0) {
  const int es = (flags & SA_FLAG_NO_EARLY_STOP) ? 0 : 1;
  const bool dense = is_dense(c);
  const bool batched = !dense && use_batched(c, B);
  const bool sec2 = use_sec2(c, B);
  pick_row(c, B);  // row kernel and its z^2 partial count
  c->zil_last = zil_for(c, B);
  // Ab partials row-block major between the pair / triple kernels and k_row2
  const int pt = pt_for(c, B, sec2);
  // partial counts of the producer of abp (Ab) and bbp (beta^2)
  const int G = dense ? dense_parts(c, B) : (batched ? c->Gb : (sec2 ? sec2_parts(c) : c->G));
  const int Gb = dense ? c->Gd : (batched ? c->Gb : (sec2 ? sec2_parts(c) : c->G));
  int rc;
  k_fill32<<<(B + 255) / 256, 256, 0, c->stream>>>((uint32_t*)c->d_iters, 0xffffffffu, (size_t)B);
  if (has_b0) {
    if (dense) {
      if ((rc = dense_start<real>(c, B, G))) return rc;
    } else {
      if ((rc = launch_sec<real>(c, B, SEC_AB, 0, 0))) return rc;
      if ((rc = launch_row<real>(c, B, ROW_INIT, 0, 0, c->G, c->G))) return rc;
    }
  } else {
    const size_t nw = (size_t)B * c->L * c->M * rsz(c) / 4;
    k_fill32<<<(int)std::min<size_t>((nw + 255) / 256, 8192), 256, 0, c->stream>>>((uint32_t*)c->d_beta, 0u, nw);
    if ((rc = launch_row<real>(c, B, ROW_INIT0, 0, 0, G, Gb))) return rc;
  }
  for (int t = 0; t < T; ++t) {
    if (dense) {
      if ((rc = dense_iter<real>(c, B, t, es, G))) return rc;
    } else if (batched) {
      if ((rc = launch_secb<real>(c, B, t, es))) return rc;
    } else {
      void* pin = (t & 1) ? c->d_beta2 : c->d_beta;
      void* pout = (t & 1) ? c->d_beta : c->d_beta2;
      if (sec2) {
        if ((rc = launch_sec2<real>(c, B, t, es, pin, pout, pt))) return rc;
      } else if ((rc = launch_sec<real>(c, B, SEC_AMP, t, es, pin, pout))) {
        return rc;
      }
    }
    if ((rc = launch_row<real>(c, B, ROW_AMP, t, es, G, Gb, pt))) return rc;
  }
  k_iters_final<<<(B + 255) / 256, 256, 0, c->stream>>>(c->d_iters, B, T);
  HIP_TRY(hipGetLastError());
  if (!dense && !batched && T > 0) {
    // the estimate of codeword b is in the buffer of parity iters[b]
    const size_t LM = (size_t)c->L * c->M;
    k_beta_final<real><<<dim3((unsigned)std::min<size_t>((LM + 255) / 256, 4096), B), 256, 0, c->stream>>>(
        (real*)c->d_beta, (const real*)c->d_beta2, c->d_iters, LM);
    HIP_TRY(hipGetLastError());
  }
  return SA_OK;
}

int ensure_beta2(sa_ctx* c, int B) {
  if (is_dense(c) || use_batched(c, B) || c->beta2_cap >= c->Bcap) return SA_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  dev_free(c->d_beta2);
  c->d_beta2 = nullptr;
  c->beta2_cap = 0;
  int rc = dev_alloc(c, &c->d_beta2, (size_t)c->Bcap * c->L * c->M * rsz(c));
  if (rc) return rc;
  c->beta2_cap = c->Bcap;
  drop_graphs(c);  // captured graphs hold the old pointer
  return SA_OK;
}

int ensure_invb(sa_ctx* c);

template <typename real>
int run_graph(sa_ctx* c, int B, int T, int flags, int has_b0) {
  int rc0 = ensure_beta2(c, B);
  if (!rc0 && use_batched(c, B)) rc0 = ensure_invb(c);  // before any capture: it uploads
  if (rc0) return rc0;
  if (c->plan & SA_PLAN_EAGER) {  // eager launches instead of the captured graph
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    int rc = seq_amp<real>(c, B, T, flags, has_b0);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    c->last_B = B;
    c->last_T = T;
    c->zil_last = zil_for(c, B);
    return SA_OK;
  }
  // the power-allocation mode selects the captured kernel arguments (c, P arrays)
  const auto key = std::make_tuple(B, T, flags | (c->pb_on ? 0x10000 : 0), has_b0);
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) {
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    int rc = seq_amp<real>(c, B, T, flags, has_b0);
    hipGraph_t cap = nullptr;
    hipError_t e = hipStreamEndCapture(c->stream, &cap);
    if (rc) {
      if (cap) (void)hipGraphDestroy(cap);
      return rc;
    }
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    g = cap;
    hipGraphExec_t ex = nullptr;
    e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    it = c->graphs.emplace(key, ex).first;
  }
  HIP_TRY(hipEventRecord(c->ev0, c->stream));
  HIP_TRY(hipGraphLaunch(it->second, c->stream));
  HIP_TRY(hipEventRecord(c->ev1, c->stream));
  c->last_B = B;
  c->last_T = T;
  c->zil_last = zil_for(c, B);  // the layout d_z is left in by THIS run (a cached graph does not run seq_amp)
  return SA_OK;
}

int check_ctx(const sa_ctx* c) {
  if (!c) return fail(SA_ERR_ARG, "null context");
  return SA_OK;
}

// Entry points that read the Hadamard design's tables (the row-parallel
// encoder and cancellation: one table entry per section and row).
int check_tables(const sa_ctx* c, const char* what) {
  if (!c) return fail(SA_ERR_ARG, "null context");
  if (c->backend != SA_BACKEND_HADAMARD && c->backend != SA_BACKEND_DENSE)
    return fail(SA_ERR_UNSUPPORTED, std::string(what) + ": needs a design built from an ordering "
                                                        "(use sa_Ab for a caller's matrix)");
  return SA_OK;
}

// Entry points that apply the design operator on the device: not on a
// host-operator context (SA_BACKEND_HOST holds no operator).
int check_op(const sa_ctx* c, const char* what) {
  if (!c) return fail(SA_ERR_ARG, "null context");
  if (c->backend == SA_BACKEND_HOST)
    return fail(SA_ERR_UNSUPPORTED, std::string(what) + ": a host-operator context has no device operator");
  return SA_OK;
}

// The caller's section vectors [B][L][Mu] <-> the device's padded layout
// [B][L][M] (a padded section's dead leading columns zero); identity when M
// is the caller's.
int upload_sections(sa_ctx* c, void* dst, const double* src, int B) {
  const size_t LM = (size_t)c->L * c->M;
  if (c->dead == 0) return upload(c, dst, src, (size_t)B * LM);
  std::vector<double> pad((size_t)B * LM, 0.0);
  for (size_t bl = 0; bl < (size_t)B * c->L; ++bl)
    std::memcpy(pad.data() + bl * c->M + c->dead, src + bl * c->Mu, (size_t)c->Mu * sizeof(double));
  int rc = upload(c, dst, pad.data(), pad.size());
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));  // pad is a host temporary
  return SA_OK;
}

int download_sections(sa_ctx* c, double* dst, const void* src, int B) {
  const size_t LM = (size_t)c->L * c->M;
  if (c->dead == 0) return download(c, dst, src, (size_t)B * LM);
  std::vector<double> pad((size_t)B * LM);
  int rc = download(c, pad.data(), src, pad.size());
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (size_t bl = 0; bl < (size_t)B * c->L; ++bl)
    std::memcpy(dst + bl * c->Mu, pad.data() + bl * c->M + c->dead, (size_t)c->Mu * sizeof(double));
  return SA_OK;
}

int set_power(sa_ctx* c, const double* Pl) {
  if (!Pl) return fail(SA_ERR_ARG, "Pl is NULL");
  std::vector<double> cl(c->L);
  double P = 0;
  for (int l = 0; l < c->L; ++l) {
    if (!(Pl[l] >= 0)) return fail(SA_ERR_ARG, "Pl must be non-negative");
    cl[l] = std::sqrt((double)c->n * Pl[l]);  // np.sqrt(n*Pl), sparc_ldpc.py:214
    P += Pl[l];                                // np.sum(Pl), sparc_ldpc.py:190
  }
  c->P = P;
  c->cmax = 0;
  for (int l = 0; l < c->L; ++l) c->cmax = cl[l] > c->cmax ? cl[l] : c->cmax;
  int rc = upload(c, c->d_c, cl.data(), c->L);
  if (!rc) rc = upload(c, c->d_P1, &P, 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_cd, cl.data(), (size_t)c->L * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));  // cl is a host temporary
  c->pb_on = false;  // back to one allocation (graphs are keyed on the mode)
  c->shared_power = true;
  c->power_set = true;
  if (c->d_bfix && (rc = i8_set_bfix(c))) return rc;
  return SA_OK;
}

// Per-codeword power allocations Pl [B][L] for the next runs of B' <= B
// codewords (c_{b,l} = sqrt(n Pl_{b,l}), P_b = sum_l Pl_{b,l}).  A section with
// Pl = 0 has c = 0, so its estimate stays exactly 0 (beta = c e / S) and it
// adds nothing to A beta or to sum(beta^2): AMP over the remaining sections
// with the same n, i.e. the reference's sparc_transforms_shorter decode
// (amp_exit.py:113-116) as a mask, per codeword, in one batch.
int set_power_batch(sa_ctx* c, int B, const double* Pl) {
  if (!Pl) return fail(SA_ERR_ARG, "Pl is NULL");
  if (is_dense(c)) return fail(SA_ERR_UNSUPPORTED, "per-codeword power: Hadamard backend only");
  const size_t L = (size_t)c->L;
  std::vector<double> cb((size_t)B * L), Pb(B);
  for (int b = 0; b < B; ++b) {
    double P = 0;
    for (size_t l = 0; l < L; ++l) {
      const double p = Pl[(size_t)b * L + l];
      if (!(p >= 0)) return fail(SA_ERR_ARG, "Pl must be non-negative");
      cb[(size_t)b * L + l] = std::sqrt((double)c->n * p);
      P += p;
    }
    Pb[b] = P;
  }
  int rc = upload(c, c->d_cb, cb.data(), (size_t)B * L);
  if (!rc) rc = upload(c, c->d_Pb, Pb.data(), (size_t)B);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->pb_on = true;
  c->power_set = true;
  return SA_OK;
}

// Tables of a k_secg operator: the bucket table with 32-bit row entries and
// the 4-section Ab table (k | sign << 15 per row, any n).
int build_tables_big(sa_ctx* c) {
  const int L = c->L, n = c->n, w = c->w, M = c->M;
  const int lgM = ilog2(M);
  std::vector<uint32_t> inv((size_t)L * w, (uint32_t)n);
  const int G = (L + kSG - 1) / kSG * (kSG / kSpw);
  std::vector<uint16_t> fwd((size_t)G * n * kSpw, 0);
  for (int l = 0; l < L; ++l) {
    const uint32_t* o = c->ordering.data() + (size_t)l * n;
    uint32_t* il = inv.data() + (size_t)l * w;
    for (int r = 0; r < n; ++r) {
      const uint32_t v = o[r];
      if (v == 0 || v >= (uint32_t)w)
        return fail(SA_ERR_ORDERING, "ordering[" + std::to_string(l) + "," + std::to_string(r) +
                                         "] = " + std::to_string(v) + " outside [1, w=" + std::to_string(w) + ")");
      if (il[v] != (uint32_t)n)
        return fail(SA_ERR_ORDERING, "ordering row " + std::to_string(l) + " repeats value " + std::to_string(v));
      il[v] = (uint32_t)r;
      const uint32_t hi = v >> lgM;
      fwd[((size_t)(l / kSpw) * n + r) * kSpw + (l % kSpw)] =
          (uint16_t)((v & (uint32_t)(M - 1)) | ((__builtin_popcount(hi) & 1u) << 15));
    }
  }
  int rc;
  if ((rc = dev_alloc(c, (void**)&c->d_inv32, inv.size() * 4))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->d_fwd, fwd.size() * 2))) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_inv32, inv.data(), inv.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_fwd, fwd.data(), fwd.size() * 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int build_tables(sa_ctx* c) {
  const int L = c->L, n = c->n, w = c->w, M = c->M;
  const int lgM = ilog2(M);
  if (c->big) return build_tables_big(c);
  std::vector<uint16_t> inv((size_t)L * w, (uint16_t)n);
  const int G = (L + kSG - 1) / kSG * (kSG / kSpw);  // padded to whole batched groups
  std::vector<uint16_t> fwd((size_t)G * n * kSpw, 0);  // [G][n][4]; missing sections -> (k 0, +)
  std::vector<uint32_t> fwd2((size_t)((L + 1) / 2) * n, 0);  // [L/2][n] section pairs
  std::vector<uint32_t> fwd3(c->sec3 ? (size_t)c->G3 * n : 0, 0);  // [L/3][n] section triples
  // sections in blocks of 12 over the host's cores (a pair / triple word is
  // filled by one block); the first bad entry of each section is reported
  std::vector<std::string> bad((size_t)L);
  parallel_for(L, 12, [&](int l) {
    const uint32_t* o = c->ordering.data() + (size_t)l * n;
    uint16_t* il = inv.data() + (size_t)l * w;
    for (int r = 0; r < n; ++r) {
      const uint32_t v = o[r];
      if (v == 0 || v >= (uint32_t)w) {
        bad[l] = "ordering[" + std::to_string(l) + "," + std::to_string(r) + "] = " + std::to_string(v) +
                 " outside [1, w=" + std::to_string(w) + ")";
        return;
      }
      if (il[v] != (uint16_t)n) {
        bad[l] = "ordering row " + std::to_string(l) + " repeats value " + std::to_string(v);
        return;
      }
      il[v] = (uint16_t)r;
      const uint32_t hi = v >> lgM;
      const uint16_t e = (uint16_t)((v & (uint32_t)(M - 1)) | ((__builtin_popcount(hi) & 1u) << 15));
      fwd[((size_t)(l / kSpw) * n + r) * kSpw + (l % kSpw)] = e;
      fwd2[(size_t)(l / 2) * n + r] |= (uint32_t)e << (16 * (l & 1));
      if (c->sec3)  // M <= 512: k in 9 bits, the sign in bit 9 of a 10-bit field
        fwd3[(size_t)(l / 3) * n + r] |= (uint32_t)((e & 0x1ffu) | ((e >> 15) << 9)) << (10 * (l % 3));
    }
  });
  for (int l = 0; l < L; ++l)
    if (!bad[l].empty()) return fail(SA_ERR_ORDERING, bad[l]);
  int rc;
  if ((rc = dev_alloc(c, (void**)&c->d_inv, inv.size() * 2))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->d_fwd, fwd.size() * 2))) return rc;
  if ((rc = dev_alloc(c, (void**)&c->d_fwd2, fwd2.size() * 4))) return rc;
  if (c->sec3 && (rc = dev_alloc(c, (void**)&c->d_fwd3, fwd3.size() * 4))) return rc;
  // On the context's (non-blocking) stream and waited for: a pageable
  // hipMemcpy may return once the data is staged, before the DMA lands, and
  // the null stream does not order the kernels of a non-blocking stream.
  HIP_TRY(hipMemcpyAsync(c->d_inv, inv.data(), inv.size() * 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_fwd, fwd.data(), fwd.size() * 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_fwd2, fwd2.data(), fwd2.size() * 4, hipMemcpyHostToDevice, c->stream));
  if (c->sec3)
    HIP_TRY(hipMemcpyAsync(c->d_fwd3, fwd3.data(), fwd3.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->backend == SA_BACKEND_HADAMARD && c->CB > 0) {  // kept for the batched tables (ensure_invb)
    c->h_inv = std::move(inv);
    c->h_fwd = std::move(fwd);
  }
  return SA_OK;
}

// ---- bank-aware bucket order --------------------------------------------
// The batched section kernel gathers z from LDS, one read per (bucket step,
// element) for a whole wave: 64 random row addresses, served in fixed lane
// groups (MI355X_MICROARCH.md §LDS) where each extra distinct address on a
// busy bank adds one LDS cycle.  k_secb reads 16-byte rows of CB codewords
// (ds_read_b128: four 16-lane groups, 16 bank groups = row % 16).  Visited in
// h order the c3 gather took 2.30 LDS cycles per lane group.  (The same
// order for the single-codeword kernels' 4-byte reads — two 32-lane groups,
// 32 banks — measured neutral: those kernels are latency-bound)  The sum of a
// bucket column k over its slots h does not depend on the order of the
// slots, so these tables re-order them: the slots of sign +1 (popcount(h)
// even) fill steps 0 .. nhi/2 - 1, those of sign -1 steps nhi/2 .. nhi - 1
// (the sign stays uniform per step), and within each half a local search
// swaps a column's slots between steps to minimise, per lane group, the
// largest number of distinct rows on one bank (c3: 1.1 cycles per group
// instead of 2.3).  Empty slots read one of `nbank` zero rows n .. n+nbank-1,
// the one on the step's least loaded bank (all empty lanes of a group read the
// same row: a broadcast).  Seeded per section: the table, and every decode,
// is reproducible.
constexpr int kLdsGroups16[4][16] = {  // ds_read_b128
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

// sets: nsets x gsize columns read by one lane group of one read
// instruction; writes out[h * M + k] (h < nhi) for every column of the sets
void banked_section(const sa_ctx* c, int l, const uint16_t* inv_l, uint16_t* out, const std::vector<int>& sets,
                    int gsize, int nbank, uint32_t* hs, int kh) {
  const int M = c->M, n = c->n, Sh = c->nhi / 2;
  const int nsets = (int)sets.size() / gsize;
  std::mt19937 rng(0x5eed0000u + (uint32_t)l);
  // per sign class, the section's largest number of occupied slots in one
  // column (rounded up to whole blocks of kh steps): the steps used
  int Sc[2] = {0, 0};
  for (int cls = 0; cls < 2; ++cls) {
    for (int col = 0; col < M; ++col) {
      int m = 0;
      for (int h = 0; h < c->nhi; ++h)
        if ((__builtin_popcount(h) & 1) == cls && inv_l[(size_t)h * M + col] != (uint16_t)n) ++m;
      Sc[cls] = std::max(Sc[cls], m);
    }
    Sc[cls] = std::min(Sh, std::max(kh, (Sc[cls] + kh - 1) / kh * kh));
  }
  if (hs) hs[l] = (uint32_t)Sc[0] | ((uint32_t)Sc[1] << 16);
  std::vector<int> A((size_t)gsize * Sh), cnt((size_t)Sh * nbank), emp(Sh), cost(Sh);
  auto step_cost = [&](int st) {
    const int* ct = &cnt[(size_t)st * nbank];
    int mx = 0, mn = 1 << 30;
    for (int g = 0; g < nbank; ++g) { mx = std::max(mx, ct[g]); mn = std::min(mn, ct[g]); }
    return emp[st] ? std::max(mx, mn + 1) : mx;
  };
  auto take = [&](int st, int v, int d) {
    if (v < 0) emp[st] += d;
    else cnt[(size_t)st * nbank + (v % nbank)] += d;
  };
  for (int si = 0; si < nsets; ++si) {
    const int* cols = &sets[(size_t)si * gsize];
    for (int cls = 0; cls < 2; ++cls) {
      const int S = Sc[cls];
      std::fill(cnt.begin(), cnt.end(), 0);
      std::fill(emp.begin(), emp.end(), 0);
      for (int j = 0; j < gsize; ++j) {
        int m = 0;
        int* a = &A[(size_t)j * S];
        for (int h = 0; h < c->nhi; ++h)
          if ((__builtin_popcount(h) & 1) == cls && inv_l[(size_t)h * M + cols[j]] != (uint16_t)n)
            a[m++] = inv_l[(size_t)h * M + cols[j]];
        for (; m < S; ++m) a[m] = -1;
        std::shuffle(a, a + S, rng);
        for (int st = 0; st < S; ++st) take(st, a[st], +1);
      }
      for (int st = 0; st < S; ++st) cost[st] = step_cost(st);
      // moves target the conflict: a column of the worst step that sits on
      // that step's most loaded bank (random columns: the same tables after
      // 4000 moves that these reach after 256, c3 1.10 / c4 1.005 LDS cycles
      // per lane group, ~1 / 16 of the host time)
      for (int it = 0; it < 256; ++it) {
        int s1 = 0;
        for (int st = 1; st < S; ++st)
          if (cost[st] > cost[s1]) s1 = st;
        if (cost[s1] <= 1) break;  // conflict-free
        int j;
        {
          const int* ct = &cnt[(size_t)s1 * nbank];
          int bm = 0;
          for (int g = 1; g < nbank; ++g)
            if (ct[g] > ct[bm]) bm = g;
          int cand[64], nc = 0;
          for (int jj = 0; jj < gsize && nc < 64; ++jj) {
            const int v = A[(size_t)jj * S + s1];
            if (v >= 0 && v % nbank == bm) cand[nc++] = jj;
          }
          j = nc > 0 ? cand[rng() % (unsigned)nc] : (int)(rng() % (unsigned)gsize);
        }
        const int s2 = (int)(rng() % (unsigned)S);
        if (s2 == s1) continue;
        int& x = A[(size_t)j * S + s1];
        int& y = A[(size_t)j * S + s2];
        if (x == y) continue;
        take(s1, x, -1); take(s2, y, -1); take(s1, y, +1); take(s2, x, +1);
        const int n1 = step_cost(s1), n2 = step_cost(s2);
        if (n1 + n2 <= cost[s1] + cost[s2]) {
          std::swap(x, y);
          cost[s1] = n1;
          cost[s2] = n2;
        } else {
          take(s1, y, -1); take(s2, x, -1); take(s1, x, +1); take(s2, y, +1);
        }
      }
      for (int st = 0; st < S; ++st) {
        int zg = 0;
        for (int g = 1; g < nbank; ++g)
          if (cnt[(size_t)st * nbank + g] < cnt[(size_t)st * nbank + zg]) zg = g;
        const int zrow = n + ((zg - n % nbank + nbank) % nbank);  // the zero row on bank zg
        for (int j = 0; j < gsize; ++j) {
          const int v = A[(size_t)j * S + st];
          out[(size_t)(cls * Sh + st) * M + cols[j]] = (uint16_t)(v >= 0 ? v : zrow);
        }
      }
      for (int st = S; st < Sh; ++st)  // never gathered (every column's slots sit in the first S steps)
        for (int j = 0; j < gsize; ++j) out[(size_t)(cls * Sh + st) * M + cols[j]] = (uint16_t)n;
    }
  }
}

// All sections in parallel on the host; uploaded into *dst.
int build_banked(sa_ctx* c, const std::vector<int>& sets, int gsize, int nbank, uint16_t** dst, int kh) {
  const int L = c->L, n = c->n, w = c->w;
  std::vector<uint16_t> inv_own, out((size_t)L * w, 0);
  std::vector<uint32_t> hs((size_t)L, 0);
  if (c->h_inv.size() != (size_t)L * w) {  // the host copy went (or never was): rebuild it
    inv_own.assign((size_t)L * w, (uint16_t)n);
    parallel_for(L, 1, [&](int l) {
      for (int r = 0; r < n; ++r) inv_own[(size_t)l * w + c->ordering[(size_t)l * n + r]] = (uint16_t)r;
    });
  }
  const uint16_t* inv = inv_own.empty() ? c->h_inv.data() : inv_own.data();
  parallel_for(L, 1, [&](int l) {
    banked_section(c, l, inv + (size_t)l * w, out.data() + (size_t)l * w, sets, gsize, nbank, hs.data(), kh);
  });
  int rc = dev_alloc(c, (void**)dst, out.size() * 2);
  if (!rc) rc = dev_alloc(c, (void**)&c->d_hs, hs.size() * 4);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(*dst, out.data(), out.size() * 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_hs, hs.data(), hs.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

bool banks_enabled(const sa_ctx* c) { return !(c->plan & SA_PLAN_NO_BANKS); }

// [L][w] bucket table (slot h * M + column) -> [L][nhi][64][E]: lane L's E
// entries of step h contiguous, in register order (columns elem_index<E >= 4>
// of lane L ^ 3 in binary32 (sgn), of L in binary64)
__global__ void k_lane_major(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst, int L, int nhi, int M,
                             int w, int E, int sgn) {
  const size_t tot = (size_t)L * nhi * 64 * E;
  for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < tot; x += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(x % E);
    size_t t = x / E;
    const int lane = (int)(t % 64);
    t /= 64;
    const int h = (int)(t % nhi), l = (int)(t / nhi);
    const int lp = sgn ? (lane ^ 3) : lane;
    const int e = (i / 4) * 256 + lp * 4 + (i % 4);
    dst[x] = src[(size_t)l * w + (size_t)h * M + e];
  }
}

// ---- bank-aware Ab row order ----------------------------------------------
// k_secb's Ab pass gives lane L of a wave row r0 + L and reads, per step, one
// staged T element (section s, column k(r, s)) per lane: for 16-byte T rows a
// ds_read_b128 whose four 16-lane groups each take one LDS cycle per distinct
// row on their busiest 16-byte bank group (MI355X_MICROARCH.md §LDS).  In
// section order the columns k(r, s) of 16 rows are random: ~3 cycles per
// group.  A row's partial sum does not care in which order its W sections
// are added, so each row gets its own step order: a local search over swaps
// of two steps of one row that lowers, per lane group, the largest number of
// rows on one bank in a step (the addition order changes, the terms do not).
// Rows n .. npad-1 (the last block's idle lanes) repeat a real row of their
// lane group (a broadcast); sections past L read column 0 (a broadcast).
// LDS position of T column e in k_secb's staged image: the element index of
// (lane, register i) is (i / Q) 64 Q + lane Q + i % Q (elem_index), staged at
// (i / Q) 64 Q + (i % Q) 64 + lane
unsigned t_pos(int E, unsigned e) {
  const unsigned Q = E < 4 ? (unsigned)E : 4u;
  const unsigned blk = e / (64 * Q), rem = e % (64 * Q);
  return blk * 64 * Q + (rem % Q) * 64 + rem / Q;
}

void fwdb_group(const sa_ctx* c, int g, const uint16_t* fwd, int npad, uint16_t* out) {
  const int W = c->WB, M = c->M, n = c->n, L = c->L;
  const int rowb = c->CB * (int)rsz(c);  // bytes per staged T element
  const bool b128 = rowb == 16;
  const int gsize = b128 ? 16 : 32, nbank = b128 ? 16 : 32, ngroups = 64 / gsize;
  const bool search = banks_enabled(c);
  std::mt19937 rng(0xab0000u + (uint32_t)g);
  std::vector<int> cnt((size_t)W * nbank), perm((size_t)gsize * W), bank((size_t)gsize * W), cost(W);
  std::vector<uint16_t> ent((size_t)gsize * W);
  auto step_cost = [&](int st) {
    int mx = 0;
    for (int b = 0; b < nbank; ++b) mx = std::max(mx, cnt[(size_t)st * nbank + b]);
    return mx;
  };
  for (int b0 = 0; b0 < npad; b0 += 64) {
    for (int G = 0; G < ngroups; ++G) {
      int rows[32], nreal = 0;
      for (int j = 0; j < gsize; ++j) {
        const int lane = b128 ? kLdsGroups16[G][j] : G * 32 + j;
        rows[j] = b0 + lane;
      }
      // entries (s * M + k | sign) and banks of the real rows, identity order
      std::fill(cnt.begin(), cnt.end(), 0);
      for (int j = 0; j < gsize; ++j) {
        const int r = rows[j];
        if (r >= n) continue;
        ++nreal;
        for (int sl = 0; sl < W; ++sl) {
          const int l = g * W + sl;
          uint16_t e = 0;
          if (l < L) e = fwd[((size_t)(l / kSpw) * n + r) * kSpw + (l % kSpw)];
          const unsigned k = t_pos(c->E, e & 0x7fffu);
          ent[(size_t)j * W + sl] = (uint16_t)(((unsigned)sl * M + k) | (e & 0x8000u));
          bank[(size_t)j * W + sl] = l < L ? (int)(((unsigned)sl * M + k) % (unsigned)nbank) : -1;
          perm[(size_t)j * W + sl] = sl;
          if (l < L) ++cnt[(size_t)sl * nbank + bank[(size_t)j * W + sl]];
        }
      }
      if (search && nreal > 1) {
        for (int st = 0; st < W; ++st) cost[st] = step_cost(st);
        // 16 W moves: the searched tables reach a sum of step costs 1.17x that
        // of 64 W moves (C4), with the same C3 / C4 throughput, in a quarter
        // of the host time (0.11 -> 0.05 s at C4)
        for (int it = 0; it < 16 * W; ++it) {
          int s1 = 0;
          for (int st = 1; st < W; ++st)
            if (cost[st] > cost[s1]) s1 = st;
          if (cost[s1] <= 1) break;
          int bm = 0;
          for (int b = 1; b < nbank; ++b)
            if (cnt[(size_t)s1 * nbank + b] > cnt[(size_t)s1 * nbank + bm]) bm = b;
          int cand[32], nc = 0;
          for (int j = 0; j < gsize; ++j)
            if (rows[j] < n && bank[(size_t)j * W + perm[(size_t)j * W + s1]] == bm) cand[nc++] = j;
          if (nc == 0) break;
          const int j = cand[rng() % (unsigned)nc];
          const int s2 = (int)(rng() % (unsigned)W);
          if (s2 == s1) continue;
          int& x = perm[(size_t)j * W + s1];
          int& y = perm[(size_t)j * W + s2];
          const int bx = bank[(size_t)j * W + x], by = bank[(size_t)j * W + y];
          auto mv = [&](int st, int b, int d) {
            if (b >= 0) cnt[(size_t)st * nbank + b] += d;
          };
          mv(s1, bx, -1); mv(s2, by, -1); mv(s1, by, +1); mv(s2, bx, +1);
          const int n1 = step_cost(s1), n2 = step_cost(s2);
          if (n1 + n2 <= cost[s1] + cost[s2]) {
            std::swap(x, y);
            cost[s1] = n1;
            cost[s2] = n2;
          } else {
            mv(s1, by, -1); mv(s2, bx, -1); mv(s1, bx, +1); mv(s2, by, +1);
          }
        }
      }
      // out [g * W/4 + q][npad][4]: step st = 4 q + slot; idle rows copy the
      // group's first real row (or, with none, row 0 of the block's order)
      int jr = -1;
      for (int j = 0; j < gsize && jr < 0; ++j)
        if (rows[j] < n) jr = j;
      for (int j = 0; j < gsize; ++j) {
        const int src = rows[j] < n ? j : jr;
        for (int st = 0; st < W; ++st) {
          const uint16_t e = src >= 0 ? ent[(size_t)src * W + perm[(size_t)src * W + st]] : (uint16_t)((unsigned)st * M);
          out[((size_t)(g * (W / 4) + st / 4) * npad + rows[j]) * 4 + (st % 4)] = e;
        }
      }
    }
  }
}

int build_fwdb(sa_ctx* c) {
  const int n = c->n, npad = (n + 63) & ~63, Gb = c->Gb, W = c->WB;
  // the host copy of d_fwd, [G][n][4] (built again from the ordering: the
  // same entries build_tables uploads)
  const int lgM = ilog2(c->M);
  const int G = (c->L + kSG - 1) / kSG * (kSG / kSpw);
  std::vector<uint16_t> fwd_own;
  if (c->h_fwd.size() != (size_t)G * n * kSpw) {  // the host copy went (or never was): rebuild it
    fwd_own.assign((size_t)G * n * kSpw, 0);
    parallel_for(c->L, 4, [&](int l) {
      for (int r = 0; r < n; ++r) {
        const uint32_t v = c->ordering[(size_t)l * n + r];
        fwd_own[((size_t)(l / kSpw) * n + r) * kSpw + (l % kSpw)] =
            (uint16_t)((v & (uint32_t)(c->M - 1)) | ((__builtin_popcount(v >> lgM) & 1u) << 15));
      }
    });
  }
  const uint16_t* fwd = fwd_own.empty() ? c->h_fwd.data() : fwd_own.data();
  std::vector<uint16_t> out((size_t)Gb * W * npad, 0);
  parallel_for(Gb, 1, [&](int g) { fwdb_group(c, g, fwd, npad, out.data()); });
  int rc = dev_alloc(c, (void**)&c->d_fwdb, out.size() * 2);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_fwdb, out.data(), out.size() * 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

// k_secb (16-byte rows: binary32 CB = 4, binary64 CB = 2; E >= 4): lane L of a
// wave holds columns elem_index<E>(L ^ 3 in binary32, i) (quad-mirrored positions)
int ensure_invb(sa_ctx* c) {
  // the Ab table first (every k_secb configuration reads it)
  if (c->backend == SA_BACKEND_HADAMARD && c->CB > 0 && !c->big && !c->d_fwdb) {
    if (c->WB * c->M >= 32768) return fail(SA_ERR_UNSUPPORTED, "k_secb: W * M >= 2^15");
    if (int rc = build_fwdb(c)) return rc;
  }
  if (c->invb_done) return SA_OK;
  c->invb_done = true;
  const bool sgn = c->prec == SA_PREC_F32;  // k_secb's SGN (E >= 2)
  const bool rows16 = c->backend == SA_BACKEND_HADAMARD && c->CB > 0 && c->CB * (int)rsz(c) == 16 && !c->big;
  if (rows16 && banks_enabled(c) && c->E >= 4 && c->nhi >= 2 && c->n + kInvbZeroRows <= 65535) {
    std::vector<int> sets;
    for (int i = 0; i < c->E; ++i)
      for (int G = 0; G < 4; ++G)
        for (int j = 0; j < 16; ++j) {
          const int lane = kLdsGroups16[G][j], lp = sgn ? (lane ^ 3) : lane;
          sets.push_back((i / 4) * 256 + lp * 4 + (i % 4));  // elem_index<E >= 4>
        }
    // (the kernel's h-steps per table block: kSecbKH64 in binary64, kSecbKH32 at CB = 4)
    const int kh = sgn ? kSecbKH32 : kSecbKH64;
    if (int rc = build_banked(c, sets, 16, 16, &c->d_invb, kh)) return rc;
  }
  // the codeword-interleaved k_secb's copy of its bucket table with each
  // lane's E entries of a step contiguous (one 16-byte load per lane and
  // step at E = 8 instead of two 8-byte loads 512 B apart)
  if (rows16 && c->E >= 4 && c->E % 4 == 0) {
    const size_t cnt = (size_t)c->L * c->nhi * 64 * c->E;
    if (int rc = dev_alloc(c, (void**)&c->d_invl, cnt * 2)) return rc;
    k_lane_major<<<(int)std::min<size_t>((cnt + 255) / 256, 16384), 256, 0, c->stream>>>(
        c->d_invb ? c->d_invb : c->d_inv, c->d_invl, c->L, c->nhi, c->M, c->w, c->E, sgn ? 1 : 0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  std::vector<uint16_t>().swap(c->h_inv);  // the host copies have served
  std::vector<uint16_t>().swap(c->h_fwd);
  return SA_OK;
}


// Every section-kernel instantiation may use the full 160 KB LDS, the MFMA
// GEMMs their staging buffers (once per process).
int set_lds_limits() {
  static int done = 0;
  if (done) return SA_OK;
  if (!secb_no_static_lds())
    return fail(SA_ERR_HIP, "k_secb has static LDS: absolute LDS addressing in gather_step4 is invalid");
  hipError_t e = sec_lds_attrs();
  if (e == hipSuccess) e = secb_lds_attrs();
  if (e == hipSuccess) e = dense_lds_attrs();
  if (e == hipSuccess) e = mc_lds_attrs();
  if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  done = 1;
  return SA_OK;
}

int create_impl(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int prec,
                int device, int plan, const sa_ctx* share) {
  if (!out) return fail(SA_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (L <= 0 || M <= 0 || n <= 0) return fail(SA_ERR_ARG, "L, M, n must be positive");
  if (backend != SA_BACKEND_HADAMARD && backend != SA_BACKEND_DENSE && backend != SA_BACKEND_HOST &&
      backend != SA_BACKEND_MATRIX)
    return fail(SA_ERR_ARG, "unknown backend");
  if (!ordering && backend != SA_BACKEND_HOST && backend != SA_BACKEND_MATRIX)
    return fail(SA_ERR_ARG, "ordering is NULL");
  if (prec != SA_PREC_F32 && prec != SA_PREC_F64) return fail(SA_ERR_ARG, "unknown precision");
  if (plan & ~SA_PLAN_ALL) return fail(SA_ERR_ARG, "unknown plan option bits");
  if (backend == SA_BACKEND_DENSE && prec != SA_PREC_F32)
    return fail(SA_ERR_UNSUPPORTED, "dense backend streams an fp32 matrix (precision must be F32)");
  const bool pow2 = (M & (M - 1)) == 0;
  if (M > 4096) return fail(SA_ERR_UNSUPPORTED, "M must be <= 4096");
  // the Hadamard operator takes n past 16-bit row indices (k_secg); the
  // materialised designs and the host-operator loop keep the 16-bit limit
  if (n >= (backend == SA_BACKEND_HADAMARD ? (1 << 24) : 65535))
    return fail(SA_ERR_UNSUPPORTED, backend == SA_BACKEND_HADAMARD ? "n must be < 2^24" : "n must be < 65535");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SA_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(SA_ERR_ARG, "device index out of range");
  HIP_TRY(hipSetDevice(device));

  sa_ctx* c = new sa_ctx();
  c->L = L; c->M = M; c->n = n; c->backend = backend; c->prec = prec; c->device = device; c->plan = plan;
  c->Mu = M;
  const int mx = (M + 1) > (n + 1) ? (M + 1) : (n + 1);
  c->w = 1 << ilog2(mx);  // 2^ceil(log2(max(M+1, n+1))), sparc_ldpc.py:52/:110
  if (!pow2 && backend == SA_BACKEND_HADAMARD) {
    // any M on the matrix-free operator: the reference keeps the last M of the
    // w columns (sparc_ldpc.py:68/:77), which are the last M of the last
    // Mp = 2^ceil(log2 M) <= w, whose high index bits are all ones: a section
    // is a padded section of Mp columns whose first Mp - M never carry an
    // estimate (the denoiser excludes them, beta stays 0 there); the caller's
    // beta / A^T z move in and out of the padded layout at the boundary
    c->M = 1 << ilog2(M);
    c->dead = c->M - M;
    M = c->M;
  }
  c->nhi = c->w / M;
  c->E = 1;  // elements per lane of a one-wave section: the power of two covering M
  while (c->E * 64 < M) c->E *= 2;
  c->pow2 = pow2;
  if (ordering) c->ordering.assign(ordering, ordering + (size_t)L * n);
  c->NZ = (n + kRowsPerBlk - 1) / kRowsPerBlk;
  c->NZ16 = (n + kRow2Rows - 1) / kRow2Rows;
  c->NZh = (n + 15) / 16;
  c->NZ4 = (n + 255) / 256;
  c->NZ2 = (n + 127) / 128;
  c->nz_cur = c->NZ;
  // section kernel LDS: z slots + 4 sections x M + 4 beta^2 partials
  const size_t s = rsz(c);
  const size_t zbytes = ((size_t)(n + 1) * s + 15) / 16 * 16;
  c->sec_lds = zbytes + (size_t)kSpw * M * s + (size_t)kSpw * s;
  if (backend == SA_BACKEND_HADAMARD && (n >= 65535 || c->sec_lds > 160 * 1024)) {
    // z from global memory, 32-bit bucket entries (k_secg); the multi-wave and
    // batched kernels' LDS images need z too: they stay off (G2, CB below)
    c->big = true;
    c->sec_lds = (size_t)kSpw * M * s + (size_t)kSpw * s;
  }
  if (c->dead > 0 && c->big) {
    delete c;
    return fail(SA_ERR_UNSUPPORTED, "M not a power of two: the Hadamard operator keeps z in LDS (n < 65535 and "
                                    "the z image within 160 KB)");
  }
  if (c->sec_lds > 160 * 1024) {
    delete c;
    return fail(SA_ERR_UNSUPPORTED, "section kernel does not fit in LDS (n and M too large for this precision)");
  }
  c->G = (L + kSpw - 1) / kSpw;
  c->Gb = (L + kWB - 1) / kWB;  // (re-set after the batched width is chosen)
  // (a padded section runs on k_sec alone, the one section kernel that masks dead columns)
  if (M >= 128 && M <= 4096 && !c->big && c->dead == 0) {  // k_sec2: z + 2 sections' T + top-bit exchange + reductions
    const size_t need = zbytes + 2 * (size_t)M * s + 4 * (size_t)(M / 2) * s + 16 * s;
    if (need <= 160 * 1024) {
      c->G2 = (L + 1) / 2;
      c->sec2_lds = need;
    }
    // k_sec4: z + 2 sections' T + one exchange image per section + reductions
    const size_t need4 = zbytes + 4 * (size_t)M * s + 32 * s;
    if (c->G2 > 0 && M >= 256 && need4 <= 160 * 1024) {
      c->sec4 = true;
      c->sec4_lds = need4;
    }
    // row-block-major Ab partials for k_row2 (SA_PLAN_NO_PT: the [G][n] layout):
    // each k_row2 workgroup reads one contiguous G x 128-B block instead of G
    // lines n rows apart.  C4 single codeword 880 -> 950 cw/s (k_row2 4.1 ->
    // 3.4 us, two interleaved A/B rounds); c2 within noise
    c->pt_on = !(plan & SA_PLAN_NO_PT);
    // 16-row k_row2 blocks for one codeword where the z^2 partials still fit
    // the section kernels' registers (ceil(n / 16) <= 320; C2: 288 workgroups
    // instead of 144, every CU pulls partials): c2 1362-1374 -> 1396 cw/s
    // (two interleaved A/B rounds).  Binary32 only: in binary64 the 32-row
    // blocks are faster (c2 fp64 984-988 -> 990-1013 cw/s, two interleaved
    // rounds, round 3).  SA_PLAN_NO_ROW16 / SA_PLAN_ROW16 force 32- / 16-row blocks
    const bool r16 = (plan & SA_PLAN_ROW16) ? true : (plan & SA_PLAN_NO_ROW16) ? false : s == 4;
    c->row16 = r16 && c->pt_on && c->sec4 && c->NZh <= 320;
  }

  // batched kernel: the most codewords per workgroup (CB in {4, 2, 1}; 4 for
  // fp32 only) whose LDS image (z and T share one region) still lets two
  // 8-section workgroups share a CU (CB = 1 takes the whole LDS if it must);
  // one 16-section workgroup per CU instead where its whole-LDS image holds a
  // larger chunk (L = 768, n = 8294: CB 4 instead of 2; binary64 2 instead of
  // 1), and also at equal CB (half the Ab partials: the row kernel's HBM read
  // halves, the section kernel pays a 16-wave barrier): C4 batch 256 4.45 k
  // -> 5.51 k cw/s (binary64 2.17 k -> 2.41 k), C3 11.10 k -> 11.26 k; in
  // binary64 at equal CB since round 4 (C3 fp64 with ZIL 6.44 k -> 7.02 k,
  // the joint configs[4] step 1.65 k -> 1.75 k).  SA_PLAN_WB8 / WB16 force it.
  {
    auto cb_for = [&](int W) -> std::pair<int, size_t> {
      for (int cb = (s == 4 ? 4 : 2); cb >= 1 && M <= 1024; cb >>= 1) {
        const size_t zb = (((size_t)(n + kInvbZeroRows) * cb * s) + 15) / 16 * 16;
        const size_t tb = (size_t)W * M * cb * s;
        const size_t need = (zb > tb ? zb : tb) + (size_t)W * cb * s + (s == 8 ? 64 * 8 : 0);
        if (need <= (cb == 1 || W > kWB ? 160 : 80) * 1024) return {cb, need};
      }
      return {0, 0};
    };
    const bool nob = c->big || c->dead > 0;
    const auto c8 = nob ? std::pair<int, size_t>{0, 0} : cb_for(kWB);
    const auto c16 = nob ? std::pair<int, size_t>{0, 0} : cb_for(kWB16);
    const bool w16 = (plan & SA_PLAN_WB16) ? true
                     : (plan & SA_PLAN_WB8) ? false
                                            : c16.first >= c8.first;
    c->WB = w16 && c16.first > 0 ? kWB16 : kWB;
    c->CB = c->WB == kWB16 ? c16.first : c8.first;
    c->secb_lds = c->WB == kWB16 ? c16.second : c8.second;
    c->Gb = (L + c->WB - 1) / c->WB;
    // passes over each XCD's section groups so one pass's bucket and Ab
    // tables (W sections x (w + n) x 2 B per group) stay within kSecbL2
    // bytes of the XCD's 4 MB L2 (the rest: z chunks, streamed beta)
    const size_t per_group = (size_t)c->WB * ((size_t)c->w + (size_t)n) * 2;
    const int gx = c->Gb / 8 > 0 ? c->Gb / 8 : 1;
    const int fit = (int)std::max<size_t>(1, kSecbL2 / per_group);
    int npass = (gx + fit - 1) / fit;
    c->gpx = (gx + npass - 1) / npass;  // balanced passes
    if (plan & SA_PLAN_ONE_PASS) c->gpx = 1 << 20;
  }
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->n_cus = prop.multiProcessorCount;
  }
  c->Gd = (L + 3) / 4;
  {
    // k_sec43: three sections per workgroup where pairs overfill the chip
    // (ceil(L/2) > CUs >= ceil(L/3), e.g. L = 768) — one workgroup per CU
    // instead of two on half of them; in binary64 also where pairs fill the
    // chip exactly (L = 2 x CUs, c2): a third fewer 8-byte Ab partials for
    // k_row2 outweigh the longer section step (c2 fp64 989-997 -> 1026-1027
    // cw/s, two interleaved A/B rounds, round 3; binary32 at c2: neutral, pairs
    // kept).  SA_PLAN_NO_SEC3 / SA_PLAN_SEC3 force it off / on
    const size_t need3 = (((size_t)(n + 1) * s + 15) / 16 * 16) + 6 * (size_t)M * s + 48 * s;
    const int G3 = (L + 2) / 3;
    const bool fits = c->sec4 && backend == SA_BACKEND_HADAMARD && M <= 512 && need3 <= 160 * 1024;
    const bool over = c->G2 > c->n_cus || (s == 8 && c->G2 == c->n_cus);
    const bool want = (plan & SA_PLAN_SEC3) ? true : (plan & SA_PLAN_NO_SEC3) ? false : (over && G3 <= c->n_cus);
    if (fits && want) {
      c->sec3 = true;
      c->G3 = G3;
      c->sec3_lds = need3;
    }
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    delete c;
    return fail(SA_ERR_HIP, "stream/event creation failed");
  }
  int rc = SA_OK;
  if (backend == SA_BACKEND_DENSE) {
    c->RS = 8;
    c->KS = 8;
    rc = build_tables(c);  // validates the ordering (distinct values in [1, w))
    if (!rc) rc = build_dense(c);
  } else if (backend == SA_BACKEND_HOST) {
    c->lda = (size_t)L * M;  // no operator on the device: the caller's products are uploaded
  } else if (backend == SA_BACKEND_MATRIX) {
    // the caller's matrix, uploaded by sa_create_matrix (sa_dense.hip)
    c->RS = 8;
    c->KS = 8;
    rc = matrix_init(c);
  } else if (share) {  // sa_create_twin: the same tables, read-only, borrowed
    c->d_inv = share->d_inv; c->d_inv32 = share->d_inv32; c->d_invb = share->d_invb;
    c->d_fwdb = share->d_fwdb; c->d_fwd = share->d_fwd; c->d_fwd2 = share->d_fwd2; c->d_fwd3 = share->d_fwd3;
    c->d_invl = share->d_invl; c->d_hs = share->d_hs;
    c->invb_done = share->invb_done;
    c->borrowed = true;
  } else {
    rc = build_tables(c);
  }
  if (!rc) rc = dev_alloc(c, &c->d_c, (size_t)L * s);
  if (!rc) rc = dev_alloc(c, (void**)&c->d_cd, (size_t)L * 8);
  if (!rc) rc = dev_alloc(c, &c->d_P1, s);
  if (rc) {
    sa_destroy(c);
    return rc;
  }
  if ((rc = set_lds_limits())) {
    sa_destroy(c);
    return rc;
  }
  *out = c;
  return SA_OK;
}

}  // namespace sa

using namespace sa;

extern "C" {

int sa_create(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int precision,
              int device) {
  return create_impl(out, L, M, n, ordering, backend, precision, device, SA_PLAN_DEFAULT);
}

int sa_create_ex(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int precision,
                 int device, int plan) {
  return create_impl(out, L, M, n, ordering, backend, precision, device, plan);
}


int sa_subset(const sa_ctx* parent, const int64_t* sections, int Ls, sa_ctx** out) {
  if (int rc0 = check_tables(parent, "sa_subset")) return rc0;
  if (!sections || Ls <= 0) return fail(SA_ERR_ARG, "empty section subset");
  std::vector<uint32_t> ord((size_t)Ls * parent->n);
  for (int i = 0; i < Ls; ++i) {
    int64_t s = sections[i];
    if (s < 0) s += parent->L;  // numpy negative indexing
    if (s < 0 || s >= parent->L) return fail(SA_ERR_ARG, "section index out of range");
    std::memcpy(ord.data() + (size_t)i * parent->n, parent->ordering.data() + (size_t)s * parent->n,
                (size_t)parent->n * 4);
  }
  return create_impl(out, Ls, parent->Mu, parent->n, ord.data(), parent->backend, parent->prec, parent->device,
                     parent->plan);
}

int sa_create_twin(sa_ctx* src, sa_ctx** out) {
  if (!out) return fail(SA_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (check_ctx(src)) return SA_ERR_ARG;
  if (src->backend != SA_BACKEND_HADAMARD)
    return fail(SA_ERR_UNSUPPORTED, "sa_create_twin: Hadamard-backend contexts only");
  HIP_TRY(hipSetDevice(src->device));
  // the lazily built batched-kernel tables first, so that both contexts use them
  if (int rc = ensure_invb(src)) return rc;
  return create_impl(out, src->L, src->Mu, src->n, src->ordering.data(), src->backend, src->prec, src->device,
                     src->plan, src);
}

void sa_destroy(sa_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  drop_graphs(c);
  free_workspace(c);
  mc_release(c);
  if (!c->borrowed) {
    dev_free(c->d_inv);
    dev_free(c->d_inv32);
    dev_free(c->d_invb);
    dev_free(c->d_fwdb);
    dev_free(c->d_invl);
    dev_free(c->d_hs);
    dev_free(c->d_fwd);
    dev_free(c->d_fwd2);
    dev_free(c->d_fwd3);
  }
  dev_free(c->d_A);
  dev_free(c->d_AT); dev_free(c->d_xz); dev_free(c->d_xb);
  dev_free(c->d_A8); dev_free(c->d_AT8); dev_free(c->d_zq); dev_free(c->d_bq);
  dev_free(c->d_zsc); dev_free(c->d_bsc0); dev_free(c->d_bfix);
  dev_free(c->d_c);
  dev_free(c->d_cd);
  dev_free(c->d_P1);
  dev_free(c->d_stage);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (auto& e : c->dec_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->h_dec) (void)hipHostFree(c->h_dec);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int sa_Ab(sa_ctx* c, int B, const double* beta, double* out) {
  if (int rc0 = check_op(c, "sa_Ab")) return rc0;
  if (B <= 0 || !beta || !out) return fail(SA_ERR_ARG, "sa_Ab: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, c->Tcap > 0 ? c->Tcap : 1);
  if (rc) return rc;
  if ((rc = upload_sections(c, c->d_beta, beta, B))) return rc;
  rc = c->prec == SA_PREC_F64 ? seq_ab<double>(c, B) : seq_ab<float>(c, B);
  if (rc) return rc;
  if ((rc = download(c, out, c->d_out, (size_t)B * c->n))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_Az(sa_ctx* c, int B, const double* z, double* out) {
  if (int rc0 = check_op(c, "sa_Az")) return rc0;
  if (B <= 0 || !z || !out) return fail(SA_ERR_ARG, "sa_Az: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, c->Tcap > 0 ? c->Tcap : 1);
  if (rc) return rc;
  if ((rc = upload(c, c->d_z, z, (size_t)B * c->n))) return rc;
  c->zil_last = false;  // d_z holds [B][n] now
  if (c->prec == SA_PREC_F64) {
    rc = seq_az<double>(c, B);
  } else {
    rc = seq_az<float>(c, B);
  }
  if (rc) return rc;
  if ((rc = download_sections(c, out, c->d_out, B))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_reserve(sa_ctx* c, int B, int T) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || T < 0) return fail(SA_ERR_ARG, "sa_reserve: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, T > 0 ? T : 1);
  // the batched kernel's tables (built once per operator) now, not at the first decode
  if (!rc && c->backend == SA_BACKEND_HADAMARD && use_batched(c, B)) rc = ensure_invb(c);
  return rc;
}

int sa_stage(sa_ctx* c, int B, const double* y, const double* Pl, const double* beta0) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0) return fail(SA_ERR_ARG, "sa_stage: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, c->Tcap > 0 ? c->Tcap : 1);
  if (rc) return rc;
  if (Pl && (rc = set_power(c, Pl))) return rc;
  if (y && (rc = upload(c, c->d_y, y, (size_t)B * c->n))) return rc;  // NULL: keep the staged y
  if (beta0 && (rc = upload_sections(c, c->d_beta, beta0, B))) return rc;
  return SA_OK;
}

int sa_stage_power_batch(sa_ctx* c, int B, const double* Pl) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0) return fail(SA_ERR_ARG, "sa_stage_power_batch: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, c->Tcap > 0 ? c->Tcap : 1);
  if (rc) return rc;
  return set_power_batch(c, B, Pl);
}

int sa_run(sa_ctx* c, int B, int T, int flags) {
  if (int rc0 = check_op(c, "sa_run")) return rc0;
  if (B <= 0 || T < 0) return fail(SA_ERR_ARG, "sa_run: bad arguments");
  if (!c->power_set) return fail(SA_ERR_ARG, "sa_run: power allocation not staged");
  if (B > c->Bcap) return fail(SA_ERR_ARG, "sa_run: batch larger than the staged batch");
  HIP_TRY(hipSetDevice(c->device));
  if (T > c->Tcap) {
    // growing T reallocates the workspace; keep the staged inputs
    return fail(SA_ERR_ARG, "sa_run: T larger than the workspace (call sa_reserve first)");
  }
  const int has_b0 = (flags & SA_FLAG_BETA0) ? 1 : 0;
  return c->prec == SA_PREC_F64 ? run_graph<double>(c, B, T, flags & 0xff, has_b0)
                                : run_graph<float>(c, B, T, flags & 0xff, has_b0);
}

int sa_wait(sa_ctx* c) {
  if (check_ctx(c)) return SA_ERR_ARG;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

double sa_run_event_ms(sa_ctx* c) {
  if (!c) return -1.0;
  float ms = -1.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.0;
  return ms;
}

int sa_fetch_z(sa_ctx* c, int B, double* z_out) {
  if (check_ctx(c) || !z_out) return fail(SA_ERR_ARG, "sa_fetch_z: bad arguments");
  if (B <= 0 || B > c->Bcap) return fail(SA_ERR_ARG, "sa_fetch_z: bad batch");
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if (c->zil_last) {  // [NC][n][CB] -> [B][n]
    const int CB = 16 / (int)rsz(c), NC = (B + CB - 1) / CB;
    std::vector<double> il((size_t)NC * CB * c->n);
    if ((rc = download(c, il.data(), c->d_z, il.size()))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int b = 0; b < B; ++b)
      for (int r = 0; r < c->n; ++r) z_out[(size_t)b * c->n + r] = il[((size_t)(b / CB) * c->n + r) * CB + b % CB];
    return SA_OK;
  }
  if ((rc = download(c, z_out, c->d_z, (size_t)B * c->n))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}


int sa_fetch(sa_ctx* c, int B, double* beta_out, int* iters_out) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || B > c->Bcap) return fail(SA_ERR_ARG, "sa_fetch: bad batch");
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if (beta_out && (rc = download_sections(c, beta_out, c->d_beta, B))) return rc;
  if (iters_out) HIP_TRY(hipMemcpyAsync(iters_out, c->d_iters, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_amp(sa_ctx* c, int B, const double* y, const double* Pl, int T, const double* beta0, double* beta_out,
           int* iters_out, int flags) {
  if (int rc0 = check_op(c, "sa_amp")) return rc0;
  if (B <= 0 || T < 0 || !y || !Pl || !beta_out) return fail(SA_ERR_ARG, "sa_amp: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, T > 0 ? T : 1);
  if (rc) return rc;
  if ((rc = sa_stage(c, B, y, Pl, beta0))) return rc;
  if (T == 0) {
    // the loop body never runs: beta is beta0 (or zeros)
    if (!beta0) HIP_TRY(hipMemsetAsync(c->d_beta, 0, (size_t)B * c->L * c->M * rsz(c), c->stream));
    HIP_TRY(hipMemsetAsync(c->d_iters, 0, (size_t)B * sizeof(int), c->stream));
  } else {
    if ((rc = sa_run(c, B, T, (flags & 0xff) | (beta0 ? SA_FLAG_BETA0 : 0)))) return rc;
  }
  return sa_fetch(c, B, beta_out, iters_out);
}

int sa_profile(sa_ctx* c, int B, int T, int flags, double* out) { return sa_profile_rep(c, B, T, flags, 1, out); }

int sa_profile_kinds(void) { return K_NKINDS; }

extern "C++" {
namespace {
int profile_impl(sa_ctx* c, int B, int T, int flags, int rep, bool dispatch, double* out) {
  if (int rc0 = check_op(c, "sa_profile")) return rc0;
  if (B <= 0 || T <= 0 || !out || B > c->Bcap || T > c->Tcap || !c->power_set || rep < 1 || rep > 1024)
    return fail(SA_ERR_ARG, "sa_profile: bad arguments (reserve and stage first)");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (int rcb = ensure_beta2(c, B)) return rcb;
  if (use_batched(c, B))
    if (int rci = ensure_invb(c)) return rci;
  Prof prof;
  prof.rep = rep;
  prof.dispatch = dispatch;
  c->prof = &prof;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, c->stream));
  const int has_b0 = (flags & SA_FLAG_BETA0) ? 1 : 0;
  int rc = c->prec == SA_PREC_F64 ? seq_amp<double>(c, B, T, flags & 0xff, has_b0)
                                  : seq_amp<float>(c, B, T, flags & 0xff, has_b0);
  c->prof = nullptr;
  (void)hipEventRecord(e1, c->stream);
  hipError_t e = hipStreamSynchronize(c->stream);
  if (rc == SA_OK && e != hipSuccess) rc = fail(SA_ERR_HIP, std::string("sa_profile: ") + hipGetErrorString(e));
  double sum[K_NKINDS] = {0}, cnt[K_NKINDS] = {0};
  if (rc == SA_OK) {
    for (auto& ev : prof.ev) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, std::get<1>(ev), std::get<2>(ev)) == hipSuccess) {
        sum[std::get<0>(ev)] += ms / rep;
        cnt[std::get<0>(ev)] += 1;
      }
    }
    float tot = 0.f;
    (void)hipEventElapsedTime(&tot, e0, e1);
    for (int k = 0; k < K_NKINDS; ++k) {
      out[2 * k] = cnt[k] > 0 ? sum[k] / cnt[k] : 0.0;
      out[2 * k + 1] = cnt[k];
    }
    out[2 * K_NKINDS] = tot;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}
}  // namespace
}  // extern "C++"

int sa_profile_rep(sa_ctx* c, int B, int T, int flags, int rep, double* out) {
  return profile_impl(c, B, T, flags, rep, false, out);
}

int sa_profile_dispatch(sa_ctx* c, int B, int T, int flags, double* out) {
  return profile_impl(c, B, T, flags, 1, true, out);
}


int sa_decide(sa_ctx* c, int B, int32_t* idx_out) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || B > c->Bcap || !idx_out) return fail(SA_ERR_ARG, "sa_decide: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  if (int rc = launch_decide(c, B)) return rc;
  HIP_TRY(hipMemcpyAsync(idx_out, c->d_idx, (size_t)B * c->L * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_decide_async(sa_ctx* c, int B, int slot) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || B > c->Bcap || slot < 0 || slot >= SA_DECIDE_SLOTS)
    return fail(SA_ERR_ARG, "sa_decide_async: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  const size_t per = (size_t)c->Bcap * c->L;  // one slot holds a whole staged batch
  if (!c->h_dec || c->dec_cap < per) {
    // a larger staged batch regrows the ring: refused while another slot still
    // holds decisions not collected (they would be dropped)
    for (int k = 0; k < SA_DECIDE_SLOTS; ++k)
      if (c->h_dec && c->dec_B[k] != 0)
        return fail(SA_ERR_ARG, "sa_decide_async: the staged batch grew while slot " + std::to_string(k) +
                                    " holds decisions not yet collected (sa_decide_collect them first)");
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->h_dec) (void)hipHostFree(c->h_dec);
    c->h_dec = nullptr;
    c->dec_cap = 0;
    HIP_TRY(hipHostMalloc((void**)&c->h_dec, per * SA_DECIDE_SLOTS * sizeof(int32_t), hipHostMallocDefault));
    c->dec_cap = per;
    for (int k = 0; k < SA_DECIDE_SLOTS; ++k) {
      if (!c->dec_ev[k]) HIP_TRY(hipEventCreateWithFlags(&c->dec_ev[k], hipEventDisableTiming));
      c->dec_B[k] = 0;
    }
  }
  // the slot's previous indices must have left the ring before they are overwritten
  // (the stream is in order: the copy below cannot overtake it anyway)
  if (int rc = launch_decide(c, B)) return rc;
  int32_t* dst = c->h_dec + (size_t)slot * c->dec_cap;
  HIP_TRY(hipMemcpyAsync(dst, c->d_idx, (size_t)B * c->L * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(c->dec_ev[slot], c->stream));
  c->dec_B[slot] = B;
  return SA_OK;
}

int sa_decide_collect(sa_ctx* c, int B, int slot, int32_t* idx_out) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (slot < 0 || slot >= SA_DECIDE_SLOTS || !idx_out || !c->h_dec || c->dec_B[slot] != B || B <= 0)
    return fail(SA_ERR_ARG, "sa_decide_collect: no decision of this batch queued in the slot");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(c->dec_ev[slot]));
  std::memcpy(idx_out, c->h_dec + (size_t)slot * c->dec_cap, (size_t)B * c->L * sizeof(int32_t));
  c->dec_B[slot] = 0;
  return SA_OK;
}


int sa_plan(sa_ctx* c, int B, int64_t* o) {
  if (check_ctx(c) || !o || B <= 0) return fail(SA_ERR_ARG, "sa_plan: bad arguments");
  const bool dense = is_dense(c);
  const bool batched = !dense && use_batched(c, B);
  const bool sec2 = use_sec2(c, B);
  const bool i8 = use_i8(c, B);
  const bool fg = use_fgemm(c, B);
  o[0] = i8 ? 6 : (fg ? 7 : (dense ? 3 : (batched ? 2 : (sec2 ? (c->sec3 ? 5 : (c->sec4 ? 4 : 1)) : (c->big ? 8 : 0)))));
  o[1] = dense ? dense_parts(c, B) : (batched ? c->Gb : (sec2 ? sec2_parts(c) : c->G));
  o[2] = (!dense && !batched && !sec2) ? row_splits(c, B) : 1;
  o[3] = batched ? c->CB : 1;
  o[4] = nz_for(c, row_kind_for(c, B));
  o[5] = c->w;
  o[6] = row_kind_for(c, B);
  o[7] = c->n_cus;
  return SA_OK;
}

int sa_plan_batched(sa_ctx* c, int B, int64_t* o) {
  if (check_ctx(c) || !o || B <= 0) return fail(SA_ERR_ARG, "sa_plan_batched: bad arguments");
  if (is_dense(c) || !use_batched(c, B)) return fail(SA_ERR_ARG, "sa_plan_batched: this batch does not run k_secb");
  // k_secb's XCD-grouped work order (sa_secb.hip): used when the groups and the
  // workgroups split evenly over the 8 XCDs, else one plain pass
  const int NC = (B + c->CB - 1) / c->CB;
  const bool xcd = (c->Gb % 8) == 0 && ((long long)c->Gb * NC) % 8 == 0;
  const int gx = xcd ? c->Gb / 8 : c->Gb;
  const int gp = xcd ? std::min(c->gpx, gx) : gx;
  o[0] = c->Gb;
  o[1] = c->WB;
  o[2] = gp;
  o[3] = (gx + gp - 1) / gp;
  return SA_OK;
}

int sa_info(const sa_ctx* c, int64_t* o) {
  if (check_ctx(c) || !o) return fail(SA_ERR_ARG, "sa_info: bad arguments");
  o[0] = c->L; o[1] = c->Mu; o[2] = c->n; o[3] = c->w; o[4] = c->backend; o[5] = c->prec;
  o[6] = c->device; o[7] = (int64_t)c->bytes;
  return SA_OK;
}

int sa_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* sa_last_error(void) { return g_err.c_str(); }

const char* sa_version(void) { return SA_VERSION; }

#ifdef SA_STAMPS
int sa_debug_stamps(unsigned long long* out) {
  // each unit keeps its own stamp buffer; the stamped kernel's is the non-zero one
  HIP_TRY(hipDeviceSynchronize());
  std::memset(out, 0, sizeof(unsigned long long) * 16 * 16);
  HIP_TRY(stamps_add_sec(out));
  HIP_TRY(stamps_add_secb(out));
  return SA_OK;
}
#endif

}  // extern "C"