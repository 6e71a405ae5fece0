// sa_host.h — the operator context (sa_ctx), launch timing and the host-side
// helpers shared by the kernel units and the C ABI (sparc_amp.hip).
#pragma once
#include "sa_common.h"

namespace sa {

// Per-launch timing for sa_profile (eager sequence only).
// Event mode: every profiled launch is bracketed by two HIP event records;
// with rep > 1 it is issued rep times back to back between them
// (sa_profile_rep: mean = elapsed / rep, which excludes the event packets'
// own dispatch overhead but lets each repeat re-read what its predecessor
// left in the caches).  Dispatch mode (sa_profile_dispatch): each launch goes
// out once through hipExtLaunchKernel with a start / stop event pair that the
// runtime binds to the kernel's own dispatch packet, so the pair times the
// kernel's execution in the decode's order (the quantity a rocprofv3 kernel
// trace records), with no marker packets in the stream.
struct Prof {
  std::vector<std::tuple<int, hipEvent_t, hipEvent_t>> ev;
  int rep = 1;
  bool dispatch = false;
  int kind = 0;
  int begin(hipStream_t s, int k) {
    kind = k;
    if (dispatch) return 0;
    hipEvent_t a = nullptr, b = nullptr;
    if (add(&a, &b)) return -1;
    return hipEventRecord(a, s) == hipSuccess ? 0 : -1;
  }
  void end(hipStream_t s) {
    if (!dispatch) (void)hipEventRecord(std::get<2>(ev.back()), s);
  }
  int add(hipEvent_t* a, hipEvent_t* b) {
    *a = *b = nullptr;
    if (hipEventCreate(a) != hipSuccess || hipEventCreate(b) != hipSuccess) return -1;
    ev.emplace_back(kind, *a, *b);
    return 0;
  }
  ~Prof() {
    for (auto& e : ev) {
      (void)hipEventDestroy(std::get<1>(e));
      (void)hipEventDestroy(std::get<2>(e));
    }
  }
};

enum { K_SEC = 0, K_ROW = 1, K_DAZ = 2, K_DDEN = 3, K_DAB = 4, K_QNT = 5, K_NKINDS = 6 };

}  // namespace sa

struct sa_ctx {
  sa::Prof* prof = nullptr;
  int L = 0, M = 0, n = 0, w = 0, nhi = 0, backend = 0, prec = 0, device = 0;
  int plan = 0;       // SA_PLAN_* options of sa_create_ex (0: every choice by the built-in rules)
  bool pow2 = true;  // M a power of two (the Hadamard kernels, bit-level glue)
  // the caller's section size Mu; the Hadamard backend pads a section of any
  // Mu to M = 2^ceil(log2 Mu) columns, the first dead = M - Mu of them never
  // used (column c of the reference is column dead + c: sparc_ldpc.py:54, 68)
  int Mu = 0, dead = 0;
  int G = 0, NZ = 0, E = 1;
  int n_cus = 256;
  int Gb = 0, CB = 0;  // batched kernel: groups of WB sections, codewords per workgroup (0 = off)
  int WB = 8;          // batched kernel: sections per workgroup (kWB or kWB16)
  int gpx = 1 << 20;   // batched kernel: section groups per XCD per pass (SecArgs::gpx)
  size_t secb_lds = 0;
  int RS = 1, KS = 1, Gd = 0;  // dense splits; Gd = dense denoiser groups
  size_t lda = 0;
  size_t sec_lds = 0;
  int G2 = 0;          // k_sec2 pairs of sections (0: k_sec2 unavailable)
  int G3 = 0;          // k_sec43 triples of sections (used when sec3)
  bool sec3 = false;   // k_sec43 (three sections x 4 waves per workgroup) chosen over k_sec4
  size_t sec3_lds = 0;
  uint32_t* d_fwd3 = nullptr;
  bool pt_on = false;  // row-block-major Ab partials between k_sec4 / k_sec43 and k_row2 (SecArgs::pt)
  bool sec4 = false;   // k_sec4 (4 waves per section) fits and is chosen
  size_t sec4_lds = 0;
  int NZ16 = 0;        // k_row2 32-row blocks; nz_cur = z^2 partial count of the current decode
  int NZh = 0;         // k_row2 16-row blocks (row16)
  bool row16 = false;  // k_row2<16> after k_sec4 (row-block-major partials, NZh <= 320)
  int NZ4 = 0, NZ2 = 0;  // k_rowv<4> 256-row / k_rowv<2> 128-row blocks
  int row_kind = 0;    // row kernel of the current decode: 0 k_row, 1 k_row2, 2 k_rowv<4>, 3 k_rowv<2>, 4 k_row2<16>, 5 k_rowc
  bool zil_last = false;  // the last decode left z codeword-interleaved ([NC][n][CB], zil_for)
  int nz_cur = 0;
  size_t sec2_lds = 0;
  std::vector<uint32_t> ordering;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint16_t* d_inv = nullptr;
  // operators whose z does not fit the section kernels' LDS (n >= 65535, or
  // the z image past 160 KB): k_secg with 32-bit bucket entries, no batched /
  // multi-wave kernels
  bool big = false;
  uint32_t* d_inv32 = nullptr;
  uint16_t* d_invb = nullptr;  // k_secb's bank-aware bucket table (build_invb), built on first batched use
  uint16_t* d_fwdb = nullptr;  // k_secb's Ab table, bank-aware step order per row (build_fwdb), the same
  uint16_t* d_invl = nullptr;  // the codeword-interleaved k_secb's bucket table, lane-major (k_lane_major)
  uint32_t* d_hs = nullptr;    // [L] occupied steps of d_invb's halves (build_banked)
  bool borrowed = false;       // the operator tables are another context's (sa_create_twin): not freed here
  bool invb_done = false;
  uint16_t* d_fwd = nullptr;
  uint32_t* d_fwd2 = nullptr;
  void* d_A = nullptr;  // dense [np][lda] design matrix (binary32; SA_BACKEND_MATRIX: the context precision)
  // int8 matrix-core dense path (B >= 4; dense_i8.hip): A8 [np8][LMp8], AT8 [LMp8][np8],
  // digit planes of z [3][Bp8][np8] and beta [3][Bp8][LMp8], per-codeword scales
  int8_t *d_A8 = nullptr, *d_AT8 = nullptr, *d_zq = nullptr, *d_bq = nullptr;
  double *d_zsc = nullptr, *d_bsc0 = nullptr, *d_bfix = nullptr;
  long long np8 = 0, LMp8 = 0;
  int Bp8 = 0;
  // caller's dense matrix (SA_BACKEND_MATRIX): rows padded to np (a whole
  // number of 256-row GEMM tiles); for B >= kFMinB codewords (dense_mfma.hip)
  // its transpose AT [LMy][nk] and the padded GEMM vectors xz [Bcap][nk] (z)
  // and xb [Bcap][lda] (beta, when L*M is not a whole number of K stages)
  long long np = 0, nk = 0, LMy = 0;
  void *d_AT = nullptr, *d_xz = nullptr, *d_xb = nullptr;
  int fg_cap = 0;
  double cmax = 0;  // max_l sqrt(n Pl_l) of the shared power allocation
  // workspace
  int Bcap = 0, Tcap = 0;
  void *d_y = nullptr, *d_z = nullptr, *d_beta = nullptr, *d_out = nullptr, *d_abp = nullptr;
  void *d_bbp = nullptr, *d_zzp = nullptr, *d_tau = nullptr, *d_c = nullptr, *d_azp = nullptr;
  int* d_iters = nullptr;
  int* d_stop = nullptr;  // host-operator loop: codewords whose exact-tau stop fired
  int32_t* d_idx = nullptr;
  double* d_stage = nullptr;
  size_t stage_cap = 0;
  double* d_cd = nullptr;  // c_l = sqrt(n Pl_l) in binary64 (joint-decoding glue)
  void* d_beta2 = nullptr;  // ping-pong partner of d_beta for k_sec (B x L*M), sized beta2_cap
  int beta2_cap = 0;
  double P = 0;
  bool power_set = false;
  // per-codeword power allocation (sa_stage_power_batch): c [Bcap][L], P [Bcap]
  void* d_cb = nullptr;
  void* d_Pb = nullptr;
  void* d_P1 = nullptr;  // the shared P = sum(Pl) of set_power (one `real`)
  bool pb_on = false;
  bool shared_power = false;  // sa_stage's Pl staged (c_l of the binary64 glue kernels)
  size_t bytes = 0;
  std::map<std::tuple<int, int, int, int>, hipGraphExec_t> graphs;
  int last_B = 0, last_T = 0;
  // pinned ring of sa_decide_async: SA_DECIDE_SLOTS slots of dec_cap indices
  int32_t* h_dec = nullptr;
  size_t dec_cap = 0;
  hipEvent_t dec_ev[SA_DECIDE_SLOTS] = {};
  int dec_B[SA_DECIDE_SLOTS] = {};
  // Monte-Carlo stream (sa_mc_stage / sa_mc_run, sa_mc.hip): the staged reps'
  // section indices [mc_cap][L] and noise [mc_cap][n], their decisions and stop
  // indices, the slot state of the refilled batch, and its captured graphs
  int mc_cap = 0, mc_nreps = 0;
  int32_t *d_mc_idx = nullptr, *d_mc_dec = nullptr, *d_mc_its = nullptr;
  double* d_mc_noise = nullptr;
  void *d_mc_y = nullptr, *d_mc_zzp = nullptr;  // the staged reps encoded: y [mc_cap][n], z^2 partials [mc_cap][NZ2]
  int* d_slots = nullptr;   // [4][slot_cap]: rep, t, done rep, fresh; then ctl {next, live, nreps}
  int slot_cap = 0;
  int* h_mc_live = nullptr;  // pinned ring of the live-slot counts the host polls
  hipEvent_t mc_ev[4] = {};
  const int* mc_tb = nullptr;  // the slots' t_b while an MC sequence is launched (SecArgs::tb)
  std::map<std::tuple<int, int, int, int>, hipGraphExec_t> mc_graphs;
  // host copies of the bucket table inv [L][w] and the Ab table fwd [G][n][4]
  // (build_tables), kept until the batched tables are built from them (ensure_invb)
  std::vector<uint16_t> h_inv, h_fwd;
};

namespace sa {

// Launch of a loop kernel on the context's stream, timed as sa_profile asks
// (plain launch when no profile is running).
template <typename F, typename... Args>
void plaunch(sa_ctx* c, F kernel, dim3 grid, dim3 block, size_t lds, Args... args) {
  if (c->prof && c->prof->dispatch) {
    hipEvent_t a = nullptr, b = nullptr;
    if (c->prof->add(&a, &b) == 0) {
      hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, c->stream, a, b, 0u, args...);
      return;
    }
  }
  const int nrep = c->prof ? c->prof->rep : 1;
  for (int r = 0; r < nrep; ++r) kernel<<<grid, block, lds, c->stream>>>(args...);
}


// ---- backend / kernel choice rules (shared by the units) --------------------
constexpr int kI8MinB = 4;   // dense backend: batches at least this large take the int8 GEMM path
constexpr int kI8MaxS = 16;  // K splits of the int8 A beta GEMM (its Ab partials)
constexpr int kFMinB = 4;    // matrix backend: batches at least this large take the f32 / f64 GEMM path
constexpr int kFMaxS = 16;   // K splits of its A beta GEMM

inline size_t rsz(const sa_ctx* c) { return c->prec == SA_PREC_F64 ? 8 : 4; }

// the dense backends: a materialised n x (L*M) matrix streamed by GEMVs
// (the Hadamard design's, or a caller's own: SA_BACKEND_MATRIX)
inline bool is_dense(const sa_ctx* c) { return c->backend == SA_BACKEND_DENSE || c->backend == SA_BACKEND_MATRIX; }
inline bool use_i8(const sa_ctx* c, int B) { return c->backend == SA_BACKEND_DENSE && B >= kI8MinB; }
inline bool use_fgemm(const sa_ctx* c, int B) { return c->backend == SA_BACKEND_MATRIX && B >= kFMinB; }
inline bool use_batched(const sa_ctx* c, int B) { return c->CB > 0 && B >= 4; }

// Two-waves-per-section kernel for the unbatched path when its G2 x B
// workgroups fill at least half of the CUs (otherwise k_sec's row splits do).
inline bool use_sec2(const sa_ctx* c, int B) {
  return c->backend == SA_BACKEND_HADAMARD && !use_batched(c, B) && c->G2 > 0 && c->G2 * B * 2 >= c->n_cus;
}

// Ab / beta^2 partials per codeword of the unbatched multi-wave section kernels
inline int sec2_parts(const sa_ctx* c) { return c->sec3 ? c->G3 : c->G2; }

// Row splits for small batches: enough workgroups to cover every CU.
inline int row_splits(const sa_ctx* c, int B) {
  const int wgs = c->G * B;
  int rs = (c->n_cus + wgs - 1) / wgs;
  return rs < 1 ? 1 : (rs > 4 ? 4 : rs);
}

// The batched decode with z and the Ab partials interleaved by codeword chunk
// (SecArgs::zil, 16-byte rows of CB codewords: binary32 CB = 4, binary64
// CB = 2), row kernel k_rowc.  The default in binary32 (C3 +1.7 %, C4
// +4.7 %) and, since the binary64 k_secb no longer spills (round 4: one
// bucket h-step in flight, 16-byte non-temporal beta), in binary64 too (C3
// 6.30 k -> 6.44 k, C4 3.09-3.12 k -> 3.19 k cw/s; round 3's spilling kernel
// lost 1.6 %); SA_PLAN_NO_ZIL keeps [B][n]
inline bool zil_for(const sa_ctx* c, int B) {
  const bool on = (c->plan & SA_PLAN_NO_ZIL) ? false : true;
  return on && c->backend == SA_BACKEND_HADAMARD && use_batched(c, B) && c->CB * (int)rsz(c) == 16;
}

// Row kernel for B codewords: k_row2 (32-row blocks) while B * ceil(n/64) <
// 4 CUs, else in binary32 k_rowv<4> (n % 4 == 0) or k_rowv<2> (n even) when
// their blocks cover the CUs twice, else k_row (64 rows); k_rowc behind the
// codeword-interleaved k_secb.
inline int row_kind_for(const sa_ctx* c, int B) {
  if (zil_for(c, B)) return 5;
  if ((long long)B * c->NZ < 4LL * c->n_cus) return (c->row16 && B == 1) ? 4 : 1;
  const bool f32 = c->prec == SA_PREC_F32;
  // 16-byte rows: binary32 n % 4 == 0 (256-row blocks) or binary64 n even (128)
  if (c->n % (f32 ? 4 : 2) == 0 && (long long)B * (f32 ? c->NZ4 : c->NZ2) >= 2LL * c->n_cus) return 2;
  if (f32 && c->n % 2 == 0 && (long long)B * c->NZ2 >= 2LL * c->n_cus) return 3;  // 8-byte rows
  return 0;
}
inline int nz_for(const sa_ctx* c, int kind) {
  const bool f32 = c->prec == SA_PREC_F32;
  if (kind == 4) return c->NZh;
  if (kind == 5) return c->NZ2;  // k_rowc: 128-row blocks
  return kind == 1 ? c->NZ16 : (kind == 2 ? (f32 ? c->NZ4 : c->NZ2) : (kind == 3 ? c->NZ2 : c->NZ));
}
inline void pick_row(sa_ctx* c, int B) {
  c->row_kind = row_kind_for(c, B);
  c->nz_cur = nz_for(c, c->row_kind);  // z^2 partials per codeword
}

// Ab partial layout between the pair / triple kernels and k_row2 (SecArgs::pt):
// rows per row-major block, 0 for the [G][n] layout
inline int pt_for(const sa_ctx* c, int B, bool sec2) {
  const int rk = row_kind_for(c, B);
  return (sec2 && (c->sec3 || c->sec4) && (rk == 1 || rk == 4) && c->pt_on) ? (rk == 4 ? 16 : kRow2Rows) : 0;
}

template <typename real>
SecArgs<real> sec_args(sa_ctx* c, int mode, int t, int early_stop) {
  SecArgs<real> a;
  a.inv = c->d_inv; a.inv32 = c->d_inv32; a.invb = c->d_invb; a.invl = c->d_invl; a.hs = c->d_hs;
  a.fwd = (const ushort4*)c->d_fwd;
  a.fwdb = (const ushort4*)c->d_fwdb; a.fwd2 = c->d_fwd2; a.fwd3 = c->d_fwd3; a.c = (const real*)c->d_c;
  a.z = (const real*)c->d_z; a.beta = (real*)c->d_beta; a.beta_out = (real*)c->d_beta; a.out = (real*)c->d_out;
  a.abp = (real*)c->d_abp; a.bbp = (real*)c->d_bbp; a.zzp = (const real*)c->d_zzp;
  a.tau = (real*)c->d_tau; a.iters = c->d_iters;
  a.L = c->L; a.M = c->M; a.n = c->n; a.w = c->w; a.nhi = c->nhi; a.G = c->G; a.NZ = c->nz_cur;
  a.T1 = c->Tcap + 1; a.t = t; a.mode = mode; a.early_stop = early_stop;
  a.RS = 1;
  a.pt = 0;
  a.B = 0; a.NC = 0; a.zil = 0; a.gpx = 1 << 20;
  a.cst = c->pb_on ? c->L : 0;
  if (c->pb_on) a.c = (const real*)c->d_cb;
  a.sqrt_n = (real)std::sqrt((double)c->n);
  a.tb = c->mc_tb;
  a.dead = c->dead;
  return a;
}

template <typename real>
RowArgs<real> row_args(sa_ctx* c, int mode, int t, int early_stop, int G, int Gb) {
  RowArgs<real> a;
  a.y = (const real*)c->d_y; a.z = (real*)c->d_z; a.z_in = a.z; a.abp = (const real*)c->d_abp;
  a.bbp = (const real*)c->d_bbp; a.zzp = (real*)c->d_zzp; a.tau = (const real*)c->d_tau;
  a.out = (real*)c->d_out;
  a.n = c->n; a.G = G; a.NZ = c->nz_cur;
  a.Gb = Gb; a.T1 = c->Tcap + 1; a.t = t; a.mode = mode;
  a.early_stop = early_stop;
  // the dense matrix already carries the 1/sqrt(n) of sparc_ldpc.py:143-146
  a.sqrt_n = c->backend != SA_BACKEND_HADAMARD ? (real)1 : (real)std::sqrt((double)c->n);
  a.Pb = c->pb_on ? (const real*)c->d_Pb : (const real*)c->d_P1;
  a.Pbst = c->pb_on ? 1 : 0;
  a.pt = 0;
  a.Bc = 0;
  a.tb = c->mc_tb;
  return a;
}

// f(i) for i in [0, count) over the host's cores (at most 16 threads), in
// contiguous blocks of `grain` (callers write disjoint outputs per block)
template <typename F>
void parallel_for(int count, int grain, F f) {
  const int blocks = (count + grain - 1) / grain;
  unsigned nth = std::thread::hardware_concurrency();
  nth = nth == 0 ? 1 : (nth > 16 ? 16 : nth);
  if ((int)nth > blocks) nth = blocks > 0 ? blocks : 1;
  auto run = [&](int t) {
    for (int b = t; b < blocks; b += (int)nth)
      for (int i = b * grain; i < count && i < (b + 1) * grain; ++i) f(i);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < (int)nth; ++t) th.emplace_back(run, t);
  run(0);
  for (auto& x : th) x.join();
}

// ---- defined in sparc_amp.hip ------------------------------------------------
int check_ctx(const sa_ctx* c);
int check_tables(const sa_ctx* c, const char* what);
int dev_alloc(sa_ctx* c, void** p, size_t bytes);
void dev_free(void* p);
void drop_graphs(sa_ctx* c);
int ensure_workspace(sa_ctx* c, int B, int T);
int ensure_stage(sa_ctx* c, size_t count);
int upload(sa_ctx* c, void* dst, const double* src, size_t count);
int download(sa_ctx* c, double* dst, const void* src, size_t count);
int set_power(sa_ctx* c, const double* Pl);
int ensure_invb(sa_ctx* c);
int create_impl(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int prec, int device,
                int plan, const sa_ctx* share = nullptr);
extern __global__ void k_fill32(uint32_t* p, uint32_t v, size_t nw);

// ---- sa_sec.hip: the single-codeword section kernels ---------------------------
template <typename real>
int launch_sec(sa_ctx* c, int B, int mode, int t, int es, void* bin = nullptr, void* bout = nullptr);
template <typename real>
int launch_sec2(sa_ctx* c, int B, int t, int es, void* bin, void* bout, int pt = 0);
hipError_t sec_lds_attrs();

// ---- sa_secb.hip: the batched section kernel ------------------------------------
template <typename real>
int launch_secb(sa_ctx* c, int B, int t, int es);
hipError_t secb_lds_attrs();
bool secb_no_static_lds();

// ---- sa_row.hip: row kernels, decisions ----------------------------------------
template <typename real>
int launch_row(sa_ctx* c, int B, int mode, int t, int es, int G, int Gb, int pt = 0, void* zin = nullptr,
               void* zout = nullptr);
int launch_decide(sa_ctx* c, int B);

// ---- sa_dense.hip: the materialised-matrix backends ----------------------------
int dense_parts(const sa_ctx* c, int B);  // Ab partials of the dense A beta (GEMM K splits or GEMV splits)
int dense_den_groups(const sa_ctx* c);
template <typename real>
int dense_start(sa_ctx* c, int B, int S);  // z = y - A beta0 (the beta0 start)
template <typename real>
int dense_iter(sa_ctx* c, int B, int t, int es, int S);  // A^T z -> denoiser -> A beta partials
template <typename real>
int dense_ab(sa_ctx* c, int B);  // A beta of d_beta -> d_out
template <typename real>
int dense_az(sa_ctx* c, int B);  // A^T z of d_z -> d_out
int ensure_i8(sa_ctx* c, int B);
int ensure_fgemm(sa_ctx* c, int B);
int i8_set_bfix(sa_ctx* c);
int build_dense(sa_ctx* c);
int matrix_init(sa_ctx* c);  // a caller's matrix: padded layout, zeroed d_A
hipError_t dense_lds_attrs();

// ---- sa_mc.hip: the Monte-Carlo rep stream ------------------------------------
void mc_release(sa_ctx* c);  // its buffers and graphs (sa_destroy)
hipError_t mc_lds_attrs();

#ifdef SA_STAMPS
hipError_t stamps_add_sec(unsigned long long* out);   // adds the unit's s_memtime stamps into out
hipError_t stamps_add_secb(unsigned long long* out);
#endif

}  // namespace sa
