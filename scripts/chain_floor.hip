// chain_floor.hip — the per-iteration floor of the single-codeword two-kernel
// AMP chain at C2 geometry (L = M = 512, n = 4608, w = 8192, fp32), measured
// with the product's own launch shapes but none of its arithmetic.
//
// One AMP iteration is a section kernel (256 workgroups x 512 threads: two
// sections each) followed by a row kernel (288 workgroups x 512 threads: 16 rows
// each), every workgroup of each depending on every workgroup of the other
// (z -> all sections, Ab partials -> all rows).  This program replays 64 such
// iterations as one hipGraph (the product's form) in three modes:
//   0 empty     both kernels return at once: the two dependent boundaries alone
//   1 data      the product's memory traffic with trivial arithmetic: the section
//               kernel stages z (18 KB) into LDS by LDS-DMA with the 288 z^2
//               partials and its 32 KB of bucket tables (one memory round trip),
//               then writes 4608 Ab partials (non-temporal, row-block-major,
//               16-row blocks); the row kernel reads its 16 x 256 partials
//               (one round trip), sums them, writes 16 z rows and a z^2 partial
//   2 data+rt   as 1, plus the Ab-table rows (18 KB per workgroup) loaded after
//               the first round trip and used by the partial stores (the
//               product's second, overlapped stream)
//   3 no-tables as 2 without the bucket tables (z, z^2 partials, Ab-table rows)
//   4 fwd-only  as 3 with the Ab-table rows in the FIRST round trip (what a
//               section kernel that built its bucket tables in LDS from the
//               Ab table would have to wait for; the scatter itself not modelled)
//   5 no-parts  as 2, but the row kernel reads no partials
//   6 sec-only  as 2 with no row kernel: one launch per iteration
// and reports microseconds per iteration (HIP events around 20 replays).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/chain_floor scripts/chain_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int L = 512, M = 512, N = 4608, W = 8192;
constexpr int G = L / 2;          // section workgroups = Ab partials per row
constexpr int R = 16;             // rows per row-kernel workgroup
constexpr int NB = N / R;         // 288 row workgroups = z^2 partials
constexpr int NT = 512;

struct Bufs {
  float* z;        // [N]
  float* zzp;      // [NB]
  float* abp;      // [NB][G][R]
  uint16_t* inv;   // [L][W]
  uint32_t* fwd;   // [G][N]
  float* sink;     // [G]
};

// P (partial hand-off policy, MODE 2): 0 non-temporal stores / plain 4-B loads
// (the product), 1 default stores, 2 write-through (sc1) stores, 3 non-temporal
// loads too, 4 plain 16-B loads (4 rows per lane), 5 default stores + 16-B loads
template <int MODE, int P = 0, int S = 2>
__global__ void __launch_bounds__(S * 256) k_sec_floor(Bufs b) {
  if constexpr (MODE == 0) return;
  constexpr int NT = S * 256, GS = L / S, KR = (N + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* zs = reinterpret_cast<float*>(smem);
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // z by LDS-DMA: 18 KB = 18 wave instructions of 1 KB
  for (int ch = wv; ch * 1024 < N * 4; ch += NT / 64)
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)((const char*)b.z + ch * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)((char*)zs + ch * 1024), 16, 0, 0);
  // z^2 partials (5 per lane) and the two sections' bucket tables (16 h-steps x 512 x 2 B per section)
  float zz = 0.f;
#pragma unroll
  for (int q = 0; q < 5; ++q) { const int i = lane + 64 * q; zz += b.zzp[i < NB ? i : 0]; }
  const int sec = g * S + (wv >> 2), quarter = wv & 3;
  const uint16_t* il = b.inv + (size_t)sec * W + quarter * 128;
  ushort4 tb[16];
#pragma unroll
  for (int h = 0; h < 16; ++h)
    tb[h] = (MODE == 3 || MODE == 4) ? make_ushort4(h, 0, 0, 0)
                                     : *reinterpret_cast<const ushort4*>(il + h * M + (lane & 31) * 4);
  uint32_t f[KR];
  if constexpr (MODE == 4) {
#pragma unroll
    for (int u = 0; u < KR; ++u) { const int r = u * NT + tid; f[u] = b.fwd[(size_t)g * N + (r < N ? r : 0)]; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned acc = 0;
#pragma unroll
  for (int h = 0; h < 16; ++h) acc += tb[h].x ^ tb[h].y ^ tb[h].z ^ tb[h].w;
  const float base = zz + (float)(acc & 1);
  if constexpr (MODE == 2 || MODE == 3 || MODE >= 5) {
#pragma unroll
    for (int u = 0; u < KR; ++u) { const int r = u * NT + tid; f[u] = b.fwd[(size_t)g * N + (r < N ? r : 0)]; }
  }
  // the Ab partials of this workgroup: row r at [r / R][g][r % R]
#pragma unroll
  for (int u = 0; u < KR; ++u) {
    const int r = u * NT + tid;
    if (r >= N) break;
    float t = zs[r] + base;
    if constexpr (MODE >= 2) t += zs[f[u] & 4095u];
    float* dst = &b.abp[((size_t)(r >> 4) * GS + g) * R + (r & 15)];
    if constexpr (P == 1 || P == 5) *dst = t;
    else if constexpr (P == 2) __hip_atomic_store(dst, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __builtin_nontemporal_store(t, dst);
  }
}

template <int MODE, int P = 0, int GP = G>
__global__ void __launch_bounds__(NT) k_row_floor(Bufs b) {
  if constexpr (MODE == 0) return;
  __shared__ float red[32][R + 1];
  const int tid = threadIdx.x, rl = tid & (R - 1), pg = tid / R;  // 32 groups of 8 partials
  if constexpr (P == 4 || P == 5) {
    // 16-B loads: the block's 256 x 16 partials as 1024 float4, two per lane;
    // lane (q = tid & 3 row quad, gg = tid >> 2 group) sums groups gg, gg + 128
    const float4* p4 = reinterpret_cast<const float4*>(b.abp + (size_t)blockIdx.x * G * R);
    const int q = tid & 3, gg = tid >> 2;
    const float4 a0 = p4[gg * 4 + q], a1 = p4[(gg + 128) * 4 + q];
    __shared__ float4 r4[128][4];
    r4[gg][q] = make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
    __syncthreads();
    if (tid < 32 * R / 4) {  // 128 threads: (row quad q, group of 4 gg4) -> red[gg4][4q..4q+3]
      const int qq = tid & 3, g4 = tid >> 2;
      float4 s4 = r4[g4 * 4][qq];
#pragma unroll
      for (int k = 1; k < 4; ++k) { const float4 x = r4[g4 * 4 + k][qq]; s4.x += x.x; s4.y += x.y; s4.z += x.z; s4.w += x.w; }
      red[g4][4 * qq] = s4.x; red[g4][4 * qq + 1] = s4.y; red[g4][4 * qq + 2] = s4.z; red[g4][4 * qq + 3] = s4.w;
    }
  } else {
    const float* p = b.abp + (size_t)blockIdx.x * GP * R + rl;
    constexpr int U = GP / 32;
    float t[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      t[u] = MODE == 5 ? (float)u : (P == 3 ? __builtin_nontemporal_load(p + (size_t)(pg + 32 * u) * R)
                                            : p[(size_t)(pg + 32 * u) * R]);
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += t[u];
    red[pg][rl] = acc;
  }
  __syncthreads();
  if (tid >= 64) return;
  float zn = 0.f;
  if (tid < R) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 32; ++q) s += red[q][rl];
    zn = s * 1e-3f;
    b.z[blockIdx.x * R + rl] = zn;
  }
  float sz = zn * zn;
  for (int o = 32; o > 0; o >>= 1) sz += __shfl_xor(sz, o);
  if (tid == 0) b.zzp[blockIdx.x] = sz;
}

template <int MODE, int P = 0, int S = 2>
double run(const Bufs& b, hipStream_t s, int iters, int reps) {
  hipGraph_t gr;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int t = 0; t < iters; ++t) {
    k_sec_floor<MODE, P, S><<<L / S, S * 256, N * 4 + 64, s>>>(b);
    if (MODE != 6) k_row_floor<MODE, P, L / S><<<NB, NT, 0, s>>>(b);
  }
  CK(hipStreamEndCapture(s, &gr));
  CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  std::vector<float> ms(reps);
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms[r], e0, e1));
  }
  std::sort(ms.begin(), ms.end());
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(gr));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms[reps / 2] * 1e3 / iters;  // median replay, us per iteration
}

int main() {
  Bufs b;
  CK(hipMalloc(&b.z, N * 4));
  CK(hipMalloc(&b.zzp, NB * 4));
  CK(hipMalloc(&b.abp, (size_t)NB * G * R * 4));
  CK(hipMalloc(&b.inv, (size_t)L * W * 2));
  CK(hipMalloc(&b.fwd, (size_t)G * N * 4));
  CK(hipMalloc(&b.sink, G * 4));
  CK(hipMemset(b.z, 0, N * 4));
  CK(hipMemset(b.zzp, 0, NB * 4));
  CK(hipMemset(b.abp, 0, (size_t)NB * G * R * 4));
  CK(hipMemset(b.inv, 0, (size_t)L * W * 2));
  CK(hipMemset(b.fwd, 0, (size_t)G * N * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int iters = 64, reps = 21;
  std::printf("us per iteration (64 iterations per graph replay, median of %d replays)\n", reps);
  for (int round = 0; round < 2; ++round) {
    double t[7];
    t[0] = run<0>(b, s, iters, reps); t[1] = run<1>(b, s, iters, reps); t[2] = run<2>(b, s, iters, reps);
    t[3] = run<3>(b, s, iters, reps); t[4] = run<4>(b, s, iters, reps); t[5] = run<5>(b, s, iters, reps);
    t[6] = run<6>(b, s, iters, reps);
    std::printf("round %d: 0 empty %.2f | 1 data %.2f | 2 data+Ab-table rows %.2f | 3 no bucket tables %.2f | "
                "4 Ab table in the first trip, no bucket tables %.2f | 5 row kernel reads no partials %.2f | "
                "6 section kernel only %.2f\n", round, t[0], t[1], t[2], t[3], t[4], t[5], t[6]);
    double q[6];
    q[0] = run<2, 0>(b, s, iters, reps); q[1] = run<2, 1>(b, s, iters, reps); q[2] = run<2, 2>(b, s, iters, reps);
    q[3] = run<2, 3>(b, s, iters, reps); q[4] = run<2, 4>(b, s, iters, reps); q[5] = run<2, 5>(b, s, iters, reps);
    std::printf("round %d, mode 2 partial hand-off: nt stores %.2f | default stores %.2f | sc1 stores %.2f | "
                "nt loads %.2f | 16-B loads %.2f | default stores + 16-B loads %.2f\n",
                round, q[0], q[1], q[2], q[3], q[4], q[5]);
    std::printf("round %d, mode 2 sections per section workgroup: 2 (256 partials) %.2f | 4 (128) %.2f ; "
                "section kernel only: 2 %.2f | 4 %.2f\n", round, run<2, 0, 2>(b, s, iters, reps),
                run<2, 0, 4>(b, s, iters, reps), run<6, 0, 2>(b, s, iters, reps), run<6, 0, 4>(b, s, iters, reps));
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
