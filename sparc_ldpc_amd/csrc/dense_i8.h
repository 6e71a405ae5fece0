// dense_i8.hip — batched dense backend on the matrix cores.
// Included by sparc_amp.hip inside its anonymous namespace (one translation
// unit, one code object).
//
// For B >= 4 codewords the dense operator products Ab = A beta and
// Az = A^T z (sparc_ldpc.py:143-146) of a whole batch are true GEMMs: the
// BASELINE north star's "MFMA only for the batched-codeword case where Ab/Az
// become true GEMMs".  A is exactly +-1/sqrt(n) (sparc_ldpc.py:65-77), so it is
// stored as int8 +-1 — A8 [np][LMp] for Ab and its transpose AT8 [LMp][np]
// for Az, both with the summed (K) index contiguous, 2 x 1.2 GB at
// L = M = 512 (a quarter of the fp32 matrix each) — and every vector operand
// v of codeword b is split into NP balanced base-256 int8 digits of the
// fixed-point integer X = rint(v * s_b), s_b a power of two with
// |X| <= 2^(8 NP - 2):
//     X = sum_p d_p 256^(NP-1-p),   d_p in [-128, 127] (|d_0| <= 65).
// NP = 3 for z (2^-23 of max|z_b|), NP = 4 for beta: beta has L*M entries,
// most of them tiny posteriors, quantised at one scale set by the largest
// section amplitude c_l, and three digits (2^-19 absolute at c = 6) left
// 1.5e-5 norm-relative at convergence on C2 — four digits (2^-27) keep the
// decode inside the fp32 contract.
// v_mfma_i32_32x32x32_i8 (int32 accumulate) computes each digit plane's
// product EXACTLY (|sum| <= 128 K < 2^31 for K <= 2^24), and the epilogue
// recombines the planes in binary64 (exact: |sum| < 2^50):
//     (A v)_r = (sum_p D_p 256^(NP-1-p)) / (s_b sqrt(n)).
// The only roundings are the fixed-point quantisation of v and the final
// rounding to binary32: fp32-class results at the int8 matrix rate (2x the
// bf16 rate per clock on gfx950).
//
// Workgroup tile: 64 codewords x NP digit planes (64 NP operand rows) x 256
// matrix rows, 8 waves = 2 codeword halves x 4 row quarters; each wave owns a
// 32-codeword x 64-row block per plane (NP x 2 MFMA 32x32 tiles, 32 NP int32
// accumulators per lane), so the planes of one output sit in the same lane
// and register and recombine with no data movement.  K is streamed in
// 128-byte stages by LDS-DMA (global_load_lds_dwordx4, 1 KB per wave
// instruction): the digit planes (an L2 / Infinity Cache stream, re-read by
// every row tile) one stage ahead in two buffers, the matrix rows (the HBM
// stream) two stages ahead in three — 2 x 64 NP x 128 + 3 x 256 x 128 B =
// 160 KB at NP = 4; the 16-byte chunks of every 128-byte LDS row are
// XOR-swizzled by (row >> 1) & 7 so the operand reads (ds_read_b128, 16 rows
// per lane group) are bank-conflict free.

constexpr int kI8TX = 64;               // codewords per workgroup tile
constexpr int kI8TY = 256;              // matrix rows per workgroup tile
constexpr int kI8KS = 128;              // K bytes per LDS stage
constexpr int kI8NPZ = 3, kI8NPB = 4;   // digit planes of z and of beta
template <int NP> struct I8Tile {
  static constexpr int XR = NP * kI8TX;                // operand (digit-plane) rows per stage
  static constexpr int XStage = XR * kI8KS;            // 24 / 32 KB
  static constexpr int YStage = kI8TY * kI8KS;         // 32 KB
  static constexpr int Lds = 2 * XStage + 3 * YStage;  // X double-, Y triple-buffered: 144 / 160 KB
  static constexpr int DmaX = XR / 8;                  // wave-level DMA instructions per stage: X rows
  static constexpr int DmaY = kI8TY / 8;               // ... Y rows
  static constexpr int YPerWave = DmaY / 8;            // Y instructions per wave per stage (4)
};
constexpr int kI8LdsMax = I8Tile<kI8NPB>::Lds;

typedef int i8v4 __attribute__((ext_vector_type(4)));    // 16 int8 operands
typedef int i8acc __attribute__((ext_vector_type(16)));  // 32x32 int32 tile per wave

struct I8Args {
  const int8_t* X;      // [NP][Bp][K] digit planes of the vectors (plane stride xps)
  const int8_t* Y;      // [YT * 256][K] the +-1 matrix, K contiguous
  float* out;           // out[b * ldb + s * lds + y]
  const double* scale;  // per codeword 1 / (s_b sqrt(n)); stride sst (0: one shared value)
  long long xps, K, ldb, lds;
  int nst, kps;         // K stages; stages per K split
  int XT, YT, S;        // codeword tiles, row tiles, K splits
  int B, Ny, sst;       // valid codewords, valid rows
};

__device__ __forceinline__ int i8_swz(int r) { return (r >> 1) & 7; }

// One stage (128 K bytes) of the X (digit-plane) or Y (matrix) tile into
// LDS: wave instructions of 1 KB, DmaX / 8 or DmaY / 8 per wave; lane i of an
// instruction fills LDS row 8q + i/8, 16-B slot i%8, with the global chunk
// (i%8) ^ swz(row).
template <int NP>
__device__ __forceinline__ void i8_load_x(const I8Args& a, unsigned char* dst, int tx, long long k0, int wv, int lane) {
  using Tl = I8Tile<NP>;
  const int slot = lane & 7, rsub = lane >> 3;
#pragma unroll
  for (int i = 0; i < Tl::DmaX / 8; ++i) {
    const int q = wv + 8 * i;
    const int rr = 8 * q + rsub;  // X tile row: plane rr / 64, codeword rr % 64
    const int p = rr / kI8TX, cw = rr % kI8TX;
    const int8_t* src = a.X + (long long)p * a.xps + (long long)(tx * kI8TX + cw) * a.K + k0 + 16 * (slot ^ i8_swz(rr));
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, 0, 0);
  }
}
template <int NP>
__device__ __forceinline__ void i8_load_y(const I8Args& a, unsigned char* dst, int ty, long long k0, int wv, int lane) {
  using Tl = I8Tile<NP>;
  const int slot = lane & 7, rsub = lane >> 3;
#pragma unroll
  for (int i = 0; i < Tl::YPerWave; ++i) {
    const int q = wv + 8 * i;
    const int rr = 8 * q + rsub;
    const int8_t* src = a.Y + (long long)(ty * kI8TY + rr) * a.K + k0 + 16 * (slot ^ i8_swz(rr));
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, 0, 0);
  }
}

template <int NP>
__global__ void __launch_bounds__(512) k_gemm_i8(I8Args a) {
  using Tl = I8Tile<NP>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // XCD-aware work order: blocks b and b + 8 share an XCD, so consecutive
  // work items (the XT codeword tiles of one row tile and K split) are dealt
  // to one XCD, where they run together: the row tile comes from HBM once and
  // is re-read from that XCD's L2 (placement is a speed matter only).
  const int nb = gridDim.x, bid = blockIdx.x, per = nb / 8;
  const int wk = bid < per * 8 ? (bid % 8) * per + bid / 8 : bid;
  const int tx = wk % a.XT, rest = wk / a.XT;
  const int ty = rest % a.YT, s = rest / a.YT;
  const int st0 = s * a.kps, st1 = min(a.nst, st0 + a.kps);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wx = wv & 1, wy = wv >> 1;

  i8acc acc[NP][2];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[p][j][i] = 0;
  // the epilogue's per-codeword scales, loaded now so their latency hides
  // behind the K loop (codeword of accumulator register i: see the epilogue)
  const int h = lane >> 5;
  double scl[4][4];
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = tx * kI8TX + wx * 32 + i + 8 * g4 + 4 * h;
      scl[g4][i] = a.scale[(long long)(b < a.B ? b : 0) * a.sst];
    }

  // X buffers at 0 and XStage, Y buffers at 2 XStage + {0, 1, 2} YStage
  unsigned char* const xbuf = smem;
  unsigned char* const ybuf = smem + 2 * Tl::XStage;
  static_assert(Tl::YPerWave == 4, "the vmcnt immediates below count 4 Y loads per wave");
  if (st0 < st1) {
    i8_load_x<NP>(a, xbuf, tx, (long long)st0 * kI8KS, wv, lane);
    i8_load_y<NP>(a, ybuf, ty, (long long)st0 * kI8KS, wv, lane);
    if (st0 + 1 < st1) {
      i8_load_y<NP>(a, ybuf + Tl::YStage, ty, (long long)(st0 + 1) * kI8KS, wv, lane);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // stage st0's loads (Y of st0 + 1 may fly on)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  const int r31 = lane & 31;
  // LDS byte offsets of this lane's operand rows (chunk c of row r at
  // r * 128 + ((c ^ swz(r)) << 4)); the swizzle only depends on r
  int xo[NP], yo[2], xz[NP], yz[2];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int r = p * kI8TX + wx * 32 + r31;
    xo[p] = r * kI8KS;
    xz[p] = i8_swz(r);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = wy * 64 + j * 32 + r31;
    yo[j] = r * kI8KS;
    yz[j] = i8_swz(r);
  }
#ifdef SA_STAMPS
  // diagnostic build only: the in-kernel clock over the K loop of block 0
  // (s_memtime counts shader clocks, s_memrealtime a constant 100 MHz)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g_stamps[12] = __builtin_amdgcn_s_memtime();
    g_stamps[13] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  int yb = 0;  // (st - st0) % 3
  for (int st = st0; st < st1; ++st) {
    const int xi = (st - st0) & 1;
    // the buffers stage st - 1 read (freed by the barrier that ended it):
    // X of st + 1, then Y of st + 2
    if (st + 1 < st1) i8_load_x<NP>(a, xbuf + (xi ^ 1) * Tl::XStage, tx, (long long)(st + 1) * kI8KS, wv, lane);
    const bool y2 = st + 2 < st1;
    if (y2) {
      const int yn = yb == 0 ? 2 : yb - 1;  // (st + 2) % 3
      i8_load_y<NP>(a, ybuf + yn * Tl::YStage, ty, (long long)(st + 2) * kI8KS, wv, lane);
    }
    const unsigned char* sbx = xbuf + xi * Tl::XStage;
    const unsigned char* sby = ybuf + yb * Tl::YStage;
    // operand fragments double-buffered across the four 32-deep K steps:
    // step kk + 1's LDS reads issue one between each pair of step kk's MFMAs
    // (sched_group_barrier), so the wait before a step's MFMAs is for reads
    // issued a whole step earlier: c3 Aβ GEMM 1.09 -> 1.03 ms
    i8v4 xf[2][NP], yf[2][2];
#pragma unroll
    for (int kk = 0; kk <= kI8KS / 32; ++kk) {
      if (kk < kI8KS / 32) {
        const int c = 2 * kk + h;  // this lane's 16-B chunk of the 32-deep K step
#pragma unroll
        for (int p = 0; p < NP; ++p) xf[kk & 1][p] = *reinterpret_cast<const i8v4*>(sbx + xo[p] + ((c ^ xz[p]) << 4));
#pragma unroll
        for (int j = 0; j < 2; ++j) yf[kk & 1][j] = *reinterpret_cast<const i8v4*>(sby + yo[j] + ((c ^ yz[j]) << 4));
      }
      if (kk > 0) {
        const int q = (kk - 1) & 1;
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[p][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(xf[q][p], yf[q][j], acc[p][j], 0, 0, 0);
      }
      // one next-step read between consecutive MFMAs (the step's reads were
      // issued during the previous step's MFMAs)
      if (kk > 0 && kk < kI8KS / 32) {
#pragma unroll
        for (int u = 0; u < NP + 2; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NP - (NP + 2), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // stage st + 1's X and Y have landed (this wave's; Y of st + 2, issued
    // last, may still fly), then the barrier: every wave's, and stage st is consumed
    if (y2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    yb = yb == 2 ? 0 : yb + 1;
  }

#ifdef SA_STAMPS
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g_stamps[14] = __builtin_amdgcn_s_memtime();
    g_stamps[15] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  // epilogue: C/D layout col = lane & 31 (matrix row y), row = (i & 3) + 8 (i >> 2) + 4 (lane >> 5)
  // (codeword); the planes of (b, y) are the same register of acc[0..NP-1]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int y = ty * kI8TY + wy * 64 + j * 32 + r31;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int b = tx * kI8TX + wx * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (b < a.B && y < a.Ny) {
        double v = 0.0;
#pragma unroll
        for (int p = 0; p < NP; ++p) v = v * 256.0 + (double)acc[p][j][i];
        a.out[(long long)b * a.ldb + (long long)s * a.lds + y] = (float)(v * scl[i >> 2][i & 3]);
      }
    }
  }
}

// Balanced base-256 digits of X (|X| <= 2^(8 NP - 2)), most significant first:
// X = sum_p d[p] 256^(NP-1-p).
template <int NP>
__device__ __forceinline__ void i8_digits(int X, int (&d)[NP]) {
#pragma unroll
  for (int p = NP - 1; p > 0; --p) {
    d[p] = ((X + 128) & 255) - 128;
    X = (X - d[p]) >> 8;  // exact
  }
  d[0] = X;
}
template <int NP> constexpr int i8_bits() { return 8 * NP - 2; }  // |X| <= 2^bits

// Quantise one vector per codeword (workgroup b): s_b = 2^(bits - E) with
// max|v_b| < 2^E, digits into q[p][b][:len] (the padding stays zero), and
// sc[b] = post / s_b (post = 1/sqrt(n): the epilogue's scale).
template <int NP>
__global__ void __launch_bounds__(256) k_i8_quant(const float* __restrict__ src, long long ld_src, int len,
                                                  int8_t* __restrict__ q, long long qps, long long ldq,
                                                  double* __restrict__ sc, double post) {
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* x = src + (long long)b * ld_src;
  float m = 0.f;
  for (int i = tid; i < len; i += 256) m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if (lane == 0) red[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int E = 0;
  if (m > 0.f) (void)frexp((double)m, &E);  // m < 2^E
  const double s = ldexp(1.0, i8_bits<NP>() - E);
  if (tid == 0) sc[b] = post / s;
  int8_t* qb = q + (long long)b * ldq;
  for (int i = tid * 4; i < len; i += 1024) {
    if (i + 4 <= len) {
      int d[4][NP];
#pragma unroll
      for (int u = 0; u < 4; ++u) i8_digits<NP>((int)rint((double)x[i + u] * s), d[u]);
#pragma unroll
      for (int p = 0; p < NP; ++p)
        *reinterpret_cast<char4*>(qb + p * qps + i) = make_char4(d[0][p], d[1][p], d[2][p], d[3][p]);
    } else {
      for (int u = i; u < len; ++u) {
        int d[NP];
        i8_digits<NP>((int)rint((double)x[u] * s), d);
#pragma unroll
        for (int p = 0; p < NP; ++p) qb[p * qps + u] = (int8_t)d[p];
      }
    }
  }
}

// The +-1 matrix as int8: A8[r][j] (rows r < n, K = j) or, transposed,
// AT8[j][r]; A[r, l*M + c] = (-1)^popcount(ordering[l][r] & (w - M + c))
// (sparc_ldpc.py:65-77; the 1/sqrt(n) goes into the epilogue scale).
// Padding rows / columns are zero.  Each thread writes 16 bytes.
__global__ void k_i8_build(const uint32_t* __restrict__ ord, int8_t* __restrict__ D, int L, int M, int n, int w,
                           long long rows, long long cols, int transposed) {
  const long long LM = (long long)L * M;
  const long long n16 = rows * (cols / 16);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n16; t += (long long)gridDim.x * blockDim.x) {
    const long long row = t / (cols / 16), c0 = (t % (cols / 16)) * 16;
    char v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const long long col = c0 + u;
      const long long r = transposed ? col : row, j = transposed ? row : col;
      int8_t s = 0;
      if (r < n && j < LM) {
        const int l = (int)(j / M), cc = (int)(j % M);
        const uint32_t o = ord[(long long)l * n + r];
        s = (__popc(o & (uint32_t)(w - M + cc)) & 1) ? -1 : 1;
      }
      v[u] = (char)s;
    }
    *reinterpret_cast<int4*>(D + row * cols + c0) = *reinterpret_cast<const int4*>(v);
  }
}
