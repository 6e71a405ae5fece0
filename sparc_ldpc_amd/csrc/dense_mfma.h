// dense_mfma.hip — batched products of a caller's dense design matrix
// (SA_BACKEND_MATRIX, e.g. an i.i.d. Gaussian design) on the matrix cores.
// Included by sparc_amp.hip inside its anonymous namespace (one translation
// unit, one code object).
//
// The reference's amp() takes any pair of callables (sparc_ldpc.py:189,213,
// 220); with a dense n x (L*M) matrix A they are Ab(beta) = A beta and
// Az(z) = A^T z.  For B >= 4 codewords both are GEMMs over a shared matrix,
// computed here in the context precision with exact-precision MFMAs:
//   binary32: v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate, one rounding per
//             product: bitwise a k-ordered fmaf chain; 157 TF/s dense peak)
//   binary64: v_mfma_f64_16x16x4_f64 (78.6 TF/s dense peak)
// Both GEMMs are "NT": out[b][y] = sum_k X[b][k] Y[y][k] with K contiguous in
// both operands — Ab: X = beta [B][LM], Y = A [np][lda]; Az: X = z (padded
// copy) [B][nk], Y = A^T [LMy][nk] (a transposed copy built on first batched
// use; 288 GB of HBM make the second copy cheap).
//
// Workgroup tile: 64 codewords x 256 matrix rows, 8 waves = 2 codeword halves
// x 4 row quarters (each wave 32 codewords x 64 rows); K streamed in 128-byte
// stages (32 binary32 / 16 binary64 per row), double-buffered in LDS
// (2 x 320 x 128 B = 80 KB: two workgroups per CU) by LDS-DMA
// (global_load_lds_dwordx4), the 16-B chunks of each 128-B LDS row
// XOR-swizzled by (row >> 1) & 7 as in dense_i8.hip.  K order inside a stage:
// a lane reads a whole 16-B chunk and feeds its elements to consecutive
// MFMAs, so the k-slots of one MFMA hold elements of different chunks; the
// sum still covers every k exactly once (X and Y lanes of one slot read the
// same chunk).  Work order XCD-grouped: the XT codeword tiles of one row tile
// and K split run on one XCD, so the row tile is fetched from HBM once and
// re-read from that XCD's L2.

constexpr int kFTX = 64;                       // codewords per workgroup tile
constexpr int kFTY = 256;                      // matrix rows per workgroup tile
constexpr int kFKB = 128;                      // K bytes per LDS row per stage
constexpr int kFStage = (kFTX + kFTY) * kFKB;  // 40960 B
constexpr int kFLds = 2 * kFStage;             // double buffered: 80 KB
constexpr int kFDma = (kFTX + kFTY) / 8;       // wave-level DMA instructions per stage (8 rows each)

template <typename real>
struct FArgs {
  const real* X;  // [rows][ldx]: the vectors, K contiguous; rows >= B are read clamped to B - 1
  const real* Y;  // [YT * 256][ldy]: matrix rows, K contiguous (zero rows / columns as padding)
  real* out;      // out[b * ldb + s * lds + y]
  long long ldx, ldy, ldb, lds;
  int nst, kps;   // K stages; stages per K split
  int XT, YT, S;  // codeword tiles, row tiles, K splits
  int B, Ny;      // valid codewords, valid rows
};

__device__ __forceinline__ int f_swz(int r) { return (r >> 1) & 7; }

template <typename real>
__device__ __forceinline__ void f_stage_load(const FArgs<real>& a, unsigned char* dst, int tx, int ty, long long kb,
                                             int wv, int lane) {
  const int slot = lane & 7, rsub = lane >> 3;
  const char* Xb = reinterpret_cast<const char*>(a.X);
  const char* Yb = reinterpret_cast<const char*>(a.Y);
#pragma unroll
  for (int i = 0; i < kFDma / 8; ++i) {
    const int q = wv + 8 * i;
    const char* src;
    unsigned char* d;
    if (q < kFTX / 8) {
      const int rr = 8 * q + rsub;
      const int b = min(tx * kFTX + rr, a.B - 1);
      src = Xb + ((long long)b * a.ldx) * (long long)sizeof(real) + kb + 16 * (slot ^ f_swz(rr));
      d = dst + q * 1024;
    } else {
      const int rr = 8 * (q - kFTX / 8) + rsub;
      src = Yb + ((long long)(ty * kFTY + rr) * a.ldy) * (long long)sizeof(real) + kb + 16 * (slot ^ f_swz(rr));
      d = dst + kFTX * kFKB + (q - kFTX / 8) * 1024;
    }
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)d, 16, 0, 0);
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <typename real>
struct FAcc;
template <>
struct FAcc<float> {  // 2 tiles of 32 x 32 per wave
  f32x16 acc[2];
};
template <>
struct FAcc<double> {  // 2 x 4 tiles of 16 x 16 per wave
  f64x4 acc[2][4];
};

// AB: 0 for A^T z, 1 for A beta — the same code, two names in the profiles
template <typename real, int AB>
__global__ void __launch_bounds__(512) k_gemm_f(FArgs<real> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nb = gridDim.x, bid = blockIdx.x, per = nb / 8;
  const int wk = bid < per * 8 ? (bid % 8) * per + bid / 8 : bid;
  const int tx = wk % a.XT, rest = wk / a.XT;
  const int ty = rest % a.YT, s = rest / a.YT;
  const int st0 = s * a.kps, st1 = min(a.nst, st0 + a.kps);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wx = wv & 1, wy = wv >> 1;

  FAcc<real> F;
  if constexpr (sizeof(real) == 4) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) F.acc[j][i] = 0.f;
  } else {
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int i = 0; i < 4; ++i) F.acc[ti][tj][i] = 0.0;
  }
  if (st0 < st1) {
    f_stage_load<real>(a, smem, tx, ty, (long long)st0 * kFKB, wv, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int st = st0; st < st1; ++st) {
    const int buf = (st - st0) & 1;
    if (st + 1 < st1) f_stage_load<real>(a, smem + (buf ^ 1) * kFStage, tx, ty, (long long)(st + 1) * kFKB, wv, lane);
    const unsigned char* sb = smem + buf * kFStage;
    if constexpr (sizeof(real) == 4) {
      // lane (r31, h): X row wx*32 + r31, Y rows wy*64 + j*32 + r31; chunk 2kk + h
      const int r31 = lane & 31, h = lane >> 5;
      const int xr = wx * 32 + r31;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int c = 2 * kk + h;
        const f4 xf = *reinterpret_cast<const f4*>(sb + xr * kFKB + ((c ^ f_swz(xr)) << 4));
        f4 yf[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int yr = wy * 64 + j * 32 + r31;
          yf[j] = *reinterpret_cast<const f4*>(sb + kFTX * kFKB + yr * kFKB + ((c ^ f_swz(yr)) << 4));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < 2; ++j) F.acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xf[e], yf[j][e], F.acc[j], 0, 0, 0);
      }
    } else {
      // lane (r15, q4): X rows wx*32 + ti*16 + r15, Y rows wy*64 + tj*16 + r15; chunk 4kk + q4
      const int r15 = lane & 15, q4 = lane >> 4;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = 4 * kk + q4;
        d2v xf[2], yf[4];
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
          const int xr = wx * 32 + ti * 16 + r15;
          xf[ti] = *reinterpret_cast<const d2v*>(sb + xr * kFKB + ((c ^ f_swz(xr)) << 4));
        }
#pragma unroll
        for (int tj = 0; tj < 4; ++tj) {
          const int yr = wy * 64 + tj * 16 + r15;
          yf[tj] = *reinterpret_cast<const d2v*>(sb + kFTX * kFKB + yr * kFKB + ((c ^ f_swz(yr)) << 4));
        }
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 4; ++tj)
              F.acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(xf[ti][e], yf[tj][e], F.acc[ti][tj], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next stage's DMA has landed (this wave's)
    __syncthreads();                                   // ... every wave's, and this stage is consumed
  }
  // epilogue
  if constexpr (sizeof(real) == 4) {
    // 32x32 C/D: col = lane & 31 (matrix row y), row = (i & 3) + 8 (i >> 2) + 4 (lane >> 5) (codeword)
    const int r31 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int y = ty * kFTY + wy * 64 + j * 32 + r31;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int b = tx * kFTX + wx * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (b < a.B && y < a.Ny) a.out[(long long)b * a.ldb + (long long)s * a.lds + y] = F.acc[j][i];
      }
    }
  } else {
    // f64 16x16 C/D: col = lane & 15 (matrix row y), row = (lane >> 4) + 4 i (codeword)
    const int r15 = lane & 15, q4 = lane >> 4;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj) {
        const int y = ty * kFTY + wy * 64 + tj * 16 + r15;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = tx * kFTX + wx * 32 + ti * 16 + q4 + 4 * i;
          if (b < a.B && y < a.Ny) a.out[(long long)b * a.ldb + (long long)s * a.lds + y] = F.acc[ti][tj][i];
        }
      }
  }
}

// B rows of len values (ld_src apart) into dst [B][ld_dst], zero beyond len.
template <typename real>
__global__ void k_pad_rows(const real* __restrict__ src, long long ld_src, long long len, real* __restrict__ dst,
                           long long ld_dst, int B) {
  const long long total = (long long)B * ld_dst;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / ld_dst, k = i % ld_dst;
    dst[i] = k < len ? src[b * ld_src + k] : (real)0;
  }
}

// AT[j][r] = A[r][j] for r < n, j < LM; zero elsewhere (AT: [rows_t][ld_t]).
// 64 x 64 tiles through LDS: coalesced reads of A rows and writes of AT rows.
template <typename real>
__global__ void __launch_bounds__(256) k_transpose(const real* __restrict__ A, long long lda, int n, long long LM,
                                                   real* __restrict__ AT, long long rows_t, long long ld_t) {
  __shared__ real tile[64][65];
  const long long j0 = (long long)blockIdx.x * 64, r0 = (long long)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int rr = ty; rr < 64; rr += 4) {
    const long long r = r0 + rr, j = j0 + tx;
    tile[rr][tx] = (r < n && j < LM) ? A[r * lda + j] : (real)0;
  }
  __syncthreads();
  for (int jj = ty; jj < 64; jj += 4) {
    const long long j = j0 + jj, r = r0 + tx;
    if (j < rows_t && r < ld_t) AT[j * ld_t + r] = tile[tx][jj];
  }
}

// ---- an i.i.d. Gaussian design generated on the device ----------------------
// (sa_create_matrix_random: the design of a simulation that never needs it on
// the host).  Philox4x32-10 (Salmon et al., SC'11) keyed by the seed, counter
// = element index / 4; its four 32-bit words give two Box-Muller pairs, i.e.
// four N(0, 1) values for four consecutive elements of a row-major n x (L*M)
// matrix: reproducible per (seed, element) whatever the launch shape.
__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

template <typename real>
__global__ void k_matrix_gauss(real* __restrict__ A, long long n, long long LM, size_t lda, unsigned long long seed,
                               double scale) {
  const long long total4 = (n * LM + 3) / 4;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < total4;
       q += (long long)gridDim.x * blockDim.x) {
    const uint4 w = philox4x32_10(make_uint4((uint32_t)q, (uint32_t)(q >> 32), 0u, 0u), key);
    const uint32_t u[4] = {w.x, w.y, w.z, w.w};
    double g[4];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const double u1 = ((double)u[2 * p] + 1.0) * (1.0 / 4294967296.0);  // (0, 1]
      const double u2 = (double)u[2 * p + 1] * (1.0 / 4294967296.0);      // [0, 1)
      const double rad = sqrt(-2.0 * log(u1));
      double sn, cs;
      sincospi(2.0 * u2, &sn, &cs);
      g[2 * p] = rad * cs;
      g[2 * p + 1] = rad * sn;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long e = q * 4 + i;
      if (e < n * LM) {
        const long long r = e / LM, j = e % LM;
        A[(size_t)r * lda + (size_t)j] = (real)(g[i] * scale);
      }
    }
  }
}
