// sa_sec.hip — the single-codeword section kernels (k_sec, k_secg, k_sec2,
// k_sec4, k_sec43) and their launchers.
#include "sa_host.h"

namespace sa {


// One workgroup = 4 wavefronts = 4 consecutive sections of one codeword
// (blockIdx.y).  Per wave: v = bucket gather of z (LDS), M-point FWHT,
// denoise, FWHT of the new beta (the Ab operand), staged to LDS.  Then the
// workgroup gathers its 4 sections' contributions to every row of Ab into
// abp[b][g][:].  Loads independent of z (bucket table, previous beta) are
// issued before the z barrier so their latency overlaps.

template <typename real, int E>
__global__ void __launch_bounds__(256) k_sec(SecArgs<real> a) {
  STAMP(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int KH = E >= 16 ? 2 : (E >= 8 ? 16 : 16);
  constexpr int NQ = (E + 3) / 4;
  constexpr int KR = 8;  // rows per thread whose Ab-table loads are in flight together
  // The RS workgroups of a section group read the same bucket tables and
  // previous estimate: place them on one XCD (workgroup j runs on XCD j % 8)
  // so the second reader is served by that XCD's L2.
  int g, rsi;
  if (a.RS > 1 && (a.G & 7) == 0) {
    const int j = blockIdx.x, u = j >> 3;
    rsi = u % a.RS;
    g = (u / a.RS) * 8 + (j & 7);
  } else {
    g = blockIdx.x / a.RS;
    rsi = blockIdx.x % a.RS;
  }
  const int b = blockIdx.y;
  const int rows_per = (a.n + a.RS - 1) / a.RS;
  const int rb0 = rsi * rows_per, rb1 = min(a.n, rb0 + rows_per);
  const bool owner = rsi == 0;  // writes beta / beta^2 / tau for the group
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = a.M, n = a.n;
  const size_t LM = (size_t)a.L * M;
  const int mlanes = M < 64 ? M : 64;
  const int l = g * kSpw + wv;
  const bool have = l < a.L;
  const int lc = have ? l : a.L - 1;  // clamped section for unconditional loads

  real* zs = reinterpret_cast<real*>(smem);
  const int zslots = ((n + 1) * (int)sizeof(real) + 15) / 16 * 16 / (int)sizeof(real);
  real* ts = zs + zslots;     // [kSpw][M]
  real* bbw = ts + kSpw * M;  // [kSpw]

  real v[E];
  real bprev[E];
  real* bl = a.beta + (size_t)b * LM + (size_t)lc * M;
  // The RS workgroups of a group all read beta_l(t) while the owner writes
  // beta_l(t+1): the two live in different buffers (ping-pong), otherwise a
  // late reader would see the new estimate.
  real* blo = a.beta_out + (size_t)b * LM + (size_t)lc * M;
  const uint16_t* il = a.inv + (size_t)lc * a.w;
  const ushort4* fw = a.fwd + (size_t)g * n;
  ushort4 tb[KH][NQ];
  ushort4 f[KR];

  if (a.mode == SEC_AB) {
    load_section<real, E>(bl, v, lane, M);
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      const int r = rb0 + u * 256 + tid;
      f[u] = fw[r < rb1 ? r : 0];
    }
  } else {
    // Every load that does not depend on z is issued together with the z
    // loads (one round trip), in the order they are needed (vmcnt retires
    // them in order): the z^2 partials and tau_{t-1} for the stop test, z
    // (16-B loads, whole 4 KB chunks), the first bucket-table chunk, the
    // previous beta, c_l, the first Ab-table rows.
    const real* zzb = a.zzp + (size_t)b * a.NZ;
    ZZParts<real> zz;
    real last = 0;
    if (a.mode == SEC_AMP) {
      zz.issue(zzb, a.NZ, lane);
      if (a.t > 0) last = ld_vmem(a.tau + (size_t)b * a.T1 + a.t - 1);
    }
    const real* zb = a.z + (size_t)b * n;
    ZStage<real> zst;
    const bool dma = stage_z_dma<real, 256>(zb, zs, n, tid);
    if (!dma) zst.issue(zb, n, tid);
    load_buckets<E, KH>(il, 0, a.nhi, M, lane, tb);
    if (a.mode == SEC_AMP) load_section<real, E>(bl, bprev, lane, M);
    const real cl = ld_vmem(a.c + (size_t)b * a.cst + lc);
    if (a.mode == SEC_AMP) {
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int r = rb0 + u * 256 + tid;
        f[u] = fw[r < rb1 ? r : 0];
      }
    }
    real tau2 = 1;
    if (a.mode == SEC_AMP) {
      const real tau = zz.tau(zzb, a.NZ, n);
      const bool stop = a.early_stop && (tau == last);
      if (blockIdx.x == 0 && tid == 0) {
        a.tau[(size_t)b * a.T1 + a.t] = tau;
        if (stop && a.iters[b] < 0) a.iters[b] = a.t;
      }
      if (stop) {  // uniform over the grid row: beta, z stay as they are
        if (dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write may outlive the workgroup
        return;
      }
      tau2 = tau * tau;
    }
    STAMP(1);
    if (!dma) zst.store(zs, zb, n, tid);
    else finish_z_dma(zb, zs, n, tid);
    __syncthreads();
  STAMP(2);

#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = 0;
    for (int h0 = 0; h0 < a.nhi; h0 += KH) {
      ushort4 tn[KH][NQ];
      const bool more = h0 + KH < a.nhi;
      if (more) load_buckets<E, KH>(il, h0 + KH, a.nhi, M, lane, tn);
      gather_buckets<real, E, KH>(zs, h0, a.nhi, tb, v);
      if (more) {
#pragma unroll
        for (int hh = 0; hh < KH; ++hh)
#pragma unroll
          for (int j = 0; j < NQ; ++j) tb[hh][j] = tn[hh][j];
      }
    }
  STAMP(3);
    fwht_wave<real, E>(v, lane, E >= 2 ? 64 : mlanes);  // E >= 2: M = 64 E, every lane
  STAMP(4);
    if (a.mode == SEC_AZ) {
      if (have && owner) {
        real* ol = a.out + (size_t)b * LM + (size_t)l * M;
#pragma unroll
        for (int i = 0; i < E; ++i) v[i] = v[i] / a.sqrt_n;
        store_section<real, E>(ol, v, lane, M);
      }
      return;  // uniform: no barrier follows in this mode
    }
    if (have) {
      const real bb = denoise_section<real, E>(v, bprev, blo, lane, M, cl, tau2, a.sqrt_n, owner, a.dead);
      if (lane == 0) bbw[wv] = bb;  // per-wave beta^2, summed below in section order
  STAMP(5);
    }
  }
  if (have) {
    fwht_wave<real, E>(v, lane, E >= 2 ? 64 : mlanes);  // T_l = H_M beta_l
  STAMP(6);
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = 0;  // missing section of the last group
    if (lane == 0) bbw[wv] = 0;
  }
  {
    real* tl = ts + wv * M;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = elem_index<E>(lane, i);
      if (e < M) tl[e] = v[i];
    }
  }
  __syncthreads();
  STAMP(7);
  if (a.mode == SEC_AMP && tid == 0 && owner)
    a.bbp[(size_t)b * a.G + g] = ((bbw[0] + bbw[1]) + bbw[2]) + bbw[3];
  // Ab partial of this group's 4 sections for this workgroup's rows: one
  // 8-B table load per row (the 4 sections' (k, sign) of that row).
  real* abp = a.abp + ((size_t)b * a.G + g) * n;
  for (int r0 = rb0; r0 < rb1; r0 += 256 * KR) {
    ushort4 fn[KR];
    const bool more = r0 + 256 * KR < rb1;
    if (more) {
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int r = r0 + 256 * KR + u * 256 + tid;
        fn[u] = fw[r < rb1 ? r : 0];
      }
    }
    real acc[KR];
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      const real v0 = ts[0 * M + (f[u].x & 0x7fffu)];
      const real v1 = ts[1 * M + (f[u].y & 0x7fffu)];
      const real v2 = ts[2 * M + (f[u].z & 0x7fffu)];
      const real v3 = ts[3 * M + (f[u].w & 0x7fffu)];
      real t = (f[u].x & 0x8000u) ? -v0 : v0;
      t += (f[u].y & 0x8000u) ? -v1 : v1;
      t += (f[u].z & 0x8000u) ? -v2 : v2;
      t += (f[u].w & 0x8000u) ? -v3 : v3;
      acc[u] = t;
    }
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      const int r = r0 + u * 256 + tid;
      if (r < rb1) st_part(&abp[r], acc[u]);
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < KR; ++u) f[u] = fn[u];
    }
  }
#ifdef SA_STAMPS
  STAMP(8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(9);
#endif
}


// ---------------------------------------------------------------------------
// Section kernel for operators whose z does not fit the section kernels' LDS
// image (n past ~38000 in binary32), including every n >= 65535, whose row
// indices need more than the 16-bit bucket entries: k_sec's structure (4
// sections per workgroup, one wave each, RS workgroups splitting the rows,
// sparc_ldpc.py:120-134 per section) with the bucket gather reading z from
// global memory (one codeword's z, 4 or 8 B x n, stays in the XCD's L2)
// through 32-bit entries inv32 [L][w] (row index, or n for an empty slot,
// which contributes 0).  The sums run in h order, as in k_sec.  LDS holds
// only the 4 sections' T = H_M beta (Ab partials) and their beta^2.
// ---------------------------------------------------------------------------
template <typename real, int E>
__global__ void __launch_bounds__(256) k_secg(SecArgs<real> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int g = blockIdx.x / a.RS, rsi = blockIdx.x % a.RS;
  const int b = blockIdx.y;
  const int rows_per = (a.n + a.RS - 1) / a.RS;
  const int rb0 = rsi * rows_per, rb1 = min(a.n, rb0 + rows_per);
  const bool owner = rsi == 0;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = a.M, n = a.n;
  const size_t LM = (size_t)a.L * M;
  const int mlanes = M < 64 ? M : 64;
  const int l = g * kSpw + wv;
  const bool have = l < a.L;
  const int lc = have ? l : a.L - 1;
  real* ts = reinterpret_cast<real*>(smem);  // [kSpw][M]
  real* bbw = ts + kSpw * M;                 // [kSpw]
  real v[E];
  real* bl = a.beta + (size_t)b * LM + (size_t)lc * M;
  real* blo = a.beta_out + (size_t)b * LM + (size_t)lc * M;
  if (a.mode == SEC_AB) {
    load_section<real, E>(bl, v, lane, M);
  } else {
    real bprev[E];
    real tau2 = 1;
    const real cl = ld_vmem(a.c + (size_t)b * a.cst + lc);
    if (a.mode == SEC_AMP) {
      const real* zzb = a.zzp + (size_t)b * a.NZ;
      const real tau = tau_from_parts(zzb, a.NZ, n);  // sparc_ldpc.py:203
      const real last = a.t > 0 ? a.tau[(size_t)b * a.T1 + a.t - 1] : (real)0;
      const bool stop = a.early_stop && (tau == last);  // :204-209
      if (blockIdx.x == 0 && tid == 0) {
        a.tau[(size_t)b * a.T1 + a.t] = tau;
        if (stop && a.iters[b] < 0) a.iters[b] = a.t;
      }
      if (stop) return;  // uniform over the grid row: beta, z stay as they are
      tau2 = tau * tau;
      load_section<real, E>(bl, bprev, lane, M);
    }
    // bucket gather (:128-134): v[k] = sum_h sgn(h) z[inv[h M + k]], h order
    const real* zb = a.z + (size_t)b * n;
    const uint32_t* il = a.inv32 + (size_t)lc * a.w;
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = 0;
    for (int h = 0; h < a.nhi; ++h) {
      const bool neg = __popc(h) & 1;
      const uint32_t* ih = il + (size_t)h * M;
      real zv[E];
#pragma unroll
      for (int i = 0; i < E; ++i) {
        const int e = elem_index<E>(lane, i);
        const uint32_t r = ih[e < M ? e : 0];
        zv[i] = (e < M && r < (uint32_t)n) ? zb[r] : (real)0;
      }
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] += neg ? -zv[i] : zv[i];
    }
    fwht_wave<real, E>(v, lane, E >= 2 ? 64 : mlanes);
    if (a.mode == SEC_AZ) {
      if (have && owner) {
        real* ol = a.out + (size_t)b * LM + (size_t)l * M;
#pragma unroll
        for (int i = 0; i < E; ++i) v[i] = v[i] / a.sqrt_n;
        store_section<real, E>(ol, v, lane, M);
      }
      return;  // uniform: no barrier follows in this mode
    }
    if (have) {
      const real bb = denoise_section<real, E>(v, bprev, blo, lane, M, cl, tau2, a.sqrt_n, owner, a.dead);
      if (lane == 0) bbw[wv] = bb;
    }
  }
  if (have) {
    fwht_wave<real, E>(v, lane, E >= 2 ? 64 : mlanes);  // T_l = H_M beta_l
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = 0;
    if (lane == 0) bbw[wv] = 0;
  }
  {
    real* tl = ts + wv * M;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int e = elem_index<E>(lane, i);
      if (e < M) tl[e] = v[i];
    }
  }
  __syncthreads();
  if (a.mode == SEC_AMP && tid == 0 && owner)
    a.bbp[(size_t)b * a.G + g] = ((bbw[0] + bbw[1]) + bbw[2]) + bbw[3];
  // Ab partial of the group's 4 sections for this workgroup's rows (:120-126)
  const ushort4* fw = a.fwd + (size_t)g * n;
  real* abp = a.abp + ((size_t)b * a.G + g) * n;
  for (int r = rb0 + tid; r < rb1; r += 256) {
    const ushort4 f = fw[r];
    const real v0 = ts[0 * M + (f.x & 0x7fffu)];
    const real v1 = ts[1 * M + (f.y & 0x7fffu)];
    const real v2 = ts[2 * M + (f.z & 0x7fffu)];
    const real v3 = ts[3 * M + (f.w & 0x7fffu)];
    real t = (f.x & 0x8000u) ? -v0 : v0;
    t += (f.y & 0x8000u) ? -v1 : v1;
    t += (f.z & 0x8000u) ? -v2 : v2;
    t += (f.w & 0x8000u) ? -v3 : v3;
    st_part(&abp[r], t);
  }
}

// ---------------------------------------------------------------------------
// Single-codeword section kernel, two wavefronts per section (M >= 128)
// ---------------------------------------------------------------------------
// One workgroup = 2 sections x 2 wavefronts; wave w of a section holds the
// half of its M entries whose top index bit is w (E2 = M/128 per lane, the
// k_sec element layout within the half).  Compared with k_sec (one wave per
// section, 4 sections per workgroup, the rows split over RS duplicated
// workgroups) every CU gathers half as many LDS words and loads a third less
// table data, and no workgroup repeats another's section work.  The top-bit
// FWHT stage and the section max / sums cross the two waves through LDS.
// Ab partials: G2 = ceil(L/2) per codeword, each over all n rows.
// FWHT stage on the top index bit, held by the two waves of a section:
// (a, b) -> (a + b, a - b) through an LDS exchange (wave w = top bit).
template <typename real, int E2>
__device__ __forceinline__ void top_bit_stage(real (&v)[E2], real* mine, const real* other, int lane, int w) {
#pragma unroll
  for (int i = 0; i < E2; ++i) mine[i * 64 + lane] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < E2; ++i) {
    const real p = other[i * 64 + lane];
    v[i] = w ? p - v[i] : v[i] + p;
  }
  __syncthreads();
}

template <typename real, int E2>
__global__ void __launch_bounds__(256) k_sec2(SecArgs<real> a) {
  STAMP(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int KH = E2 >= 16 ? 2 : 16;
  constexpr int NQ = (E2 + 3) / 4;
  // every row's Ab-table entry is loaded at kernel start (KR per thread covers
  // n <= 256 * KR in one pass; larger n loops over further passes)
  constexpr int KR = 18;
  const int g = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int sidx = wv >> 1, w = wv & 1;
  const int M = a.M, n = a.n, Mh = M >> 1;
  const size_t LM = (size_t)a.L * M;
  const int l = g * 2 + sidx;
  const bool have = l < a.L;
  const int lc = have ? l : a.L - 1;
  const int eoff = w * Mh;

  real* zs = reinterpret_cast<real*>(smem);
  const int zslots = ((n + 1) * (int)sizeof(real) + 15) / 16 * 16 / (int)sizeof(real);
  real* ts = zs + zslots;        // [2][M]   T_l = H_M beta_l
  real* xb = ts + 2 * M;         // [4][E2*64] top-bit exchange
  real* red = xb + 4 * E2 * 64;  // [4][4]   per-wave max, S, S2, beta^2

  real v[E2];
  real bprev[E2];
  const real* bl = a.beta + (size_t)b * LM + (size_t)lc * M + eoff;
  real* blo = a.beta_out + (size_t)b * LM + (size_t)lc * M + eoff;
  const uint16_t* il = a.inv + (size_t)lc * a.w + eoff;
  // (k | sign << 15) of this pair's two sections for row r (pair-major table:
  // the workgroup reads only its own lines)
  const uint32_t* fw = a.fwd2 + (size_t)g * n;
  ushort4 tb[KH][NQ];
  uint32_t f[KR];

  // loads in the order they are needed (vmcnt retires them in order)
  const real* zzb = a.zzp + (size_t)b * a.NZ;
  ZZParts<real> zz;
  zz.issue(zzb, a.NZ, lane);
  const real last = a.t > 0 ? ld_vmem(a.tau + (size_t)b * a.T1 + a.t - 1) : (real)0;
  const real* zb = a.z + (size_t)b * n;
  ZStage<real> zst;
  const bool dma = stage_z_dma<real, 256>(zb, zs, n, tid);
  if (!dma) zst.issue(zb, n, tid);
  load_buckets<E2, KH>(il, 0, a.nhi, M, lane, tb);
  load_section<real, E2>(bl, bprev, lane, Mh);
  const real cl = ld_vmem(a.c + (size_t)b * a.cst + lc);
  const int nk = min(KR, (n + 255) / 256);  // passes of 256 rows in the first chunk
#pragma unroll
  for (int u = 0; u < KR; ++u) {
    const int r = u * 256 + tid;
    if (u < nk) f[u] = fw[r < n ? r : 0];
  }
  const real tau = zz.tau(zzb, a.NZ, n);
  const bool stop = a.early_stop && (tau == last);
  if (g == 0 && tid == 0) {
    a.tau[(size_t)b * a.T1 + a.t] = tau;
    if (stop && a.iters[b] < 0) a.iters[b] = a.t;
  }
  if (stop) {  // uniform over the grid row
    if (dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write may outlive the workgroup
    return;
  }
  const real tau2 = tau * tau;
  STAMP(1);
  if (!dma) zst.store(zs, zb, n, tid);
  else finish_z_dma(zb, zs, n, tid);
  __syncthreads();
  STAMP(2);

  // bucket gather of z for this wave's half of the section
#pragma unroll
  for (int i = 0; i < E2; ++i) v[i] = 0;
  for (int h0 = 0; h0 < a.nhi; h0 += KH) {
    ushort4 tn[KH][NQ];
    const bool more = h0 + KH < a.nhi;
    if (more) load_buckets<E2, KH>(il, h0 + KH, a.nhi, M, lane, tn);
    gather_buckets<real, E2, KH>(zs, h0, a.nhi, tb, v);
    if (more) {
#pragma unroll
      for (int hh = 0; hh < KH; ++hh)
#pragma unroll
        for (int j = 0; j < NQ; ++j) tb[hh][j] = tn[hh][j];
    }
  }
  real* mine = xb + wv * (E2 * 64);
  const real* other = xb + (wv ^ 1) * (E2 * 64);
  STAMP(3);
  fwht_wave<real, E2>(v, lane, 64);
  top_bit_stage<real, E2>(v, mine, other, lane, w);
  STAMP(4);

  // denoiser (sparc_ldpc.py:213-219) over both halves of the section
  const real inv_sn = (real)1 / a.sqrt_n;
  const real kk = cl / tau2;
  real mx = neg_inf<real>();
#pragma unroll
  for (int i = 0; i < E2; ++i) {
    v[i] = fma(v[i], inv_sn, bprev[i]) * kk;
    mx = v[i] > mx ? v[i] : mx;
  }
  mx = wave_max(mx);
  if (lane == 0) red[wv * 4] = mx;
  __syncthreads();
  const int w0 = wv & ~1;
  mx = red[w0 * 4] > red[(w0 + 1) * 4] ? red[w0 * 4] : red[(w0 + 1) * 4];
  real S = 0, S2 = 0;
#pragma unroll
  for (int i = 0; i < E2; ++i) {
    v[i] = dexp<real>(v[i] - mx);
    S += v[i];
    S2 += v[i] * v[i];
  }
  wave_sum2(S, S2);
  if (lane == 0) {
    red[wv * 4 + 1] = S;
    red[wv * 4 + 2] = S2;
  }
  __syncthreads();
  S = red[w0 * 4 + 1] + red[(w0 + 1) * 4 + 1];
  S2 = red[w0 * 4 + 2] + red[(w0 + 1) * 4 + 2];
  const real scale = cl / S;
#pragma unroll
  for (int i = 0; i < E2; ++i) v[i] = have ? v[i] * scale : (real)0;
  if (have) store_section<real, E2>(blo, v, lane, Mh);
  const real bb = have ? S2 * scale * scale : (real)0;

  STAMP(5);
  fwht_wave<real, E2>(v, lane, 64);  // T_l = H_M beta_l
  top_bit_stage<real, E2>(v, mine, other, lane, w);
  STAMP(6);
  {
    real* tl = ts + sidx * M + eoff;
#pragma unroll
    for (int i = 0; i < E2; ++i) tl[elem_index<E2>(lane, i)] = v[i];
  }
  if (lane == 0) red[wv * 4 + 3] = bb;
  __syncthreads();
  STAMP(7);
  if (tid == 0) a.bbp[(size_t)b * a.G + g] = red[0 * 4 + 3] + red[2 * 4 + 3];
  // Ab partial of the pair for every row
  real* abp = a.abp + ((size_t)b * a.G + g) * n;
  for (int r0 = 0; r0 < n; r0 += 256 * KR) {
    if (r0 > 0) {  // n > 256 * KR only
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int r = r0 + u * 256 + tid;
        f[u] = fw[r < n ? r : 0];
      }
    }
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      const int r = r0 + u * 256 + tid;
      if (r < n) {
        const uint32_t e = f[u];
        const real v0 = ts[e & 0x7fffu];
        const real v1 = ts[M + ((e >> 16) & 0x7fffu)];
        real t = (e & 0x8000u) ? -v0 : v0;
        t += (e & 0x80000000u) ? -v1 : v1;
        st_part(&abp[r], t);
      }
    }
  }
#ifdef SA_STAMPS
  STAMP(8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(9);
#endif
}
// QW wavefronts per section (k_sec4: QW = 4): the k_sec2
// workgroup of two sections with 2*QW waves.  Wave q of a section holds the
// q-th 1/QW of it (the log2(QW) top index bits); those top FWHT stages cross
// the waves in one LDS exchange, applied lowest bit first like the
// single-bit stages ((x0 +- x1) +- (x2 +- x3)) ..., so the transform is
// bit-identical to k_sec2's.  Per wave the LDS gather chain and the Ab row
// loop shrink with QW, and every SIMD runs QW / 2 waves.  (QW = 8, 1024-thread
// workgroups, measured slower at c2: 8.1 vs 7.6 us per launch.)
template <typename real, int EQ, int QW>
__device__ __forceinline__ void topq_stage(real (&v)[EQ], real* xs, int lane, int q) {
  constexpr int QS = EQ * 64;  // one wave's share of the section
#pragma unroll
  for (int i = 0; i < EQ; ++i) xs[q * QS + i * 64 + lane] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < EQ; ++i) {
    real x[QW];
#pragma unroll
    for (int j = 0; j < QW; ++j) x[j] = xs[j * QS + i * 64 + lane];
#pragma unroll
    for (int k = 0, span = 1; span < QW; ++k, span <<= 1)
#pragma unroll
      for (int j = 0; j < QW; j += 2 * span) x[j] = ((q >> k) & 1) ? x[j] - x[j + span] : x[j] + x[j + span];
    v[i] = x[0];
  }
  __syncthreads();
}

// Fixed-order combination of the QW per-wave values red[(w0 + j) * 4 + f]
// of one section: max, or a pairwise tree sum ((r0 + r1) + (r2 + r3)) ...
template <typename real, int QW, bool MAX>
__device__ __forceinline__ real combine_q(const real* red, int w0, int f) {
  real x[QW];
#pragma unroll
  for (int j = 0; j < QW; ++j) x[j] = red[(w0 + j) * 4 + f];
#pragma unroll
  for (int span = 1; span < QW; span <<= 1)
#pragma unroll
    for (int j = 0; j < QW; j += 2 * span) {
      if constexpr (MAX) x[j] = x[j] > x[j + span] ? x[j] : x[j + span];
      else x[j] = x[j] + x[j + span];
    }
  return x[0];
}

// The pair / triple section kernels' body (SPW sections x QW waves).
template <typename real, int EQ, int QW, int SPW = 2>
__device__ __forceinline__ void secq_body(const SecArgs<real>& a) {
  static_assert(SPW == 2 || SPW == 3, "sections per workgroup");
  STAMP(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NT = SPW * QW * 64;
  // bucket h-steps whose table loads are in flight together: triples take 8
  // (C4, 32 h-steps: half the first round trip's table bytes, the rest lands
  // during the gather; 961 -> 996 cw/s), pairs 16 (c2: all 16 up front; 8 neutral)
  constexpr int KH = EQ >= 8 ? 4 : (SPW == 3 ? 8 : 16);
  constexpr int NQ = (EQ + 3) / 4;
  // rows per thread per pass, all Ab-table loads issued with the first loads: n <= 4608 (pairs,
  // C2) / 8448 (triples, C4 n = 8294) in one pass (a second pass reloads the table mid-phase:
  // one more memory round trip)
  constexpr int KR = ((SPW == 3 ? 8448 : 4608) + NT - 1) / NT;
  const int g = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int sidx = wv / QW, q = wv % QW;
  const int M = a.M, n = a.n, Mq = M / QW;
  const size_t LM = (size_t)a.L * M;
  const int l = g * SPW + sidx;
  const bool have = l < a.L;
  const int lc = have ? l : a.L - 1;
  const int eoff = q * Mq;

  real* zs = reinterpret_cast<real*>(smem);
  const int zslots = ((n + 1) * (int)sizeof(real) + 15) / 16 * 16 / (int)sizeof(real);
  real* ts = zs + zslots;          // [SPW][M]   T_l = H_M beta_l
  real* xb = ts + SPW * M;         // [SPW][M]   top-stage exchange, one M per section
  real* red = xb + SPW * M;        // [SPW*QW][4] per-wave max, S, S2, beta^2

  real v[EQ];
  real bprev[EQ];
  const real* bl = a.beta + (size_t)b * LM + (size_t)lc * M + eoff;
  real* blo = a.beta_out + (size_t)b * LM + (size_t)lc * M + eoff;
  // the HBM bucket tables as a workgroup-uniform base + this wave's 32-bit offset
  const uint16_t* ibase = a.inv + (size_t)g * SPW * a.w;
  const unsigned ioff = (unsigned)((lc - g * SPW) * a.w + eoff);
  const uint32_t* fw = (SPW == 2 ? a.fwd2 : a.fwd3) + (size_t)g * n;
  ushort4 tb[KH][NQ];
  uint32_t f[KR];  // Ab-table entries of this thread's rows

  // Load order: z's LDS-DMA first, then the z^2 partials and tau_{t-1}, then
  // the tables, all unconditional (straight-line).  While an LDS-DMA is in
  // flight the compiler waits for any loaded register with vmcnt(0) (checked
  // on a minimal kernel), so tau waits for every load whatever the order; the
  // earliest possible DMA (z is the last thing the gather needs) and no
  // branches around loads measured c2 1316 -> 1372 cw/s (k_sec4 7.45 ->
  // 6.68 us); register-staged z with exact waits instead: 1337
  const real* zb = a.z + (size_t)b * n;
  ZStage<real, NT> zst;
  const real* zzb = a.zzp + (size_t)b * a.NZ;
  // z^2 partials held in registers: k_row2 writes ceil(n / 32) (C4 n = 8294:
  // 260, past the 256 of K = 4, whose fallback re-reads them: one more memory
  // round trip before tau), k_row2<16> ceil(n / 16) (C2: 288)
  ZZParts<real, 5> zz;
  const bool dma = stage_z_dma<real, NT>(zb, zs, n, tid);
  if (!dma) zst.issue(zb, n, tid);
  zz.issue(zzb, a.NZ, lane);
  const real last = a.t > 0 ? ld_vmem(a.tau + (size_t)b * a.T1 + a.t - 1) : (real)0;
  load_buckets_off<EQ, KH>(ibase, ioff, 0, a.nhi, M, lane, tb);  // bucket stride M; lane elements < Mq
  load_section<real, EQ>(bl, bprev, lane, Mq);
  const real cl = ld_vmem(a.c + (size_t)b * a.cst + lc);
  const real tau = zz.tau(zzb, a.NZ, n);
  const bool stop = a.early_stop && (tau == last);
  if (g == 0 && tid == 0) {
    a.tau[(size_t)b * a.T1 + a.t] = tau;
    if (stop && a.iters[b] < 0) a.iters[b] = a.t;
  }
  if (stop) {  // uniform over the grid row
    if (dma) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write may outlive the workgroup
    return;
  }
  const real tau2 = tau * tau;
  // the denoiser's scalars now, off its dependency chain (computed while the
  // z staging and the bucket gather run)
  const real inv_sn = (real)1 / a.sqrt_n;
  const real kk = cl / tau2;
  STAMP(1);
  if (!dma) zst.store(zs, zb, n, tid);
  else finish_z_dma<real>(zb, zs, n, tid);
  __syncthreads();
  STAMP(2);
#ifdef SA_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic: table loads landed
  STAMP(10);
#endif
#pragma unroll
  for (int i = 0; i < EQ; ++i) v[i] = 0;
  for (int h0 = 0; h0 < a.nhi; h0 += KH) {
    ushort4 tn[KH][NQ];
    const bool more = h0 + KH < a.nhi;
    if (more) load_buckets_off<EQ, KH>(ibase, ioff, h0 + KH, a.nhi, M, lane, tn);
    gather_buckets<real, EQ, KH>(zs, h0, a.nhi, tb, v);
    if (more) {
#pragma unroll
      for (int hh = 0; hh < KH; ++hh)
#pragma unroll
        for (int j = 0; j < NQ; ++j) tb[hh][j] = tn[hh][j];
    }
  }
  real* xs = xb + sidx * M;
  // the Ab-table rows (not needed before the row phase) issued only now: they
  // land under the transforms and the denoiser, where no other load is in
  // flight, instead of adding their bytes (C2 18 KB, C4 33 KB per workgroup)
  // to the first memory round trip, which every wave waits for (C4 single
  // codeword 860 -> 894 cw/s, c2 1378 -> 1394; `k_sec43` 11.0 -> 10.7 us)
#pragma unroll
  for (int u = 0; u < KR; ++u) {  // unconditional (clamped): see load_section
    const int r = u * NT + tid;
    f[u] = ld_off(fw, (unsigned)(r < n ? r : 0) * 4u);  // uniform base + 32-bit offset
  }
  STAMP(3);
  fwht_wave<real, EQ>(v, lane, 64);
  topq_stage<real, EQ, QW>(v, xs, lane, q);
  STAMP(4);

  // denoiser (sparc_ldpc.py:213-219) over the four quarters of the section
  // (inv_sn, kk: computed after tau)

  real mx = neg_inf<real>();
#pragma unroll
  for (int i = 0; i < EQ; ++i) {
    v[i] = fma(v[i], inv_sn, bprev[i]) * kk;
    mx = v[i] > mx ? v[i] : mx;
  }
  mx = wave_max(mx);
  if (lane == 0) red[wv * 4] = mx;
  __syncthreads();
  const int w0 = wv & ~(QW - 1);
  mx = combine_q<real, QW, true>(red, w0, 0);
  real S = 0, S2 = 0;
#pragma unroll
  for (int i = 0; i < EQ; ++i) {
    v[i] = dexp<real>(v[i] - mx);
    S += v[i];
    S2 += v[i] * v[i];
  }
  wave_sum2(S, S2);
  if (lane == 0) {
    red[wv * 4 + 1] = S;
    red[wv * 4 + 2] = S2;
  }
  __syncthreads();
  S = combine_q<real, QW, false>(red, w0, 1);
  S2 = combine_q<real, QW, false>(red, w0, 2);
  const real scale = cl * rcp_fast(S);  // one v_rcp (1 ulp) instead of a division chain on the critical path
#pragma unroll
  for (int i = 0; i < EQ; ++i) v[i] = have ? v[i] * scale : (real)0;
  if (have) store_section<real, EQ>(blo, v, lane, Mq);
  const real bb = have ? S2 * scale * scale : (real)0;

  STAMP(5);
  fwht_wave<real, EQ>(v, lane, 64);  // T_l = H_M beta_l
  topq_stage<real, EQ, QW>(v, xs, lane, q);
  STAMP(6);
  {
    real* tl = ts + sidx * M + eoff;
#pragma unroll
    for (int i = 0; i < EQ; ++i) tl[elem_index<EQ>(lane, i)] = v[i];
  }
  if (lane == 0) red[wv * 4 + 3] = bb;
  __syncthreads();
  STAMP(7);
  if (tid == 0) {
    real bsum = red[0 * 4 + 3] + red[QW * 4 + 3];
    if constexpr (SPW == 3) bsum += red[2 * QW * 4 + 3];
    a.bbp[(size_t)b * a.G + g] = bsum;
  }
  // Ab partial of the pair (triple) for every row
  real* abp = a.abp + ((size_t)b * a.G + g) * n;
  const int psh = a.pt == 16 ? 4 : 5;  // pt: rows per block 16 / 32
  const size_t npad = (size_t)((n + (1 << psh) - 1) >> psh) << psh;
  real* abq = a.abp + (size_t)b * a.G * npad + ((size_t)g << psh);  // pt: + (r >> psh) * G * R + (r & (R - 1))
  real* const sbase = a.pt ? abq : abp;
  const int sh = a.pt ? psh : 31;
  const size_t gstride = (size_t)a.G << sh;
  const int smask = (int)((1u << sh) - 1u);
  static_assert(NT % 32 == 0, "a pass of rows is a whole number of row blocks");
  const size_t ustep = sh < 31 ? (size_t)(NT >> sh) * gstride : (size_t)NT;
  for (int r0 = 0; r0 < n; r0 += NT * KR) {
    if (r0 > 0) {  // n > NT * KR only
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int r = r0 + u * NT + tid;
        f[u] = fw[r < n ? r : 0];
      }
    }
    real* const pbase = sbase + (size_t)((r0 + tid) >> sh) * gstride + ((r0 + tid) & smask);
    // row r's term of the pair (triple) and its store
    auto row = [&](int u, int r) {
      real t;
      if constexpr (SPW == 2) {
        const uint32_t e = f[u];
        const real v0 = ts[e & 0x7fffu];
        const real v1 = ts[M + ((e >> 16) & 0x7fffu)];
        t = (e & 0x8000u) ? -v0 : v0;
        t += (e & 0x80000000u) ? -v1 : v1;
      } else {
        const uint32_t e = f[u];
        const real v0 = ts[e & 0x1ffu];
        const real v1 = ts[M + ((e >> 10) & 0x1ffu)];
        const real v2 = ts[2 * M + ((e >> 20) & 0x1ffu)];
        t = (e & 0x200u) ? -v0 : v0;
        t += (e & 0x80000u) ? -v1 : v1;
        t += (e & 0x20000000u) ? -v2 : v2;
      }
      // one branch-free store for both layouts ([G][n] is the row-block form
      // with sh = 31); triples: row r0 + tid + u NT at pbase + u ustep (NT is
      // a whole number of 16- / 32-row blocks; pairs measured faster with the
      // address from r)
      if constexpr (SPW == 3) st_part(pbase + u * ustep, t);
      else st_part(&sbase[(size_t)(r >> sh) * gstride + (r & smask)], t);
    };
    if (r0 + NT * KR <= n) {
      // uniform: every row of the pass exists; no per-row branch, so the
      // LDS reads of several rows are in flight together (c2: n = 9 x 512)
#pragma unroll
      for (int u = 0; u < KR; ++u) row(u, r0 + u * NT + tid);
    } else {
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int r = r0 + u * NT + tid;
        if (r < n) row(u, r);
      }
    }
  }
#ifdef SA_STAMPS
  STAMP(8);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(9);
#endif
}

template <typename real, int E4>
__global__ void __launch_bounds__(512) k_sec4(SecArgs<real> a) { secq_body<real, E4, 4, 2>(a); }
// Three sections per workgroup (12 waves): L = 3 x CUs (L = 768 on 256 CUs)
// puts one workgroup on every CU where pairs leave half the CUs with two.
template <typename real, int E4>
__global__ void __launch_bounds__(768) k_sec43(SecArgs<real> a) { secq_body<real, E4, 4, 3>(a); }

// ---- launchers ------------------------------------------------------------
template <typename real, int E>
void launch_sec_e(sa_ctx* c, int B, SecArgs<real> a) {
  a.RS = row_splits(c, B);
  dim3 grid(c->G * a.RS, B);
  if (c->prof) c->prof->begin(c->stream, K_SEC);
  if (c->big)
    plaunch(c, k_secg<real, E>, grid, 256, c->sec_lds, a);
  else
    plaunch(c, k_sec<real, E>, grid, 256, c->sec_lds, a);
  if (c->prof) c->prof->end(c->stream);
}

template <typename real>
int launch_sec2(sa_ctx* c, int B, int t, int es, void* bin, void* bout, int pt) {
  SecArgs<real> a = sec_args<real>(c, SEC_AMP, t, es);
  a.pt = pt;
  a.beta = (real*)bin;
  a.beta_out = (real*)bout;
  a.G = sec2_parts(c);
  dim3 grid(a.G, B);
  if (c->prof) c->prof->begin(c->stream, K_SEC);
  if (c->sec3) {
    switch (c->M / 256) {
      case 1: plaunch(c, k_sec43<real, 1>, grid, 768, c->sec3_lds, a); break;
      case 2: plaunch(c, k_sec43<real, 2>, grid, 768, c->sec3_lds, a); break;
      default: return fail(SA_ERR_UNSUPPORTED, "k_sec43: M");
    }
    if (c->prof) c->prof->end(c->stream);
    HIP_TRY(hipGetLastError());
    return SA_OK;
  }
  if (c->sec4) {
    switch (c->M / 256) {
      case 1: plaunch(c, k_sec4<real, 1>, grid, 512, c->sec4_lds, a); break;
      case 2: plaunch(c, k_sec4<real, 2>, grid, 512, c->sec4_lds, a); break;
      case 4: plaunch(c, k_sec4<real, 4>, grid, 512, c->sec4_lds, a); break;
      case 8: plaunch(c, k_sec4<real, 8>, grid, 512, c->sec4_lds, a); break;
      case 16: plaunch(c, k_sec4<real, 16>, grid, 512, c->sec4_lds, a); break;
      default: return fail(SA_ERR_UNSUPPORTED, "k_sec4: M");
    }
    if (c->prof) c->prof->end(c->stream);
    HIP_TRY(hipGetLastError());
    return SA_OK;
  }
  switch (c->M / 128) {
    case 1: plaunch(c, k_sec2<real, 1>, grid, 256, c->sec2_lds, a); break;
    case 2: plaunch(c, k_sec2<real, 2>, grid, 256, c->sec2_lds, a); break;
    case 4: plaunch(c, k_sec2<real, 4>, grid, 256, c->sec2_lds, a); break;
    case 8: plaunch(c, k_sec2<real, 8>, grid, 256, c->sec2_lds, a); break;
    case 16: plaunch(c, k_sec2<real, 16>, grid, 256, c->sec2_lds, a); break;
    case 32: plaunch(c, k_sec2<real, 32>, grid, 256, c->sec2_lds, a); break;
    default: return fail(SA_ERR_UNSUPPORTED, "k_sec2: M");
  }
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

template <typename real>
int launch_sec(sa_ctx* c, int B, int mode, int t, int es, void* bin, void* bout) {
  SecArgs<real> a = sec_args<real>(c, mode, t, es);
  if (bin) a.beta = (real*)bin;
  if (bout) a.beta_out = (real*)bout;
  switch (c->E) {
    case 1: launch_sec_e<real, 1>(c, B, a); break;
    case 2: launch_sec_e<real, 2>(c, B, a); break;
    case 4: launch_sec_e<real, 4>(c, B, a); break;
    case 8: launch_sec_e<real, 8>(c, B, a); break;
    case 16: launch_sec_e<real, 16>(c, B, a); break;
    case 32: launch_sec_e<real, 32>(c, B, a); break;
    case 64: launch_sec_e<real, 64>(c, B, a); break;
    default: return fail(SA_ERR_UNSUPPORTED, "bad E");
  }
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

template int launch_sec<float>(sa_ctx*, int, int, int, int, void*, void*);
template int launch_sec<double>(sa_ctx*, int, int, int, int, void*, void*);
template int launch_sec2<float>(sa_ctx*, int, int, int, void*, void*, int);
template int launch_sec2<double>(sa_ctx*, int, int, int, void*, void*, int);

// Every single-codeword section-kernel instantiation may use the full 160 KB LDS.
template <typename real>
static hipError_t sec_lds_attrs_t() {
  const int mx = 160 * 1024;
  hipError_t e = hipSuccess;
#define SA_A(F) if (e == hipSuccess) e = hipFuncSetAttribute((const void*)F, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
  SA_A((k_sec<real, 1>)) SA_A((k_sec<real, 2>)) SA_A((k_sec<real, 4>)) SA_A((k_sec<real, 8>))
  SA_A((k_sec<real, 16>)) SA_A((k_sec<real, 32>)) SA_A((k_sec<real, 64>))
  SA_A((k_secg<real, 1>)) SA_A((k_secg<real, 2>)) SA_A((k_secg<real, 4>)) SA_A((k_secg<real, 8>))
  SA_A((k_secg<real, 16>)) SA_A((k_secg<real, 32>)) SA_A((k_secg<real, 64>))
  SA_A((k_sec2<real, 1>)) SA_A((k_sec2<real, 2>)) SA_A((k_sec2<real, 4>)) SA_A((k_sec2<real, 8>))
  SA_A((k_sec2<real, 16>)) SA_A((k_sec2<real, 32>))
  SA_A((k_sec4<real, 1>)) SA_A((k_sec4<real, 2>)) SA_A((k_sec4<real, 4>)) SA_A((k_sec4<real, 8>))
  SA_A((k_sec4<real, 16>))
  SA_A((k_sec43<real, 1>)) SA_A((k_sec43<real, 2>))
#undef SA_A
  return e;
}

hipError_t sec_lds_attrs() {
  hipError_t e = sec_lds_attrs_t<float>();
  return e == hipSuccess ? sec_lds_attrs_t<double>() : e;
}

#ifdef SA_STAMPS
hipError_t stamps_add_sec(unsigned long long* out) {
  unsigned long long s[16 * 16];
  hipError_t e = hipMemcpyFromSymbol(s, HIP_SYMBOL(g_stamps), sizeof(s));
  for (int i = 0; i < 16 * 16; ++i) out[i] += s[i];
  return e;
}
#endif

}  // namespace sa
