// sa_row.hip — the row kernels (Ab partial sums + Onsager residual + z^2
// partials: k_row, k_rowv, k_rowc, k_row2), the section decision k_decide
// and their launchers.
#include "sa_host.h"

namespace sa {

// Residual update with the Onsager term (sparc_ldpc.py:220):
//   z = y - Ab(beta) + (z / tau^2) * (P - sum(beta^2) / n)
// and the per-block partial sums of z^2 for the next tau.  64 rows per
// workgroup (lane = row); the 16 waves split the G Ab partials (all of a
// wave's loads in flight together), combined in wave order through LDS.
template <typename real, int kRowWaves>
__global__ void __launch_bounds__(kRowWaves * 64) k_row(RowArgs<real> a) {
  __shared__ real red[kRowWaves][kRowsPerBlk];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = blockIdx.x * kRowsPerBlk + lane;
  const int n = a.n;
  // tau_t and tau_{t-1} are loaded with everything else; the early-stop
  // test waits for them only after the Ab-partial loads are in flight
  // (testing first cost a whole memory round trip per launch)
  real tau = 1, last = 0;
  if (a.mode == ROW_AMP) {
    tau = ld_vmem(a.tau + (size_t)b * a.T1 + a.t);
    last = a.t > 0 ? ld_vmem(a.tau + (size_t)b * a.T1 + a.t - 1) : (real)0;
  }
  // wave 0 finishes the rows: its operands that do not depend on the Ab
  // partials (y, z, the beta^2 partials) are loaded up front, in the same
  // round trip as the partials
  const size_t o = (size_t)b * n + (r < n ? r : 0);
  real yv = 0, zv = 0, bbv[2] = {0, 0};
  if (wv == 0) {
    yv = a.y[o];
    if (a.mode == ROW_AMP) {
      zv = a.z[o];
      const real* bp = a.bbp + (size_t)b * a.Gb;
      bbv[0] = lane < a.Gb ? bp[lane] : (real)0;
      bbv[1] = lane + 64 < a.Gb ? bp[lane + 64] : (real)0;
    }
  }
  if (a.mode != ROW_INIT0) {
    const int gq = (a.G + kRowWaves - 1) / kRowWaves;
    const int g0 = wv * gq, g1 = min(a.G, g0 + gq);
    const real* p = a.abp + (size_t)b * a.G * n + (r < n ? r : 0);
    real acc = 0;
    constexpr int U = 16;
    for (int gg = g0; gg < g1; gg += U) {
      real t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = p[(size_t)(gg + u < g1 ? gg + u : g0) * n];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (gg + u < g1) acc += t[u];
    }
    red[wv][lane] = acc;
  }
  if (a.mode == ROW_AMP && a.early_stop && tau == last) return;  // uniform over the workgroup
  const real tau2 = tau * tau;
  __syncthreads();
  if (wv != 0) return;
  real ons = 0;
  if (a.mode == ROW_AMP) {
    const real bb = a.Gb <= 128 ? wave_sum_pair(bbv[0], bbv[1]) : wave_sum_parts(a.bbp + (size_t)b * a.Gb, a.Gb);
    ons = a.Pb[(size_t)b * a.Pbst] - bb / (real)n;
  }
  real zn = 0;
  if (r < n) {
    if (a.mode == ROW_INIT0) {
      zn = yv;
    } else {
      real acc = 0;
      for (int w = 0; w < kRowWaves; ++w) acc += red[w][lane];
      const real ab = acc / a.sqrt_n;
      if (a.mode == ROW_ABOUT) {
        a.out[o] = ab;
        return;
      }
      zn = yv - ab;
      if (a.mode == ROW_AMP) zn += (zv / tau2) * ons;
    }
    a.z[o] = zn;
  }
  if (a.mode == ROW_ABOUT) return;
  const real s = wave_sum(zn * zn);
  if (lane == 0) a.zzp[(size_t)b * a.NZ + blockIdx.x] = s;
}

// k_row with V-element accesses (n % V == 0, many codewords; binary32 V = 4:
// 16 bytes, 256 rows per workgroup, or V = 2: 8 bytes, 128 rows; binary64
// V = 2: 16 bytes, 128 rows): V rows per lane, so each load instruction of
// the partial stream moves 64 V elements per wave (k_row: 64).  Per row the same sums as k_row in the same order (wave w
// adds its partial range in order, the four wave sums are added in wave
// order); the z^2 partials cover 64 V rows.
template <typename real, int V>
__global__ void __launch_bounds__(256) k_rowv(RowArgs<real> a) {
  using fv = real __attribute__((ext_vector_type(V)));
  __shared__ fv red[4][64];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = a.n;
  const int r = blockIdx.x * 64 * V + lane * V;  // the lane's first row
  const bool in = r < n;                          // n % V == 0: V rows or none
  real tau = 1, last = 0;
  if (a.mode == ROW_AMP) {
    tau = ld_vmem(a.tau + (size_t)b * a.T1 + a.t);
    last = a.t > 0 ? ld_vmem(a.tau + (size_t)b * a.T1 + a.t - 1) : (real)0;
  }
  const size_t o = (size_t)b * n + (in ? r : 0);
  fv yv = {}, zv = {};
  real bbv[2] = {0, 0};
  if (wv == 0) {
    yv = *reinterpret_cast<const fv*>(a.y + o);
    if (a.mode == ROW_AMP) {
      zv = *reinterpret_cast<const fv*>(a.z + o);
      const real* bp = a.bbp + (size_t)b * a.Gb;
      bbv[0] = lane < a.Gb ? bp[lane] : (real)0;
      bbv[1] = lane + 64 < a.Gb ? bp[lane + 64] : (real)0;
    }
  }
  if (a.mode != ROW_INIT0) {
    const int gq = (a.G + 3) / 4;
    const int g0 = wv * gq, g1 = min(a.G, g0 + gq);
    const real* p = a.abp + (size_t)b * a.G * n + (in ? r : 0);
    fv acc = {};
    constexpr int U = 8;
    for (int gg = g0; gg < g1; gg += U) {
      fv t[U];
#pragma unroll
      for (int u = 0; u < U; ++u)  // the partials are dead after this read: streaming loads
        t[u] = __builtin_nontemporal_load(reinterpret_cast<const fv*>(p + (size_t)(gg + u < g1 ? gg + u : g0) * n));
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (gg + u < g1) acc += t[u];
    }
    red[wv][lane] = acc;
  }
  if (a.mode == ROW_AMP && a.early_stop && tau == last) return;  // uniform over the workgroup
  const real tau2 = tau * tau;
  __syncthreads();
  if (wv != 0) return;
  real ons = 0;
  if (a.mode == ROW_AMP) {
    const real bb = a.Gb <= 128 ? wave_sum_pair(bbv[0], bbv[1]) : wave_sum_parts(a.bbp + (size_t)b * a.Gb, a.Gb);
    ons = a.Pb[(size_t)b * a.Pbst] - bb / (real)n;
  }
  fv zn = {};
  if (in) {
    if (a.mode == ROW_INIT0) {
      zn = yv;
    } else {
      fv sv = {};
#pragma unroll
      for (int w = 0; w < 4; ++w) sv += red[w][lane];
      const fv ab = sv / a.sqrt_n;
      if (a.mode == ROW_ABOUT) {
        *reinterpret_cast<fv*>(a.out + o) = ab;
        return;
      }
      zn = yv - ab;
      if (a.mode == ROW_AMP) zn += (zv / tau2) * ons;
    }
    *reinterpret_cast<fv*>(a.z + o) = zn;
  }
  if (a.mode == ROW_ABOUT) return;
  real q = 0;
#pragma unroll
  for (int j = 0; j < V; ++j) q += zn[j] * zn[j];
  const real s = wave_sum(q);
  if (lane == 0) a.zzp[(size_t)b * a.NZ + blockIdx.x] = s;
}

// Row kernel of the codeword-interleaved batched layout (SecArgs::zil): rows
// of a chunk of CB codewords (CB x sizeof(real) = 16 bytes: binary32 CB = 4,
// binary64 CB = 2), 128 rows per 256-thread workgroup (lane l: rows l and
// l + 64), blockIdx.y the chunk.  The four waves split the G Ab partials of
// those rows (wave w adds its range in order, all its loads in flight
// together; the four wave sums added in wave order, as k_rowv); the partials
// are 16-byte vectors [NC][G][n][CB] (pil, behind k_secb) or per codeword
// [B][G][n] (behind k_sec's SEC_AB, the beta0 start).  Wave 0 then forms the
// Onsager residual (sparc_ldpc.py:220), stores z [NC][n][CB] as one 16-byte
// vector per row, and the z^2 partial of each codeword's block.  A stopped
// codeword keeps its z and z^2 partials.
template <typename real, int CB, int U = 8>
__global__ void __launch_bounds__(256) k_rowc(RowArgs<real> a, int pil) {
  using V = real __attribute__((ext_vector_type(CB)));
  constexpr int RPL = 2;  // rows per lane
  __shared__ V red[4][RPL][64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int chunk = blockIdx.y, n = a.n;
  int rr[RPL], ro[RPL];
  bool in[RPL];
#pragma unroll
  for (int k = 0; k < RPL; ++k) {
    rr[k] = blockIdx.x * 64 * RPL + k * 64 + lane;
    in[k] = rr[k] < n;
    ro[k] = in[k] ? rr[k] : 0;
  }
  const int B = a.Bc;
  int bc[CB], tcur[CB];
  bool valid[CB];
  bool anyv = false;
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int b = chunk * CB + c;
    valid[c] = b < B;
    bc[c] = valid[c] ? b : B - 1;
    tcur[c] = a.t;
    if (a.tb) {  // Monte-Carlo stream: the slot's own iteration, -1 for an empty slot
      tcur[c] = ld_smem(a.tb + bc[c]);
      valid[c] = valid[c] && tcur[c] >= 0;
    }
    anyv |= valid[c];
  }
  if (!anyv) return;  // uniform: a chunk of empty slots (Monte-Carlo stream tail)
  // wave 0's operands that do not depend on the partials, loaded with them
  real tau[CB], last[CB], yv[RPL][CB], bbv[CB][2];
  V zo[RPL] = {};
  if (wv == 0) {
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      tau[c] = 1;
      last[c] = 0;
      if (a.mode == ROW_AMP) {
        tau[c] = ld_vmem(a.tau + (size_t)bc[c] * a.T1 + tcur[c]);
        last[c] = tcur[c] > 0 ? ld_vmem(a.tau + (size_t)bc[c] * a.T1 + tcur[c] - 1) : (real)0;
        const real* bp = a.bbp + (size_t)bc[c] * a.Gb;
        bbv[c][0] = lane < a.Gb ? bp[lane] : (real)0;
        bbv[c][1] = lane + 64 < a.Gb ? bp[lane + 64] : (real)0;
      }
#pragma unroll
      for (int k = 0; k < RPL; ++k) yv[k][c] = a.y[(size_t)bc[c] * n + ro[k]];
    }
    if (a.mode == ROW_AMP)
#pragma unroll
      for (int k = 0; k < RPL; ++k) zo[k] = *reinterpret_cast<const V*>(a.z_in + ((size_t)chunk * n + ro[k]) * CB);
  }
  if (a.mode != ROW_INIT0) {
    const int gq = (a.G + 3) / 4, g0 = wv * gq, g1 = min(a.G, g0 + gq);
    V acc[RPL] = {};
    if (pil) {
      const V* p = reinterpret_cast<const V*>(a.abp) + (size_t)chunk * a.G * n;
      for (int gg = g0; gg < g1; gg += U) {
        V t[RPL][U];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int k = 0; k < RPL; ++k)  // dead after this read: streaming loads
            t[k][u] = __builtin_nontemporal_load(p + (size_t)(gg + u < g1 ? gg + u : g0) * n + ro[k]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (gg + u < g1)
#pragma unroll
            for (int k = 0; k < RPL; ++k) acc[k] += t[k][u];
      }
    } else {  // the beta0 start only (once per decode): a plain loop
      for (int g = g0; g < g1; ++g)
#pragma unroll
        for (int k = 0; k < RPL; ++k)
#pragma unroll
          for (int c = 0; c < CB; ++c) acc[k][c] += a.abp[((size_t)bc[c] * a.G + g) * n + ro[k]];
    }
#pragma unroll
    for (int k = 0; k < RPL; ++k) red[wv][k][lane] = acc[k];
  }
  __syncthreads();
  if (wv != 0) return;
  real q[CB] = {};
  bool live[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    live[c] = valid[c] && !(a.mode == ROW_AMP && a.early_stop && tau[c] == last[c]);
    real ons = 0;
    const real tau2 = tau[c] * tau[c];
    if (a.mode == ROW_AMP) {
      real sacc = 0;
      sacc += bbv[c][0];
      sacc += bbv[c][1];
      const real bb = a.Gb <= 128 ? wave_sum(sacc) : wave_sum_parts(a.bbp + (size_t)bc[c] * a.Gb, a.Gb);
      ons = a.Pb[(size_t)bc[c] * a.Pbst] - bb / (real)n;
    }
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      real z;
      if (a.mode == ROW_INIT0) {
        z = yv[k][c];
      } else {
        const real sv = ((red[0][k][lane][c] + red[1][k][lane][c]) + red[2][k][lane][c]) + red[3][k][lane][c];
        z = yv[k][c] - sv / a.sqrt_n;
        if (a.mode == ROW_AMP) z += (zo[k][c] / tau2) * ons;
      }
      if (!valid[c]) z = 0;
      else if (!live[c]) z = zo[k][c];  // a stopped codeword keeps its residual
      zo[k][c] = z;                     // now the new residual
      if (in[k]) q[c] += z * z;
    }
  }
#pragma unroll
  for (int k = 0; k < RPL; ++k)
    if (in[k]) *reinterpret_cast<V*>(a.z + ((size_t)chunk * n + rr[k]) * CB) = zo[k];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const real sz = wave_sum(q[c]);
    if (lane == 0 && live[c]) a.zzp[(size_t)bc[c] * a.NZ + blockIdx.x] = sz;
  }
}

// Row kernel for small batches: 32 rows per 512-thread workgroup, so the
// ceil(n/32) workgroups of a codeword spread over twice as many CUs as
// k_row's 64-row workgroups.  Thread (row rl, group pg) sums the Ab
// partials g = pg, pg+16, ... of its row in order
// (all loads of a thread in flight together); the 16 group sums are added in
// group order; wave 0 finishes the rows (Onsager residual, z^2 partial).
// R = 16 (row-block-major partials only, where the line holds two partials of
// the same block): twice the workgroups, NG = 32 partial groups of G / 32
template <typename real, int R = kRow2Rows, int NT = 512>
__global__ void __launch_bounds__(NT) k_row2(RowArgs<real> a) {
  constexpr int NG = NT / R;  // partial groups
  __shared__ real red[NG][R + 1];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int rl = tid & (R - 1), pg = tid / R;
  const int r = blockIdx.x * R + rl;
  const int n = a.n;
  // tau_t and tau_{t-1} are loaded with everything else; the early-stop
  // test waits for them only after the Ab-partial loads are in flight
  // (testing first cost a whole memory round trip per launch)
  real tau = 1, last = 0;
  if (a.mode == ROW_AMP) {
    tau = ld_vmem(a.tau + (size_t)b * a.T1 + a.t);
    last = a.t > 0 ? ld_vmem(a.tau + (size_t)b * a.T1 + a.t - 1) : (real)0;
  }
  const size_t o = (size_t)b * n + (r < n ? r : 0);
  real yv = 0, zv = 0, bbv[4] = {0, 0, 0, 0};
  if (tid < 64) {
    yv = a.y[o];
    if (a.mode == ROW_AMP) {
      zv = a.z_in[o];
      const real* bp = a.bbp + (size_t)b * a.Gb;
#pragma unroll
      for (int q = 0; q < 4; ++q) bbv[q] = tid + 64 * q < a.Gb ? bp[tid + 64 * q] : (real)0;
    }
  }
  if (a.mode != ROW_INIT0) {
    // pt: partial g of row r at [b][r / R][g][r % R] (n padded to R rows)
    const size_t gs = a.pt ? (size_t)R : (size_t)n;
    const real* p = a.pt ? a.abp + (size_t)b * a.G * ((size_t)gridDim.x * R) +
                               (size_t)blockIdx.x * a.G * R + rl
                         : a.abp + (size_t)b * a.G * n + (r < n ? r : 0);
    real acc = 0;
    constexpr int U = 256 / NG;  // G = 256 (C2, C4): every load of a thread in one pass
    if (a.pt && (R == 16 || sizeof(real) == 4) && a.G == NG * U) {
      // row-block-major partials with exactly NG x U partials (32-row blocks:
      // binary32 only, C4 single codeword +1 %; the binary64 32-row blocks
      // measured 1.4 % slower in this form).  The [G][n] partials of k_sec
      // (sa_Ab, the beta0 start) take the general loop even in 16-row blocks:
      // constant strides from the block base, no bounds, 32-bit offsets (the
      // general form spent ~40 VALU ops of 64-bit address math before the
      // first load); the same loads and sums in the same order
      const real* pb = a.abp + (size_t)b * a.G * ((size_t)gridDim.x * R) + (size_t)blockIdx.x * a.G * R;
      real t[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        t[u] = ld_off(pb, (unsigned)(((pg + NG * u) * R + rl) * (int)sizeof(real)));
#pragma unroll
      for (int u = 0; u < U; ++u) acc += t[u];
    } else
    for (int g0 = pg; g0 < a.G; g0 += NG * U) {
      real t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int g = g0 + NG * u;
        t[u] = p[(size_t)(g < a.G ? g : pg) * gs];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (g0 + NG * u < a.G) acc += t[u];
    }
    red[pg][rl] = acc;
  }
  if (a.mode == ROW_AMP && a.early_stop && tau == last) return;  // uniform over the workgroup
  const real tau2 = tau * tau;
  __syncthreads();
  if (tid >= 64) return;
  real ons = 0;
  if (a.mode == ROW_AMP) {
    real bb;
    if (a.Gb <= 256) {
      real sacc = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) sacc += bbv[q];
      bb = wave_sum(sacc);
    } else {
      bb = wave_sum_parts(a.bbp + (size_t)b * a.Gb, a.Gb);
    }
    ons = a.Pb[(size_t)b * a.Pbst] - bb / (real)n;
  }
  real zn = 0;
  if (tid < R && r < n) {
    if (a.mode == ROW_INIT0) {
      zn = yv;
    } else {
      real acc = 0;
#pragma unroll
      for (int q = 0; q < NG; ++q) acc += red[q][rl];
      const real ab = acc / a.sqrt_n;
      if (a.mode == ROW_ABOUT) {
        a.out[o] = ab;
        return;
      }
      zn = yv - ab;
      if (a.mode == ROW_AMP) zn += (zv / tau2) * ons;
    }
    a.z[o] = zn;
  }
  if (a.mode == ROW_ABOUT) return;
  const real sz = wave_sum(zn * zn);
  if (tid == 0) a.zzp[(size_t)b * a.NZ + blockIdx.x] = sz;
}

// Per-section decision (sparc_ldpc.py:452-455): argmax, first index on ties.
template <typename real, int E>
__global__ void __launch_bounds__(256) k_decide(const real* beta, int32_t* idx, int L, int M, int dead) {
  const int lane = threadIdx.x & 63;
  const int l = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y;
  if (l >= L) return;
  const int bi = section_argmax<real, E>(beta + ((size_t)b * L + l) * M, lane, M, dead);
  if (lane == 0) idx[(size_t)b * L + l] = bi;
}

// ---- launchers ------------------------------------------------------------
template <typename real>
int launch_row(sa_ctx* c, int B, int mode, int t, int es, int G, int Gb, int pt, void* zin, void* zout) {
  RowArgs<real> a = row_args<real>(c, mode, t, es, G, Gb);
  a.pt = pt;
  if (zout) a.z = (real*)zout;
  if (zin) a.z_in = (const real*)zin;
  if (c->prof) c->prof->begin(c->stream, K_ROW);
  // small batch: 16-row workgroups cover the chip; many codewords: 64-row
  // workgroups, 4 waves with deeper per-lane load streams
  if (c->row_kind == 5 && mode != ROW_ABOUT) {
    constexpr int CBz = 16 / (int)sizeof(real);  // codewords per 16-byte row
    a.Bc = B;
    // each wave's G / 4 partials in one batch of loads (U = 12: C4's 48 groups)
    if ((a.G + 3) / 4 > 8 && (a.G + 3) / 4 <= 12)
      plaunch(c, k_rowc<real, CBz, 12>, dim3(c->NZ2, (B + CBz - 1) / CBz), 256, 0, a, mode == ROW_AMP ? 1 : 0);
    else
      plaunch(c, k_rowc<real, CBz>, dim3(c->NZ2, (B + CBz - 1) / CBz), 256, 0, a, mode == ROW_AMP ? 1 : 0);
  } else if (c->row_kind == 5) {  // A beta out of k_sec's [B][G][n] partials (sa_Ab after a batched decode)
    plaunch(c, k_row<real, 4>, dim3(c->NZ, B), 4 * 64, 0, a);
  } else if (c->row_kind == 1) {
    plaunch(c, k_row2<real>, dim3(c->NZ16, B), 512, 0, a);
  } else if (c->row_kind == 4) {
    plaunch(c, k_row2<real, 16>, dim3(c->NZh, B), 512, 0, a);
  } else if (c->row_kind == 2) {
    constexpr int V = 16 / (int)sizeof(real);  // 16-byte rows
    plaunch(c, k_rowv<real, V>, dim3(c->nz_cur, B), 256, 0, a);
  } else if (c->row_kind == 3) {
    if constexpr (sizeof(real) == 4) {
      plaunch(c, k_rowv<float, 2>, dim3(c->NZ2, B), 256, 0, a);
    } else {
      return SA_ERR_UNSUPPORTED;  // never chosen for binary64 (row_kind_for)
    }
  } else {
    plaunch(c, k_row<real, 4>, dim3(c->NZ, B), 4 * 64, 0, a);
  }
  if (c->prof) c->prof->end(c->stream);
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

int launch_decide(sa_ctx* c, int B) {
  dim3 grid((c->L + 3) / 4, B);
#define SA_DEC(EE)                                                                                             \
  case EE:                                                                                                     \
    if (c->prec == SA_PREC_F64)                                                                                \
      k_decide<double, EE><<<grid, 256, 0, c->stream>>>((const double*)c->d_beta, c->d_idx, c->L, c->M, c->dead);      \
    else                                                                                                       \
      k_decide<float, EE><<<grid, 256, 0, c->stream>>>((const float*)c->d_beta, c->d_idx, c->L, c->M, c->dead);        \
    break;
  switch (c->E) { SA_DEC(1) SA_DEC(2) SA_DEC(4) SA_DEC(8) SA_DEC(16) SA_DEC(32) SA_DEC(64) }
#undef SA_DEC
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

template int launch_row<float>(sa_ctx*, int, int, int, int, int, int, int, void*, void*);
template int launch_row<double>(sa_ctx*, int, int, int, int, int, int, int, void*, void*);

}  // namespace sa
