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

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <random>
#include <thread>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "sparc_amp.h"

// 0.3: sa_profile / sa_profile_rep write 2 * sa_profile_kinds() + 1 doubles (13 since 0.2)
// 0.4: sa_profile_dispatch (dispatch-bound event pairs), sa_decide_async / sa_decide_collect
#define SA_VERSION "sparc_amp 0.4 gfx950"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return fail(SA_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e));   \
  } while (0)

using f4 = float __attribute__((ext_vector_type(4)));
using d2v = double __attribute__((ext_vector_type(2)));



// Load of a uniform value as a VECTOR load (opaque zero lane offset): a scalar
// load's lgkmcnt wait would also wait for it at the next use of any other
// scalar (SMEM returns out of order), serialising a memory round trip in
// front of the kernel's other loads.
template <typename T>
__device__ __forceinline__ T ld_vmem(const T* p) {
  int z0;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
  return p[z0];
}

// Load of a uniform value through the scalar cache (constant address space):
// no VGPRs; only for values written before the kernel started (the scalar
// cache is invalidated at dispatch) and read where no LDS access is in flight
// (lgkmcnt is shared with LDS).
template <typename T>
__device__ __forceinline__ T ld_smem(const T* p) {
  return *(const __attribute__((address_space(4))) T*)(p);
}

// load at a uniform base + 32-bit byte offset (SGPR-base addressing, no
// 64-bit address arithmetic per load)
template <typename T>
__device__ __forceinline__ T ld_off(const T* base, unsigned byte_off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Store of a partial another kernel reads after the boundary (Ab partials):
// non-temporal, so no dirty L2 line is left for the kernel-end writeback to
// drain (c2: k_sec4 7.85 -> 7.65 us, +1.5 % codewords/s; c3 neutral).
template <typename T>
__device__ __forceinline__ void st_part(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------

// Element held by (lane, register i) for a section of M = 64*E columns
// (or M <= 64 with E = 1, lanes >= M idle).  The low log2(Q) index bits live
// in consecutive registers so global accesses are Q-wide vectors.
template <int E>
__device__ __forceinline__ int elem_index(int lane, int i) {
  constexpr int Q = E < 4 ? E : 4;
  return (i / Q) * (64 * Q) + lane * Q + (i % Q);
}

// Cross-lane partner x[lane ^ m] for constant m, all on the VALU:
// xor 1/2: DPP quad_perm; xor 4/8: DPP row_shl/row_shr by m selected by lane
// bit (the shifted-in out-of-row lanes are never selected); xor 16/32:
// v_permlane16_swap / v_permlane32_swap (gfx950).  Doubles move as halves.
template <int m>
__device__ __forceinline__ int xor_lane_i32(int x) {
  if constexpr (m == 1) {
    return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  } else if constexpr (m == 2) {
    return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  } else if constexpr (m == 8) {
    return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true);  // row_ror:8 = lane ^ 8
  } else if constexpr (m == 4) {
    // two bank-masked DPP moves into one register, no copy and no select:
    // the banks (4-lane groups of a 16-lane row) whose lane bit 2 is set take
    // row_shr:4 (lane - 4), the others row_shl:4 (lane + 4), every source lane
    // inside its row (the first move leaves the other banks undefined, the
    // second fills them)
    const int dn = __builtin_amdgcn_mov_dpp(x, 0x114, 0xF, 0xA, false);
    return __builtin_amdgcn_update_dpp(dn, x, 0x104, 0xF, 0x5, false);
  } else if constexpr (m == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (threadIdx.x & 16) ? (int)r[0] : (int)r[1];
  } else {
    static_assert(m == 32, "xor mask");
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (threadIdx.x & 32) ? (int)r[0] : (int)r[1];
  }
}

template <int m, typename real>
__device__ __forceinline__ real xor_lane(real x) {
  if constexpr (sizeof(real) == 4) {
    return __int_as_float(xor_lane_i32<m>(__float_as_int(x)));
  } else {
    const long long u = __double_as_longlong(x);
    const int lo = xor_lane_i32<m>((int)(u & 0xffffffffLL));
    const int hi = xor_lane_i32<m>((int)(u >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
}

// ---- binary32 cross-lane primitives with the data movement fused ---------
// DPP move with every lane valid (row_ror / quad_perm): the compiler folds it
// into the consuming add (v_add_f32_dpp).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
constexpr int kRor8 = 0x128, kRor4 = 0x124, kQuadX2 = 0x4E, kQuadX1 = 0xB1;

// v_max_f32 without the NaN-quieting canonicalisations fmaxf carries (the
// operands here are finite or -inf)
__device__ __forceinline__ float max_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Sum / max over each 16-lane row, every lane of the row receiving it: the
// xor 8 / 4 / 2 / 1 stages of wave_sum as single fused-DPP ops.  row_ror:8 is
// lane ^ 8; after it every lane holds the same value as its lane ^ 8 partner,
// so row_ror:4 adds the same operands as lane ^ 4 would (identical bits).
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f32<kRor8>(v);
  v += dpp_f32<kRor4>(v);
  v += dpp_f32<kQuadX2>(v);
  v += dpp_f32<kQuadX1>(v);
  return v;
}
// (max in inline asm: fmaxf's canonicalisations keep the compiler from fusing
// the DPP move; each DPP op reads the previous VALU result, so two wait states
// separate them, and the block is fenced by them on both sides)
__device__ __forceinline__ float row_max16(float v) {
  float r;
  asm("s_nop 1\n\t"
      "v_max_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "s_nop 1"
      : "=&v"(r)
      : "v"(v));
  return r;
}

// v_permlane{16,32}_swap of (a, b): returns {a's lower rows / half next to b's
// lower ones, a's upper next to b's upper} (the lane placement of the ISA op)
template <int m>
__device__ __forceinline__ void perm_swap(float a, float b, float& lo, float& hi) {
  static_assert(m == 16 || m == 32, "swap width");
  const auto r = m == 16 ? __builtin_amdgcn_permlane16_swap(__float_as_int(a), __float_as_int(b), false, false)
                         : __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(b), false, false);
  lo = __int_as_float((int)r[0]);
  hi = __int_as_float((int)r[1]);
}
// binary64 values cross lanes as two 32-bit halves
__device__ __forceinline__ int dlo(double x) { return (int)(__double_as_longlong(x) & 0xffffffffLL); }
__device__ __forceinline__ int dhi(double x) { return (int)(__double_as_longlong(x) >> 32); }
__device__ __forceinline__ double djoin(int lo, int hi) {
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int m>
__device__ __forceinline__ void perm_swap(double a, double b, double& lo, double& hi) {
  float l0, h0, l1, h1;
  perm_swap<m>(__int_as_float(dlo(a)), __int_as_float(dlo(b)), l0, h0);
  perm_swap<m>(__int_as_float(dhi(a)), __int_as_float(dhi(b)), l1, h1);
  lo = djoin(__float_as_int(l0), __float_as_int(l1));
  hi = djoin(__float_as_int(h0), __float_as_int(h1));
}
__device__ __forceinline__ double max_raw(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// The xor 32 (16) reduction stage of two values at once: lanes 0-31 (rows
// 0, 2) receive a's lower + upper halves (rows), lanes 32-63 (rows 1, 3) b's
template <int m, bool MAX, typename T>
__device__ __forceinline__ T swap_op(T a, T b) {
  T lo, hi;
  perm_swap<m>(a, b, lo, hi);
  return MAX ? max_raw(lo, hi) : lo + hi;
}
__device__ __forceinline__ float readlane_f32(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_f32(double v, int l) {
  return djoin(__builtin_amdgcn_readlane(dlo(v), l), __builtin_amdgcn_readlane(dhi(v), l));
}
// binary64 row stages: each half moved by the same DPP control, then one op
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  return djoin(__builtin_amdgcn_mov_dpp(dlo(x), CTRL, 0xF, 0xF, true),
               __builtin_amdgcn_mov_dpp(dhi(x), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_f64<kRor8>(v);
  v += dpp_f64<kRor4>(v);
  v += dpp_f64<kQuadX2>(v);
  v += dpp_f64<kQuadX1>(v);
  return v;
}
__device__ __forceinline__ double row_max16(double v) {
  v = max_raw(v, dpp_f64<kRor8>(v));
  v = max_raw(v, dpp_f64<kRor4>(v));
  v = max_raw(v, dpp_f64<kQuadX2>(v));
  v = max_raw(v, dpp_f64<kQuadX1>(v));
  return v;
}

// Reductions of CB per-codeword wave values together (binary32): codeword
// pairs share the permlane32 stage (one per 32-lane half), pairs of those the
// permlane16 stage (one codeword per 16-lane row: 0, 2, 1, 3), then one row
// reduction serves all; the same operand pairs in the same order as
// wave_sum / wave_max per codeword, so the same bits.  Results are uniform.
template <bool MAX, int CB, typename T>
__device__ __forceinline__ void wave_reduce_cb(T (&v)[CB]) {
  static_assert(CB == 1 || CB == 2 || CB == 4, "codewords per reduction");
  if constexpr (CB == 1) {
    T p = swap_op<32, MAX>(v[0], v[0]);
    p = swap_op<16, MAX>(p, p);
    v[0] = readlane_f32(MAX ? row_max16(p) : row_sum16(p), 0);
  } else if constexpr (CB == 2) {
    T p = swap_op<32, MAX>(v[0], v[1]);
    p = swap_op<16, MAX>(p, p);
    p = MAX ? row_max16(p) : row_sum16(p);
    v[0] = readlane_f32(p, 0);
    v[1] = readlane_f32(p, 32);
  } else {
    const T p01 = swap_op<32, MAX>(v[0], v[1]);
    const T p23 = swap_op<32, MAX>(v[2], v[3]);
    T q = swap_op<16, MAX>(p01, p23);
    q = MAX ? row_max16(q) : row_sum16(q);
    v[0] = readlane_f32(q, 0);
    v[2] = readlane_f32(q, 16);
    v[1] = readlane_f32(q, 32);
    v[3] = readlane_f32(q, 48);
  }
}
// Butterfly on lane bit 4 or 8 (binary32): the lower banks of each row take
// x + x[lane + m], the upper ones x[lane - m] - x, each as one bank-masked
// DPP add / sub (two VALU ops per element instead of two moves and an fma;
// the same two operands and rounding).  Two wait states fence the block.
template <int m, int E>
__device__ __forceinline__ void bfly_bank_f32(float (&x)[E]) {
  static_assert(m == 4 || m == 8, "bank butterfly");
  static_assert(E == 1 || E % 2 == 0, "pairs");
#pragma unroll
  for (int i = 0; i < E; i += 2) {
    float r0, r1;
    if constexpr (E == 1) {
      if constexpr (m == 4)
        asm("s_nop 1\n\t"
            "v_add_f32_dpp %0, %1, %1 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
            "v_sub_f32_dpp %0, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
            "s_nop 1"
            : "=&v"(r0) : "v"(x[i]));
      else
        asm("s_nop 1\n\t"
            "v_add_f32_dpp %0, %1, %1 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
            "v_sub_f32_dpp %0, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
            "s_nop 1"
            : "=&v"(r0) : "v"(x[i]));
      x[i] = r0;
    } else {
      if constexpr (m == 4)
        asm("s_nop 1\n\t"
            "v_add_f32_dpp %0, %2, %2 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
            "v_add_f32_dpp %1, %3, %3 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
            "v_sub_f32_dpp %0, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
            "v_sub_f32_dpp %1, %3, %3 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
            "s_nop 1"
            : "=&v"(r0), "=&v"(r1) : "v"(x[i]), "v"(x[i + 1]));
      else
        asm("s_nop 1\n\t"
            "v_add_f32_dpp %0, %2, %2 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
            "v_add_f32_dpp %1, %3, %3 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
            "v_sub_f32_dpp %0, %2, %2 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
            "v_sub_f32_dpp %1, %3, %3 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
            "s_nop 1"
            : "=&v"(r0), "=&v"(r1) : "v"(x[i]), "v"(x[i + 1]));
      x[i] = r0;
      x[i + 1] = r1;
    }
  }
}

// Butterfly on lane bit 16 or 32 (binary32) for two elements at once: one
// permlane swap puts both elements' lower halves (rows) in one register and
// their upper ones in another, an add and a sub form the outputs, a second
// swap puts them back in place: four VALU ops per two elements instead of six
// (lower lanes a + b, upper a - b, as before).
template <int m, typename real, int E>
__device__ __forceinline__ void bfly_swap(real (&x)[E]) {
  static_assert(E % 2 == 0, "pairs");
#pragma unroll
  for (int i = 0; i < E; i += 2) {
    real a, b;
    perm_swap<m>(x[i], x[i + 1], a, b);
    perm_swap<m>(a + b, a - b, x[i], x[i + 1]);
  }
}

// One lane-bit butterfly stage: lower lane x + p, upper lane p - x, as a
// single fma with the per-lane sign (+1 lower, -1 upper).
template <int m, typename real, int E>
__device__ __forceinline__ void lane_butterfly(real (&x)[E], int lane) {
  const real sg = (lane & m) ? (real)-1 : (real)1;
  if constexpr ((m == 4 || m == 8) && sizeof(real) == 4) {
    bfly_bank_f32<m, E>(x);
  } else if constexpr ((m == 16 || m == 32) && E % 2 == 0) {
    bfly_swap<m, real, E>(x);
  } else if constexpr ((m == 16 || m == 32) && sizeof(real) == 4) {
    // v_permlane{16,32}_swap of x with itself leaves a = the lower partner
    // and b = the upper one in every lane: lower lanes a + b, upper a - b
    // (the same two operands and rounding as fma(x, sg, partner))
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const int u = __float_as_int(x[i]);
      const auto r = m == 16 ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                             : __builtin_amdgcn_permlane32_swap(u, u, false, false);
      x[i] = fma(__int_as_float((int)r[1]), sg, __int_as_float((int)r[0]));
    }
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      const real p = xor_lane<m>(x[i]);
      x[i] = fma(x[i], sg, p);
    }
  }
}

// Full-wave xor-butterfly reductions (fixed order: deterministic bits).
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  if constexpr ((T)0.5 != 0) {  // floating point: fused stages, same pairs
    v = swap_op<32, false>(v, v);
    v = swap_op<16, false>(v, v);
    return row_sum16(v);
  }
  v += xor_lane<32>(v);
  v += xor_lane<16>(v);
  v += xor_lane<8>(v);
  v += xor_lane<4>(v);
  v += xor_lane<2>(v);
  v += xor_lane<1>(v);
  return v;
}

template <typename T>
__device__ __forceinline__ void wave_sum2(T& a, T& b) {
  if constexpr ((T)0.5 != 0) {  // floating point: both in one register after xor 32
    T v[2] = {a, b};
    wave_reduce_cb<false, 2>(v);
    a = v[0];
    b = v[1];
    return;
  }
  a += xor_lane<32>(a); b += xor_lane<32>(b);
  a += xor_lane<16>(a); b += xor_lane<16>(b);
  a += xor_lane<8>(a); b += xor_lane<8>(b);
  a += xor_lane<4>(a); b += xor_lane<4>(b);
  a += xor_lane<2>(a); b += xor_lane<2>(b);
  a += xor_lane<1>(a); b += xor_lane<1>(b);
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
  if constexpr ((T)0.5 != 0) {  // floating point
    T r[1] = {v};
    wave_reduce_cb<true, 1>(r);
    return r[0];
  }
  T o;
  o = xor_lane<32>(v); v = o > v ? o : v;
  o = xor_lane<16>(v); v = o > v ? o : v;
  o = xor_lane<8>(v); v = o > v ? o : v;
  o = xor_lane<4>(v); v = o > v ? o : v;
  o = xor_lane<2>(v); v = o > v ? o : v;
  o = xor_lane<1>(v); v = o > v ? o : v;
  return v;
}

// In-wave natural-order Walsh-Hadamard transform of one section.
// Butterfly (a, b) -> (a + b, a - b) on every index bit: register bits first,
// then lane bits (only the first log2(mlanes) lane bits when M < 64).
template <typename real, int E>
__device__ __forceinline__ void fwht_wave(real (&x)[E], int lane, int mlanes) {
#pragma unroll
  for (int h = 1; h < E; h <<= 1) {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (!(i & h)) {
        real a = x[i], b = x[i | h];
        x[i] = a + b;
        x[i | h] = a - b;
      }
    }
  }
  if (mlanes > 1) lane_butterfly<1>(x, lane);
  if (mlanes > 2) lane_butterfly<2>(x, lane);
  if (mlanes > 4) lane_butterfly<4>(x, lane);
  if (mlanes > 8) lane_butterfly<8>(x, lane);
  if (mlanes > 16) lane_butterfly<16>(x, lane);
  if (mlanes > 32) lane_butterfly<32>(x, lane);
}

// The same transform (binary32, E >= 2, all 64 lanes) with the lane-bit 0 / 1
// butterflies as single in-place DPP fmas x += s * x[lane ^ m] (s = +1 in the
// lower lane, -1 in the upper): the upper lane then holds b - a = -(a - b),
// exactly (rounding is sign-symmetric), and the later stages pair lanes of
// equal sign, so lane L ends with (-1)^(L0 + L1) times the value fwht_wave
// leaves there.  s1 / s2 are the per-lane signs of lane bits 0 / 1.  The
// caller cancels the sign (k_secb: input signs, quad-mirrored section
// positions and a signed 1/sqrt(n); see there).
template <int E>
__device__ __forceinline__ void fwht_wave_sgn(float (&x)[E], float s1, float s2) {
  static_assert(E >= 2 && E % 2 == 0, "pairs of elements");
#pragma unroll
  for (int h = 1; h < E; h <<= 1) {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (!(i & h)) {
        const float a = x[i], b = x[i | h];
        x[i] = a + b;
        x[i | h] = a - b;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < E; i += 2)
    asm("s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %0, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %0, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %1, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(x[i]), "+v"(x[i + 1])
        : "v"(s1), "v"(s2));
  bfly_bank_f32<4, E>(x);
  bfly_bank_f32<8, E>(x);
  bfly_swap<16, float, E>(x);
  bfly_swap<32, float, E>(x);
}

// fwht_wave_sgn of two sections' values at once (binary32): each DPP stage is
// one asm block over four registers of x and y (one pair of wait states per
// block instead of per two registers, and four independent ops between a
// register's write and its next DPP read); the same operations on every
// register, so the same bits as two fwht_wave_sgn calls.
__device__ __forceinline__ void quad_fmac4(float& a, float& b, float& c, float& d, float s1, float s2) {
  asm("s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %0, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %0, %5 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %1, %5 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %2, %5 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %3, %5 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
      : "v"(s1), "v"(s2));
}
template <int m>
__device__ __forceinline__ void bank_bfly4(float& a, float& b, float& c, float& d) {
  static_assert(m == 4 || m == 8, "bank butterfly");
  float r0, r1, r2, r3;
  if constexpr (m == 4)
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %4, %4 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_add_f32_dpp %1, %5, %5 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_add_f32_dpp %2, %6, %6 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_add_f32_dpp %3, %7, %7 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
        "v_sub_f32_dpp %0, %4, %4 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
        "v_sub_f32_dpp %1, %5, %5 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
        "v_sub_f32_dpp %2, %6, %6 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
        "v_sub_f32_dpp %3, %7, %7 row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
        "s_nop 1"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(a), "v"(b), "v"(c), "v"(d));
  else
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %4, %4 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %1, %5, %5 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %2, %6, %6 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_add_f32_dpp %3, %7, %7 row_shl:8 row_mask:0xf bank_mask:0x3\n\t"
        "v_sub_f32_dpp %0, %4, %4 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
        "v_sub_f32_dpp %1, %5, %5 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
        "v_sub_f32_dpp %2, %6, %6 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
        "v_sub_f32_dpp %3, %7, %7 row_shr:8 row_mask:0xf bank_mask:0xc\n\t"
        "s_nop 1"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3) : "v"(a), "v"(b), "v"(c), "v"(d));
  a = r0; b = r1; c = r2; d = r3;
}
template <int E>
__device__ __forceinline__ void fwht_wave_sgn_pair(float (&x)[E], float (&y)[E], float s1, float s2) {
  static_assert(E >= 2 && E % 2 == 0, "pairs of elements");
#pragma unroll
  for (int h = 1; h < E; h <<= 1) {
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (!(i & h)) {
        const float a = x[i], b = x[i | h];
        x[i] = a + b;
        x[i | h] = a - b;
        const float c = y[i], d = y[i | h];
        y[i] = c + d;
        y[i | h] = c - d;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < E; i += 2) quad_fmac4(x[i], x[i + 1], y[i], y[i + 1], s1, s2);
#pragma unroll
  for (int i = 0; i < E; i += 2) bank_bfly4<4>(x[i], x[i + 1], y[i], y[i + 1]);
#pragma unroll
  for (int i = 0; i < E; i += 2) bank_bfly4<8>(x[i], x[i + 1], y[i], y[i + 1]);
  bfly_swap<16, float, E>(x);
  bfly_swap<16, float, E>(y);
  bfly_swap<32, float, E>(x);
  bfly_swap<32, float, E>(y);
}

// exp(x) for x <= 0 in binary64 from a 64-entry table of 2^(j/64) in LDS:
// k = rint(x 64 / ln 2), r = x - k ln2/64 (Cody-Waite, |r| <= ln2/128),
// e^x = 2^(k >> 6) 2^((k & 63)/64) e^r with e^r by a degree-5 polynomial
// (truncation below 4e-17): within two ulps of the correctly rounded value;
// 0 below -745.2 (where exp underflows to 0) and for -inf.
__constant__ double c_exp2_64[64] = {  // 2^(j/64), correctly rounded (generated with decimal, 80 digits)
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0};
__device__ __forceinline__ double exp_neg_tab(double x, const double* tab) {
  const double kd = __builtin_rint(x * 0x1.71547652b82fep+6);  // x 64 / ln 2
  double r = fma(kd, -0x1.62e42fefa0000p-7, x);                  // ln2/64, high part (exact products)
  r = fma(kd, -0x1.cf79abc9e3b3ap-46, r);  // ln2/64, low part
  const int k = (int)kd;
  double p = fma(r, 1.0 / 120, 1.0 / 24);
  p = fma(r, p, 1.0 / 6);
  p = fma(r, p, 0.5);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  const double y = __builtin_amdgcn_ldexp(tab[k & 63] * p, k >> 6);
  return x < -745.2 ? 0.0 : y;
}

template <typename real> __device__ __forceinline__ real dsqrt(real x);
template <> __device__ __forceinline__ float dsqrt<float>(float x) { return sqrtf(x); }
template <> __device__ __forceinline__ double dsqrt<double>(double x) { return sqrt(x); }
template <typename real> __device__ __forceinline__ real dexp(real x);
// binary32: the native v_exp_f32 (exp2 of x log2 e; relative error ~1e-7 near
// the section maximum, ~5e-6 at e^-87), well inside the fp32 parity bound,
// instead of the ~10-instruction range-reduced expf
template <> __device__ __forceinline__ float dexp<float>(float x) { return __expf(x); }
template <> __device__ __forceinline__ double dexp<double>(double x) { return exp(x); }
// 1/x to about 1 ulp in one instruction (binary32 v_rcp_f32); binary64 keeps the division
__device__ __forceinline__ float rcp_fast(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double rcp_fast(double x) { return 1.0 / x; }
template <typename real> __device__ __forceinline__ real neg_inf();
template <> __device__ __forceinline__ float neg_inf<float>() { return -INFINITY; }
template <> __device__ __forceinline__ double neg_inf<double>() { return -INFINITY; }

// Deterministic sum of `cnt` partials by one full wavefront: lane i adds
// partials i, i+64, ... in order, then a fixed xor-butterfly.  Every wave
// that evaluates it (in any workgroup) gets the same bits, and all loads of
// a lane are independent, so the latency is one round trip, not cnt.
// (Loads are unconditional with a clamped index and issued four at a time
// before the adds: a conditional load with its add sunk into the branch makes
// the compiler wait for each load on the spot, one round trip per partial.)
template <typename real>
__device__ __forceinline__ real wave_sum_parts(const real* p, int cnt) {
  const int lane = threadIdx.x & 63;
  real s = 0;
  for (int i0 = lane; i0 < cnt; i0 += 256) {
    real t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 64 * u;
      t[u] = p[i < cnt ? i : i0];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s += i0 + 64 * u < cnt ? t[u] : (real)0;
  }
  return wave_sum(s);
}

// The same sum for cnt <= 128 partials already loaded by the caller (lane i
// holds partials i and i + 64, zero beyond cnt).
template <typename real>
__device__ __forceinline__ real wave_sum_pair(real a, real b) {
  real s = 0;
  s += a;
  s += b;
  return wave_sum(s);
}

// The z^2 partials for tau, loaded ahead of everything else a kernel needs
// (vmcnt retires loads in order: tau then waits for these alone).  Same sum
// as wave_sum_parts for NZ <= 64 * K.  The loads are unconditional (clamped
// index, masked in tau()): with `cond ? p[i] : 0` the compiler sank the first
// add into the branch and waited for that load before issuing anything else.
template <typename real, int K = 4>
struct ZZParts {
  real v[K];
  template <bool SC1 = false>
  __device__ __forceinline__ void issue(const real* p, int cnt, int lane) {
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const int i = lane + 64 * q;
      v[q] = SC1 ? __hip_atomic_load(p + (i < cnt ? i : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : p[i < cnt ? i : 0];
    }
  }
  __device__ __forceinline__ real tau(const real* p, int cnt, int n) const {
    const int lane = threadIdx.x & 63;
    real s;
    if (cnt <= 64 * K) {
      s = 0;
#pragma unroll
      for (int q = 0; q < K; ++q) s += lane + 64 * q < cnt ? v[q] : (real)0;
      s = wave_sum(s);
    } else {
      s = wave_sum_parts(p, cnt);
    }
    return dsqrt<real>(s / (real)n);
  }
};

// tau_t from the row kernel's per-block partial sums of z^2: sparc_ldpc.py:203.
template <typename real>
__device__ __forceinline__ real tau_from_parts(const real* zzp, int NZ, int n) {
  return dsqrt<real>(wave_sum_parts(zzp, NZ) / (real)n);
}

template <typename real, int E>
__device__ __forceinline__ void store_section(real* p, const real (&x)[E], int lane, int M);

// Section-wise denoiser eta (sparc_ldpc.py:213-219) on one wave's section.
// v holds Az_l(z) * sqrt(n) (unscaled); bprev the previous estimate (same
// element layout).  v receives the new estimate, which is also stored to
// beta_l; returns sum(beta_new^2) over the section (every lane).
// The max is per section rather than global (:216): the ratio exp(u-m)/sum is
// independent of m, and the per-section max cannot underflow a section.
template <typename real, int E>
__device__ __forceinline__ real denoise_section(real (&v)[E], const real (&bprev)[E], real* beta_l,
                                                int lane, int M, real cl, real tau2, real sqrt_n,
                                                bool store = true) {
  // u = (beta + Az/sqrt(n)) * sqrt(n Pl) / tau^2 with the two divisions of
  // :213/:215 folded into one per-section scale
  const real inv_sn = (real)1 / sqrt_n;
  const real k = cl / tau2;
  real u[E];
  real mx = neg_inf<real>();
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = elem_index<E>(lane, i);
    const real s = fma(v[i], inv_sn, bprev[i]);   // :213
    const real uu = s * k;                          // :215
    u[i] = e < M ? uu : neg_inf<real>();
    mx = u[i] > mx ? u[i] : mx;
  }
  mx = wave_max(mx);                                // :216 (per section)
  real S = 0, S2 = 0;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    u[i] = dexp<real>(u[i] - mx);                   // :217; exp(-inf) = 0 on idle lanes
    S += u[i];
    S2 += u[i] * u[i];
  }
  wave_sum2(S, S2);                                 // :218 and sum(beta^2) together
  const real scale = cl / S;                        // :219
#pragma unroll
  for (int i = 0; i < E; ++i) v[i] = u[i] * scale;
  if (store) store_section<real, E>(beta_l, v, lane, M);
  return S2 * scale * scale;                        // sum(beta^2) over the section
}

// Q-wide vector load / store of one wave's section elements (E per lane).
template <typename real, int E>
__device__ __forceinline__ void load_section(const real* p, real (&x)[E], int lane, int M) {
  constexpr int Q = E < 4 ? E : 4;
#pragma unroll
  for (int i = 0; i < E; i += Q) {
    const int e0 = elem_index<E>(lane, i);
    if constexpr (Q == 4 && sizeof(real) == 4) {
      const float4 t = *reinterpret_cast<const float4*>(p + e0);
      x[i] = t.x; x[i + 1] = t.y; x[i + 2] = t.z; x[i + 3] = t.w;
    } else {
      // unconditional loads (clamped index, masked after): a load inside a
      // branch keeps the compiler from counting the loads in flight, and a
      // later wait for an earlier load then becomes a wait for all of them
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if constexpr (sizeof(real) == 4) {
          const real t = p[e0 + q < M ? e0 + q : 0];
          x[i + q] = e0 + q < M ? t : (real)0;
        } else {  // binary64: the conditional form (the select costs the 128-VGPR batched kernel spills)
          x[i + q] = e0 + q < M ? p[e0 + q] : (real)0;
        }
      }
    }
  }
}

// Streaming (non-temporal) forms for beta in the batched kernel: read once
// and written once per launch, 268 MB at c3 (537 MB in binary64), it
// otherwise sweeps each XCD's 4 MB L2 and evicts the section tables and z
// that the XCD's workgroups share.  16-B vectors (binary64: two per group of
// four elements; element-wise non-temporal binary64 access measured 18 %
// slower at c3).  Only for the batched kernel's sections,
// where E >= 4 means M = 64 E: every element of a lane's groups exists.
template <typename real, int E>
__device__ __forceinline__ void load_section_nt(const real* p, real (&x)[E], int lane, int M) {
  constexpr int Q = E < 4 ? E : 4;
  if constexpr (Q == 4 && sizeof(real) == 4) {
#pragma unroll
    for (int i = 0; i < E; i += Q) {
      const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p + elem_index<E>(lane, i)));
      x[i] = t.x; x[i + 1] = t.y; x[i + 2] = t.z; x[i + 3] = t.w;
    }
  } else if constexpr (Q == 4 && sizeof(real) == 8) {
#pragma unroll
    for (int i = 0; i < E; i += Q) {
      const d2v* q = reinterpret_cast<const d2v*>(p + elem_index<E>(lane, i));
      const d2v t0 = __builtin_nontemporal_load(q), t1 = __builtin_nontemporal_load(q + 1);
      x[i] = t0.x; x[i + 1] = t0.y; x[i + 2] = t1.x; x[i + 3] = t1.y;
    }
  } else {
    load_section<real, E>(p, x, lane, M);
  }
}
template <typename real, int E>
__device__ __forceinline__ void store_section_nt(real* p, const real (&x)[E], int lane, int M) {
  constexpr int Q = E < 4 ? E : 4;
  if constexpr (Q == 4 && sizeof(real) == 4) {
#pragma unroll
    for (int i = 0; i < E; i += Q) {
      const f4 t = {x[i], x[i + 1], x[i + 2], x[i + 3]};
      __builtin_nontemporal_store(t, reinterpret_cast<f4*>(p + elem_index<E>(lane, i)));
    }
  } else if constexpr (Q == 4 && sizeof(real) == 8) {
#pragma unroll
    for (int i = 0; i < E; i += Q) {
      d2v* q = reinterpret_cast<d2v*>(p + elem_index<E>(lane, i));
      const d2v t0 = {x[i], x[i + 1]}, t1 = {x[i + 2], x[i + 3]};
      __builtin_nontemporal_store(t0, q);
      __builtin_nontemporal_store(t1, q + 1);
    }
  } else {
    store_section<real, E>(p, x, lane, M);
  }
}

template <typename real, int E>
__device__ __forceinline__ void store_section(real* p, const real (&x)[E], int lane, int M) {
  constexpr int Q = E < 4 ? E : 4;
#pragma unroll
  for (int i = 0; i < E; i += Q) {
    const int e0 = elem_index<E>(lane, i);
    if constexpr (Q == 4 && sizeof(real) == 4) {
      *reinterpret_cast<float4*>(p + e0) = make_float4(x[i], x[i + 1], x[i + 2], x[i + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (e0 + q < M) p[e0 + q] = x[i + q];
    }
  }
}

// The same for any M (the dense and host-operator backends accept M that is
// not a power of two, like the reference's sub_fht, sparc_ldpc.py:32-79):
// 16-B vectors only where the four elements exist and the section is 16-B
// aligned, element by element otherwise.
template <typename real, int E>
__device__ __forceinline__ void load_section_any(const real* p, real (&x)[E], int lane, int M) {
  constexpr int Q = E < 4 ? E : 4;
#pragma unroll
  for (int i = 0; i < E; i += Q) {
    const int e0 = elem_index<E>(lane, i);
    if (Q == 4 && sizeof(real) == 4 && (M & 3) == 0 && e0 + 4 <= M) {
      const float4 t = *reinterpret_cast<const float4*>(p + e0);
      x[i] = t.x; x[i + 1] = t.y; x[i + 2] = t.z; x[i + 3] = t.w;
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) x[i + q] = e0 + q < M ? p[e0 + q] : (real)0;
    }
  }
}

template <typename real, int E>
__device__ __forceinline__ void store_section_any(real* p, const real (&x)[E], int lane, int M) {
  constexpr int Q = E < 4 ? E : 4;
#pragma unroll
  for (int i = 0; i < E; i += Q) {
    const int e0 = elem_index<E>(lane, i);
    if (Q == 4 && sizeof(real) == 4 && (M & 3) == 0 && e0 + 4 <= M) {
      *reinterpret_cast<float4*>(p + e0) = make_float4(x[i], x[i + 1], x[i + 2], x[i + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (e0 + q < M) p[e0 + q] = x[i + q];
    }
  }
}

// ---------------------------------------------------------------------------
// Matrix-free Hadamard backend
// ---------------------------------------------------------------------------

enum { SEC_AMP = 0, SEC_AZ = 1, SEC_AB = 2 };
enum { ROW_INIT0 = 0, ROW_INIT = 1, ROW_AMP = 2, ROW_ABOUT = 3 };

constexpr int kSpw = 4;      // sections (wavefronts) per section-kernel workgroup
constexpr int kRowsPerBlk = 64;  // rows per row-kernel workgroup (one per lane)

template <typename real>
struct SecArgs {
  const uint16_t* __restrict__ inv;  // [L][w]  row of ordering value o, or n (zero slot)
  // k_secb: the bucket table in bank-aware step order (build_invb), or null
  const uint16_t* __restrict__ invb;
  // the codeword-interleaved k_secb: invb (or inv) lane-major [L][nhi][64][E]
  const uint16_t* __restrict__ invl;
  // [L] steps of invb's two halves that hold occupied slots (s0 | s1 << 16), or null
  const uint32_t* __restrict__ hs;
  const ushort4* __restrict__ fwd;   // [G][n]  4 sections: (o & (M-1)) | parity(o >> log2 M) << 15
  // k_secb's Ab table (build_fwdb): [Gb * W / 4][npad][4] with npad = n rounded
  // up to 64; entry (s * M + t_pos(k)) | sign << 15 for the workgroup's local
  // section s (t_pos: the staged image's position of column k), each row's W
  // entries in a bank-aware step order
  const ushort4* __restrict__ fwdb;
  const uint32_t* __restrict__ fwd2; // [ceil(L/2)][n] the same entries of one section pair (k_sec2)
  const uint32_t* __restrict__ fwd3; // [ceil(L/3)][n] a section triple, 10-bit fields k | sign<<9 (M <= 512)
  const uint32_t* __restrict__ inv32;  // [L][w] k_secg: inv with 32-bit rows (n >= 65535 or z past the LDS)
  const real* __restrict__ c;        // [L] sqrt(n * Pl), or [B][L] per codeword (cst = L)
  const real* __restrict__ z;        // [B][n]
  real* __restrict__ beta;           // [B][L*M] previous estimate (read)
  real* __restrict__ beta_out;       // [B][L*M] new estimate (k_sec: the other ping-pong buffer)
  real* __restrict__ out;            // [B][L*M] (SEC_AZ)
  real* __restrict__ abp;            // [B][G][n] partial sums of Ab over this group's sections
  real* __restrict__ bbp;            // [B][G]    partial sums of beta^2
  const real* __restrict__ zzp;      // [B][NZ]
  real* __restrict__ tau;            // [B][T1]
  int* __restrict__ iters;           // [B]
  int L, M, n, w, nhi, G, NZ, T1, t, mode, early_stop;
  int cst;  // codeword stride of c: 0 (one power allocation) or L (sa_stage_power_batch)
  int RS;  // row splits: RS workgroups share a section group, each gathers n/RS rows of Ab
  // Ab partial layout of the multi-wave single-codeword kernels: 0 [B][G][n];
  // 1 row-block major [B][ceil(n/32)][G][32] (k_row2 reads one contiguous
  // G x 128-B block per workgroup)
  int pt;
  int B, NC;  // batched kernel: codewords, codeword chunks of CB
  // batched kernel: z and the Ab partials codeword-interleaved by chunk,
  // z [NC][n][CB] and abp [NC][G][n][CB] (16-byte rows, k_rowc), else [B][n] / [B][G][n]
  int zil;
  // batched kernel: section groups per XCD per pass of the work order (the
  // groups whose tables one XCD's L2 holds at a time); >= G / 8: one pass
  int gpx;
  real sqrt_n;
};

template <typename real>
struct RowArgs {
  const real* __restrict__ y;    // [B][n]
  real* __restrict__ z;          // [B][n] the residual (k_row2: the new one is written here)
  const real* __restrict__ z_in; // [B][n] the previous residual (= z)
  const real* __restrict__ abp;  // [B][G][n]
  const real* __restrict__ bbp;  // [B][G]
  real* __restrict__ zzp;        // [B][NZ]
  const real* __restrict__ tau;  // [B][T1]
  real* __restrict__ out;        // [B][n] (ROW_ABOUT)
  int n, G, Gb, NZ, T1, t, mode, early_stop;  // G Ab partials, Gb beta^2 partials
  real sqrt_n;
  // total power P = sum(Pl) read from device memory (never a captured
  // argument: a graph replayed after set_power must see the new P):
  // [B] per codeword (sa_stage_power_batch, Pbst = 1) or one shared value (Pbst = 0)
  const real* __restrict__ Pb;
  int Pbst;
  int pt;  // Ab partial layout (SecArgs::pt); k_row2 only
  int Bc;  // k_rowc: codewords of the decode (the last chunk may be partial)
};

// One workgroup = 4 wavefronts = 4 consecutive sections of one codeword
// (blockIdx.y).  Per wave: v = bucket gather of z (LDS), FWHT, denoise,
// FWHT of the new beta (for Ab), staged to LDS.  Then the workgroup gathers
// its sections' contributions to every row of Ab into abp[b][g][:].
// Bucket-table loads of KH consecutive h-steps for one wave's section:
// tb[hh][j] = inv[h*M + e0(j) .. +Q) (lanes >= M of a small-M section read
// column 0; their values are discarded).
// Staging z (n values) into LDS with 16-B loads: all kZU loads per thread
// are issued up front (static register indices: no scratch), stored after the
// round trip; n beyond 256*kZU 16-B vectors falls back to a plain loop.
constexpr int kZU = 10;
// (explicit members rather than an array: the array form was not promoted to
// registers and its spill store waited for the loads at kernel start)
#define SA_ZU_EACH(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9)
template <typename real, int NT = 256>
struct ZStage {
  // native vector types: HIP's float4 (a struct of unions) defeats SROA
  using vec_t = typename std::conditional<sizeof(real) == 4, f4, d2v>::type;
  static constexpr int V = 16 / sizeof(real);
#define SA_ZU_DECL(u) vec_t t##u;
  SA_ZU_EACH(SA_ZU_DECL)
#undef SA_ZU_DECL
  int nv;
  __device__ __forceinline__ void issue(const real* zb, int n, int tid) {
    nv = ((reinterpret_cast<uintptr_t>(zb) & 15) == 0) ? n / V : 0;
    const vec_t* zv = reinterpret_cast<const vec_t*>(zb);
    const int last = nv > 0 ? nv - 1 : 0;
    // unconditional (clamped): straight-line loads the compiler can count
#define SA_ZU_LOAD(u) { const int j = u * NT + tid; t##u = zv[j < nv ? j : last]; }
    SA_ZU_EACH(SA_ZU_LOAD)
#undef SA_ZU_LOAD
  }
  __device__ __forceinline__ void store(real* zs, const real* zb, int n, int tid) const {
    vec_t* zsv = reinterpret_cast<vec_t*>(zs);
    const vec_t* zv = reinterpret_cast<const vec_t*>(zb);
#define SA_ZU_STORE(u) { const int j = u * NT + tid; if (j < nv) zsv[j] = t##u; }
    SA_ZU_EACH(SA_ZU_STORE)
#undef SA_ZU_STORE
    for (int j = kZU * NT + tid; j < nv; j += NT) zsv[j] = zv[j];
    for (int i = nv * V + tid; i < n; i += NT) zs[i] = zb[i];
    if (tid == 0) zs[n] = 0;
  }
};

// z of one codeword straight into LDS by LDS-DMA (global_load_lds_dwordx4:
// 1 KB per wave-instruction, no VGPR round trip and no ds_write), all of it
// issued at once; the barrier that follows waits for it (vmcnt).  Returns
// false (nothing issued) when z is not 16-B aligned: ZStage then.  c2: k_sec4
// 7.51 -> 7.26 us, +2 % codewords/s.
template <typename real, int NT, int AUX = 0>
__device__ __forceinline__ bool stage_z_dma(const real* zb, real* zs, int n, int tid) {
  if (reinterpret_cast<uintptr_t>(zb) & 15) return false;
  const int lane = tid & 63, nbytes = n * (int)sizeof(real);
  for (int ch = tid >> 6; ch * 1024 < nbytes; ch += NT / 64) {
    const int off = ch * 1024 + lane * 16;
    // whole 16-B pieces only: a piece straddling the end would land z's
    // neighbour in the zero slot zs[n] (any wave's DMA may land after
    // finish_z_dma's store); the tail goes through finish_z_dma
    if (off + 16 <= nbytes)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)((const char*)zb + off),
                                       (__attribute__((address_space(3))) void*)((char*)zs + ch * 1024), 16, 0, AUX);
  }
  return true;
}

// After stage_z_dma: the < 16-B tail of z by ordinary loads, and the zero
// slot zs[n] (gathered for empty buckets).
template <typename real>
__device__ __forceinline__ void finish_z_dma(const real* zb, real* zs, int n, int tid) {
  const int n0 = n * (int)sizeof(real) / 16 * 16 / (int)sizeof(real);
  if (tid < n - n0) zs[n0 + tid] = zb[n0 + tid];
  if (tid == 0) zs[n] = 0;
}

template <int E, int KH>
__device__ __forceinline__ void load_buckets(const uint16_t* __restrict__ il, int h0, int nhi, int M,
                                             int lane, ushort4 (&tb)[KH][(E + 3) / 4]) {
  constexpr int Q = E < 4 ? E : 4;
#pragma unroll
  for (int hh = 0; hh < KH; ++hh) {
    const int h = h0 + hh < nhi ? h0 + hh : nhi - 1;
    const uint16_t* ih = il + (size_t)h * M;
#pragma unroll
    for (int i = 0; i < E; i += Q) {
      int e0 = elem_index<E>(lane, i);
      e0 = e0 < M ? e0 : 0;
      if constexpr (Q == 4) {
        tb[hh][i / Q] = *reinterpret_cast<const ushort4*>(ih + e0);
      } else if constexpr (Q == 2) {
        const ushort2 t2 = *reinterpret_cast<const ushort2*>(ih + e0);
        tb[hh][i / Q] = make_ushort4(t2.x, t2.y, 0, 0);
      } else {
        tb[hh][i / Q] = make_ushort4(ih[e0], 0, 0, 0);
      }
    }
  }
}

// load_buckets from a workgroup-uniform base and a 32-bit element offset
// (SGPR base + VGPR offset addressing: no 64-bit address math per load)
template <int E, int KH>
__device__ __forceinline__ void load_buckets_off(const uint16_t* __restrict__ base, unsigned off0, int h0, int nhi,
                                                 int M, int lane, ushort4 (&tb)[KH][(E + 3) / 4]) {
  constexpr int Q = E < 4 ? E : 4;
#pragma unroll
  for (int hh = 0; hh < KH; ++hh) {
    const int h = h0 + hh < nhi ? h0 + hh : nhi - 1;
#pragma unroll
    for (int i = 0; i < E; i += Q) {
      int e0 = elem_index<E>(lane, i);
      e0 = e0 < M ? e0 : 0;
      const unsigned bo = (off0 + (unsigned)(h * M + e0)) * 2u;
      if constexpr (Q == 4) {
        tb[hh][i / Q] = ld_off(reinterpret_cast<const ushort4*>(base), bo);
      } else if constexpr (Q == 2) {
        const ushort2 t2 = ld_off(reinterpret_cast<const ushort2*>(base), bo);
        tb[hh][i / Q] = make_ushort4(t2.x, t2.y, 0, 0);
      } else {
        tb[hh][i / Q] = make_ushort4(ld_off(base, bo), 0, 0, 0);
      }
    }
  }
}

template <typename real, int E, int KH>
__device__ __forceinline__ void gather_buckets(const real* zs, int h0, int nhi,
                                               const ushort4 (&tb)[KH][(E + 3) / 4], real (&v)[E]) {
  constexpr int Q = E < 4 ? E : 4;
  if constexpr (KH * E <= 64) {
    if (h0 + KH <= nhi) {  // uniform: every step of the block exists
      // all KH x E LDS reads issued before the first add: the guarded per-step
      // form below made the compiler wait for each step's reads before the
      // next step's (lgkmcnt(0) per step: 16 LDS latencies in a row at c2)
      real zz[KH][E];
#pragma unroll
      for (int hh = 0; hh < KH; ++hh)
#pragma unroll
        for (int i = 0; i < E; i += Q) {
          const ushort4 r4 = tb[hh][i / Q];
          const unsigned short rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            zz[hh][i + q] = zs[rr[q]];
          }
        }
      if constexpr (KH * E > 16) {
#pragma unroll
        for (int hh = 0; hh < KH; ++hh) {
          const bool neg = __popc(h0 + hh) & 1;  // the same adds in the same (h) order as below
#pragma unroll
          for (int i = 0; i < E; ++i) v[i] += neg ? -zz[hh][i] : zz[hh][i];
        }
      } else {
#pragma unroll
        for (int hh = 0; hh < KH; ++hh) {
          // the same sums in the same (h) order: fma(z, -1, v) is v - z
          // rounded once, as v + (-z) is; one VALU op per element
          const real sg = (__popc(h0 + hh) & 1) ? (real)-1 : (real)1;
#pragma unroll
          for (int i = 0; i < E; ++i) v[i] = fma(zz[hh][i], sg, v[i]);
        }
        // blocks of at most 16 reads (C4 triples: 8 h-steps x 2): software
        // pipeline, 14 reads in flight up front, then one read per fma (the
        // default schedule issued 8, waited them all out, then 8 more): C4
        // single codeword +1.5-2.4 %.  For the 32 reads of a c2 block the
        // default schedule and the select + add form measured faster (c2
        // -0.9 % with the pipeline; -1.5-4 % with the fma form and the
        // precomputed partial-store addresses of the Ab rows)
        constexpr int kPre = KH * E < 14 ? KH * E : 14;
        __builtin_amdgcn_sched_group_barrier(0x100, kPre, 0);  // DS read
#pragma unroll
        for (int k = kPre; k < KH * E; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);    // VALU
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x002, kPre, 0);
      }
      return;
    }
  }
#pragma unroll
  for (int hh = 0; hh < KH; ++hh) {
    if (h0 + hh < nhi) {
      const bool neg = __popc(h0 + hh) & 1;  // sgn(h): the high index bits of w-M+c are all ones
#pragma unroll
      for (int i = 0; i < E; i += Q) {
        const ushort4 r4 = tb[hh][i / Q];
        const unsigned short rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const real zz = zs[rr[q]];
          v[i + q] += neg ? -zz : zz;
        }
      }
    }
  }
}

// One workgroup = 4 wavefronts = 4 consecutive sections of one codeword
// (blockIdx.y).  Per wave: v = bucket gather of z (LDS), M-point FWHT,
// denoise, FWHT of the new beta (the Ab operand), staged to LDS.  Then the
// workgroup gathers its 4 sections' contributions to every row of Ab into
// abp[b][g][:].  Loads independent of z (bucket table, previous beta) are
// issued before the z barrier so their latency overlaps.
#ifdef SA_STAMPS
// [wave][stamp]: every wave of the stamped workgroup records its own phases
__device__ unsigned long long g_stamps[16 * 16];
#ifndef SA_STAMP_BLOCK
#define SA_STAMP_BLOCK 0  // the workgroup whose phases are stamped (-DSA_STAMP_BLOCK=gridDim.x-1: the last)
#endif
#define STAMP(i)                                                                        \
  do {                                                                                  \
    if (blockIdx.x == SA_STAMP_BLOCK && blockIdx.y == 0 && (threadIdx.x & 63) == 0) {   \
      __builtin_amdgcn_sched_barrier(0);                                                \
      unsigned long long _t;                                                            \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");       \
      g_stamps[(threadIdx.x >> 6) * 16 + (i)] = _t;                                     \
      __builtin_amdgcn_sched_barrier(0);                                                \
    }                                                                                   \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#endif

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
      const real bb = denoise_section<real, E>(v, bprev, blo, lane, M, cl, tau2, a.sqrt_n, owner);
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
      const real bb = denoise_section<real, E>(v, bprev, blo, lane, M, cl, tau2, a.sqrt_n, owner);
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
// ---------------------------------------------------------------------------
// Batched section kernel (B codewords share the operator)
// ---------------------------------------------------------------------------
// One workgroup = 4 wavefronts x CB codewords, sweeping kSG = 16 consecutive
// sections in 4 rounds of 4.  z of the CB codewords is staged interleaved
// ([row][CB]) so one LDS gather fetches the same row of every codeword
// (ds_read_b64 for CB = 2 fp32); the staged T_l = H_M beta_l are interleaved
// the same way ([section][k][CB]); the Ab contributions of all 16 sections are
// accumulated per row in LDS and written once (G = L / 16 partials).  The
// bucket / Ab tables are read once per workgroup for CB codewords, and all
// workgroups of a section group are placed on one XCD (blockIdx % 8 labels
// the XCD) so the group's tables stay in that XCD's L2.
constexpr int kSG = 16;  // fwd table padding (sections)
// table bytes of the section groups one XCD works on at a time (SecArgs::gpx).
// C4 binary32 k_secb HBM bytes per launch (PMC, round 4; the 1.7 / 0.9 MB
// points on an intermediate build with an L2-budget switch since removed):
// one pass (6 groups, 4.7 MB) 1.715 GB; 2.5 MB -> 2 x 3 groups 1.495 GB;
// 1.7 MB -> 3 x 2 groups 1.514 GB; 0.9 MB -> 6 x 1 group 1.711 GB (every
// pass re-reads z)
constexpr size_t kSecbL2 = (size_t)5 << 19;  // 2.5 MB of the 4 MB L2
// sections (waves) per batched workgroup: 8 (two workgroups per CU), or 16
// (one per CU) where the wider workgroup's LDS holds a larger codeword chunk
// (sa_ctx::WB, chosen at context creation)
constexpr int kWB = 8, kWB16 = 16;
// zero rows after z in the batched kernel's LDS image (empty bucket slots read
// them; 16, one per 16-byte bank group: build_invb)
constexpr int kInvbZeroRows = 16;

template <typename real, int CB>
struct cbvec;
template <> struct cbvec<float, 1> { using t = float; };
template <> struct cbvec<float, 2> { using t = float2; };
template <> struct cbvec<float, 4> { using t = float4; };
template <> struct cbvec<double, 1> { using t = double; };
template <> struct cbvec<double, 2> { using t = double2; };

template <typename real, int CB>
__device__ __forceinline__ void vload(const real* p, real (&o)[CB]) {
  using V = typename cbvec<real, CB>::t;
  const V t = *reinterpret_cast<const V*>(p);
  if constexpr (CB == 1) {
    o[0] = t;
  } else if constexpr (CB == 2) {
    o[0] = t.x; o[1] = t.y;
  } else {
    o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = t.w;
  }
}
template <typename real, int CB>
__device__ __forceinline__ void vstore(real* p, const real (&o)[CB]) {
  using V = typename cbvec<real, CB>::t;
  V t;
  if constexpr (CB == 1) {
    t = o[0];
  } else if constexpr (CB == 2) {
    t.x = o[0]; t.y = o[1];
  } else {
    t.x = o[0]; t.y = o[1]; t.z = o[2]; t.w = o[3];
  }
  *reinterpret_cast<V*>(p) = t;
}

// LDS byte offset of the 16-bit row index in half `HALF` of w, scaled by
// 2^SH (the [row][CB] element size): one SDWA VALU op (word select + shift).
template <int SH, int HALF>
__device__ __forceinline__ unsigned sdwa_shl16(unsigned w) {
  unsigned r;
  if constexpr (HALF == 0)
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
        : "=v"(r) : "v"(w), "i"(SH));
  else
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
        : "=v"(r) : "v"(w), "i"(SH));
  return r;
}

template <int N>
constexpr int ilog2c() { return N <= 1 ? 0 : 1 + ilog2c<N / 2>(); }

// One h-step of the bucket gather for E >= 4 (Q = 4): the wave's 4*NQ
// bucket rows are turned into LDS addresses, all E gathers are issued, then
// v[c][i] += sgn(h) * z[row][c] as fmas with a wave-uniform sign.
template <typename real, int E, int CB>
__device__ __forceinline__ void gather_step4(const unsigned char* zsb, const ushort4 (&t)[(E + 3) / 4],
                                             real sg, real (&v)[CB][E]) {
  constexpr int SH = ilog2c<CB * (int)sizeof(real)>();
  unsigned ad[E];
#pragma unroll
  for (int j = 0; j < E / 4; ++j) {
    const uint2 w = *reinterpret_cast<const uint2*>(&t[j]);
    ad[4 * j + 0] = sdwa_shl16<SH, 0>(w.x);
    ad[4 * j + 1] = sdwa_shl16<SH, 1>(w.x);
    ad[4 * j + 2] = sdwa_shl16<SH, 0>(w.y);
    ad[4 * j + 3] = sdwa_shl16<SH, 1>(w.y);
  }
  // zsb is the start of the dynamic LDS region, which is LDS address 0 in
  // this kernel (it declares no static LDS: checked on the host at context
  // creation), so the scaled row index is the LDS address itself.
  (void)zsb;
  using V = real __attribute__((ext_vector_type(CB)));
  using lds_v = __attribute__((address_space(3))) const V;
  real zz[E][CB];
#ifdef SA_DIAG_GATHER_NOCONF
#pragma unroll
  for (int i = 0; i < E; ++i) ad[i] = (((threadIdx.x & 15) + 16 * i) << SH) + (ad[i] & 0);
#endif
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const V x = *reinterpret_cast<lds_v*>((size_t)ad[i]);
#pragma unroll
    for (int c = 0; c < CB; ++c) zz[i][c] = x[c];
  }
#pragma unroll
  for (int i = 0; i < E; ++i)
#pragma unroll
    for (int c = 0; c < CB; ++c) v[c][i] = fma(zz[i][c], sg, v[c][i]);
}

// Build-time switches of k_secb (A/B builds; the defaults are the measured
// best, every combination bit-identical, scripts/run_r05h.sh):
//   SA_F64_KH      binary64 bucket h-steps in flight (2 once LATE_B frees the registers)
//   SA_F64_LATE_F  binary64: the first Ab-table rows loaded after the gather
//   SA_F64_LATE_B  binary64: codeword 0's previous estimate loaded after the gather
//   SA_F64_SLAST   binary64: tau_{t-1} through the scalar cache (no VGPRs, no
//                  extra round trip after tau)
//   SA_GSIGN       the gather's sign a constant of each half of the bank-aware
//                  step order (two loops) instead of selected per step
//   SA_F32_KH      binary32 (CB = 4 or E = 16) bucket h-steps in flight
//   SA_F32_LATE_F / SA_F32_LATE_B  binary32 (CB = 4): the Ab-table rows / the
//                  previous estimate after the gather (C3 +1.5 %, C4 neutral;
//                  with the freed registers a third table buffer (loads two
//                  blocks ahead) measured -2 %, KH = 4 -5 %: spills)
// Round 5, interleaved A/B x2: binary32 C3 14.55 k -> 14.96 k, C4 6.93 k ->
// 7.12 k cw/s (SA_GSIGN); binary64 C3 7.03 k -> 7.33 k, C4 3.22 k -> 3.36 k
// (all three; SA_GSIGN alone 7.21 k / 3.32 k); then LATE_B with KH = 2: C3
// fp64 7.39 k -> 7.46 k, C4 fp64 3.38 k -> 3.46 k (LATE_B alone: neutral).
#ifndef SA_F64_KH
#define SA_F64_KH 2
#endif
#ifndef SA_F64_LATE_F
#define SA_F64_LATE_F 1
#endif
#ifndef SA_F64_SLAST
#define SA_F64_SLAST 1
#endif
#ifndef SA_GSIGN
#define SA_GSIGN 1
#endif
#ifndef SA_F64_LATE_B
#define SA_F64_LATE_B 1
#endif
#ifndef SA_F32_KH
#define SA_F32_KH 2
#endif
//   SA_FWHT_PAIR   binary32: the section transforms of codeword pairs interleaved
//   SA_SECB_COMPACT  the bank-aware halves' occupied slots in their first steps, the rest skipped
#ifndef SA_SECB_COMPACT
#define SA_SECB_COMPACT 1
#endif
//   SA_F64_EXPTAB  binary64 denoiser exp from a 64-entry LDS table (exp_neg_tab)
#ifndef SA_F64_EXPTAB
#define SA_F64_EXPTAB 1
#endif
#ifndef SA_GATHER_PRIO
#define SA_GATHER_PRIO 3
#endif
#ifndef SA_ROWC_U12
#define SA_ROWC_U12 1
#endif
#ifndef SA_FWHT_PAIR
#define SA_FWHT_PAIR 1
#endif
#ifndef SA_F32_LATE_F
#define SA_F32_LATE_F 1
#endif
#ifndef SA_F32_LATE_B
#define SA_F32_LATE_B 1
#endif
template <typename real, int E, int CB, int W, bool ZIL = false>
__global__ void __launch_bounds__(W * 64, (E <= 8 ? 4 : 1)) k_secb(SecArgs<real> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NT = W * 64;
  constexpr int NQ = (E + 3) / 4;
  // binary64: fewer loads in flight so a wave fits 128 VGPRs (two workgroups per CU)
  constexpr bool F64 = sizeof(real) == 8;
  // bucket h-steps with table loads in flight together (binary64: SA_F64_KH)
  constexpr int KH = F64 ? SA_F64_KH : ((E >= 16 || CB >= 4) ? SA_F32_KH : 4);
  // binary64: the first Ab-table rows loaded after the gather instead of with
  // the first loads (their registers are then free for the table stream)
  constexpr bool LATE_F = F64 ? SA_F64_LATE_F : SA_F32_LATE_F;
  // binary64: the previous estimate of codeword 0 loaded after the gather too
  constexpr bool LATE_B = (F64 ? SA_F64_LATE_B : SA_F32_LATE_B) && !(CB <= 2 && !F64);
  // rows per thread whose Ab-table loads are in flight together (one with 16
  // sections at CB = 4: their 4 table words per row already fill the registers)
  constexpr int KR = (CB >= 4 || F64) ? (W > 8 && (CB >= 4 || F64) ? 1 : 2) : 3;
  constexpr bool PB = CB <= 2 && !F64;           // prefetch the previous beta with the first loads
  constexpr int W4 = W / 4;             // 4-section table groups per workgroup
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = a.M, n = a.n;
  const size_t LM = (size_t)a.L * M;
  const int mlanes = M < 64 ? M : 64;
  // SGN (binary32, E >= 2): both transforms run fwht_wave_sgn, which leaves
  // slot k (lane L) with (-1)^<k,m> = sgl times the transform, m the two
  // index bits on lane bits 0 / 1.  Cancelled exactly with no table change:
  // the bucket gather and beta use quad-mirrored section positions (lane L
  // holds index k ^ m: lane L ^ 3's) and the gathered input is multiplied by
  // sgl.  With H(x(. ^ m))[k] = (-1)^<k,m> (Hx)[k] the first transform then
  // yields Az at the mirrored positions with no sign (the denoiser and beta
  // stay in that layout) and the second, fed mirrored beta, T = H beta in
  // natural positions with no sign: the same values, bit for bit, as
  // fwht_wave on the natural layout.
  constexpr bool SGN = sizeof(real) == 4 && E >= 2;
  const int lpos = SGN ? (lane ^ 3) : lane;  // section positions of this lane
  const real sgl = (SGN && (__popc(lane & 3) & 1)) ? (real)-1 : (real)1;
  const float s1 = (lane & 1) ? -1.f : 1.f, s2 = (lane & 2) ? -1.f : 1.f;
  STAMP(0);

  // XCD-grouped work mapping (speed only: any placement is correct)
  int g, chunk;
  {
    const int bid = blockIdx.x, total = a.G * a.NC;
    if ((a.G & 7) == 0 && (total & 7) == 0) {
      const int x = bid & 7, j = bid >> 3;
      // the XCD's G/8 section groups in passes of gpx groups, the groups of
      // a pass fastest: the workgroups in flight on one XCD cover the pass's
      // tables and a few codeword chunks' z, which stay in its L2 together
      // (C4: 6 groups' tables, 4.7 MB, overflowed the 4 MB L2; two passes of 3)
      const int gx = a.G >> 3;
      int jj = j, g0 = 0, gp = a.gpx < gx ? a.gpx : gx;
      while (jj >= gp * a.NC) {  // whole passes before this item (at most G / 8 steps)
        jj -= gp * a.NC;
        g0 += gp;
        gp = gx - g0 < gp ? gx - g0 : gp;
      }
      g = (g0 + jj % gp) * 8 + x;
      chunk = jj / gp;
    } else {
      g = bid / a.NC;
      chunk = bid % a.NC;
    }
  }
  int bc[CB];
  bool valid[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int b = chunk * CB + c;
    valid[c] = b < a.B;
    bc[c] = valid[c] ? b : a.B - 1;
  }
  const int l = g * W + wv;
  const bool have = l < a.L;
  const int lc = have ? l : a.L - 1;

  // z ([n+1][CB], read by the bucket gather) and T ([W][M][CB], read by the
  // Ab gather) are never live together: they share one LDS region.
  real* zs = reinterpret_cast<real*>(smem);
  real* ts = zs;
  // z rows, then kInvbZeroRows zero rows (empty bucket slots; one per 16-B bank group)
  const int zslots = (((n + kInvbZeroRows) * CB * (int)sizeof(real) + 15) / 16 * 16) / (int)sizeof(real);
  const int region = zslots > W * M * CB ? zslots : W * M * CB;
  real* bbw = zs + region;                   // [W][CB]
  // binary64 (SA_F64_EXPTAB): the exp table, 64 doubles after bbw
  constexpr bool XT = F64 && SA_F64_EXPTAB;
  double* xtab = reinterpret_cast<double*>(bbw + W * CB);
  if constexpr (XT) {
    if (tid < 64) xtab[tid] = c_exp2_64[tid];  // read after the z barrier
  }

  // codeword-interleaved z (a.zil: [NC][n][CB], 16-byte rows): this chunk's
  // rows straight into LDS by LDS-DMA (1 KB per wave instruction), issued
  // before anything else; no register staging, no ds_write, no second pass
  // (a template parameter: the two z paths in one kernel cost the binary64
  // instantiations 32 bytes more scratch)
  static_assert(!ZIL || CB * sizeof(real) == 16, "codeword-interleaved rows are 16 bytes");
  constexpr bool zil = ZIL;
  if (zil) {
    const char* zsrc = reinterpret_cast<const char*>(a.z) + (size_t)chunk * n * CB * sizeof(real);
    const int nbytes = n * CB * (int)sizeof(real);
    for (int ch = wv; ch * 1024 < nbytes; ch += W) {
      const int off = ch * 1024 + lane * 16;
      if (off + 16 <= nbytes)  // rows are 16 bytes: whole rows only
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(zsrc + off),
                                         (__attribute__((address_space(3))) void*)((char*)zs + ch * 1024), 16, 0, 0);
    }
  }
  // ---- every load independent of z in flight together ---------------------
  // the z^2 partials of the CB codewords first: tau waits for these alone
  ZZParts<real, F64 ? 2 : 3> zzc[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) zzc[c].issue(a.zzp + (size_t)bc[c] * a.NZ, a.NZ, lane);
  // tau_{t-1} of the CB codewords (the exact-tau stop) right behind them: a
  // load issued after the table loads would make the stop test wait for all
  // of them (vmcnt retires in order), one more round trip per codeword
  // (binary64 keeps the late load: at 128 VGPRs the early one costs spills)
  real lastv[CB];
  if constexpr (!F64) {
#pragma unroll
    for (int c = 0; c < CB; ++c) lastv[c] = a.t > 0 ? ld_vmem(a.tau + (size_t)bc[c] * a.T1 + a.t - 1) : (real)0;
  } else if constexpr (SA_F64_SLAST) {
    // binary64: through the scalar cache, no VGPRs (tau_{t-1} was written by the previous launch)
#pragma unroll
    for (int c = 0; c < CB; ++c) lastv[c] = a.t > 0 ? ld_smem(a.tau + (size_t)bc[c] * a.T1 + a.t - 1) : (real)0;
  }
  // z rows of the CB codewords (first pass of the staging loop)
  constexpr int KZ = 4;
  real zr[KZ][CB];
  // uniform codeword bases + 32-bit unsigned row offsets (SGPR-base loads)
  const real* zc[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) zc[c] = a.z + (size_t)bc[c] * n;
  if (!zil) {
#pragma unroll
    for (int u = 0; u < KZ; ++u) {
      const int r = u * NT + tid;
#pragma unroll
      for (int c = 0; c < CB; ++c) zr[u][c] = ld_off(zc[c], (unsigned)(r < n ? r : 0) * (unsigned)sizeof(real));
    }
  }
  // the bank-aware step order (build_invb: sign +1 steps first) or h order
  const bool banked = a.invb != nullptr;
  // binary32: a workgroup-uniform base + this wave's 32-bit offset (SGPR-base
  // loads; binary64 keeps the per-wave pointer, its scratch grew otherwise)
  const uint16_t* il = (banked ? a.invb : a.inv) + (size_t)lc * a.w;
  auto load_tb = [&](int h0, ushort4 (&dst)[KH][NQ]) {
    if constexpr (ZIL && E % 4 == 0) {
      // lane-major table: this lane's NQ quads of step h in one run of E * 2 bytes
      const uint16_t* base = a.invl + (size_t)lc * a.nhi * 64 * E + (size_t)lane * E;
#pragma unroll
      for (int hh = 0; hh < KH; ++hh) {
        const int h = h0 + hh < a.nhi ? h0 + hh : a.nhi - 1;
#pragma unroll
        for (int j = 0; j < NQ; j += 2) {
          if (j + 1 < NQ) {
            const uint4 q = *reinterpret_cast<const uint4*>(base + (size_t)h * 64 * E + 4 * j);
            dst[hh][j] = *reinterpret_cast<const ushort4*>(&q.x);
            dst[hh][j + 1] = *reinterpret_cast<const ushort4*>(&q.z);
          } else {
            dst[hh][j] = *reinterpret_cast<const ushort4*>(base + (size_t)h * 64 * E + 4 * j);
          }
        }
      }
    } else if constexpr (F64)
      load_buckets<E, KH>(il, h0, a.nhi, M, lpos, dst);
    else
      load_buckets_off<E, KH>((banked ? a.invb : a.inv) + (size_t)g * W * a.w, (unsigned)((lc - g * W) * a.w), h0,
                              a.nhi, M, lpos, dst);
  };
  ushort4 tb[KH][NQ];
  load_tb(0, tb);
  // previous beta: all CB codewords up front when registers allow (CB <= 2),
  // else codeword 0 now and codeword c+1 while c is denoised (PB false)
  real bprev[PB ? CB : 2][E];
  if constexpr (PB) {
#pragma unroll
    for (int c = 0; c < CB; ++c)
      load_section_nt<real, E>(a.beta + (size_t)bc[c] * LM + (size_t)lc * M, bprev[c], lpos, M);
  } else if constexpr (!LATE_B) {
    load_section_nt<real, E>(a.beta + (size_t)bc[0] * LM + (size_t)lc * M, bprev[0], lpos, M);
  }
  real cl[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) cl[c] = ld_vmem(a.c + (size_t)bc[c] * a.cst + lc);
  // the Ab table rows: [W4][npad] of this group (rows past npad: whole waves,
  // every lane reading row 0, a broadcast)
  const int npad = (n + 63) & ~63;
  const ushort4* fw = a.fwdb + (size_t)g * W4 * npad;
  ushort4 f[KR][W4];
  auto load_f = [&]() {
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      const int r = u * NT + tid;
#pragma unroll
      for (int q = 0; q < W4; ++q) f[u][q] = fw[(size_t)q * npad + (r < npad ? r : 0)];
    }
  };
  if constexpr (!LATE_F) load_f();
  // tau per codeword (sparc_ldpc.py:203-209)
  bool live[CB];
  bool any = false;
  real tau2[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const real tau = zzc[c].tau(a.zzp + (size_t)bc[c] * a.NZ, a.NZ, n);
    if constexpr (F64 && !SA_F64_SLAST) lastv[c] = a.t > 0 ? ld_vmem(a.tau + (size_t)bc[c] * a.T1 + a.t - 1) : (real)0;
    const bool stop = a.early_stop && (tau == lastv[c]);
    if (valid[c] && g == 0 && tid == 0) {
      a.tau[(size_t)bc[c] * a.T1 + a.t] = tau;
      if (stop && a.iters[bc[c]] < 0) a.iters[bc[c]] = a.t;
    }
    live[c] = valid[c] && !stop;
    any |= live[c];
    tau2[c] = tau * tau;
  }
  if (!any) {  // uniform
    if (zil) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA write may outlive the workgroup
    return;
  }
  STAMP(1);

  // ---- z -> LDS interleaved [row][CB] ------------------------------------
  if (zil) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed (the barrier: every wave's)
  for (int r0 = 0; r0 < (zil ? 0 : n); r0 += KZ * NT) {
#pragma unroll
    for (int u = 0; u < KZ; ++u) {
      const int r = r0 + u * NT + tid;
      if (r < n) vstore<real, CB>(zs + (size_t)r * CB, zr[u]);
    }
    if (r0 + KZ * NT < n) {
#pragma unroll
      for (int u = 0; u < KZ; ++u) {
        const int r = r0 + KZ * NT + u * NT + tid;
#pragma unroll
        for (int c = 0; c < CB; ++c) zr[u][c] = ld_off(zc[c], (unsigned)(r < n ? r : 0) * (unsigned)sizeof(real));
      }
    }
  }
  if (tid < kInvbZeroRows * CB) zs[(size_t)n * CB + tid] = 0;
  __syncthreads();
  STAMP(2);

  // ---- bucket gather of the CB codewords (one LDS access per row index) ----
  // (SA_GATHER_PRIO: the gather at a raised wave priority, so every wave's
  // latency-bound gather runs before the older waves' VALU-bound denoise)
  if (SA_GATHER_PRIO) __builtin_amdgcn_s_setprio(SA_GATHER_PRIO);
  real v[CB][E];
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int i = 0; i < E; ++i) v[c][i] = 0;
  {
    constexpr int Q = E < 4 ? E : 4;
    // one block of KH h-steps; sgf >= 0: every step of the block has that
    // sign (the bank-aware order's halves), else sgn(h) per step
    // hn: the next block's first step (< 0: none)
    auto block = [&](int h0, int sgf, int hn) {
      ushort4 tn[KH][NQ];
      const bool more = hn >= 0;
      if (more) load_tb(hn, tn);
#pragma unroll
      for (int hh = 0; hh < KH; ++hh) {
        if (h0 + hh < a.nhi) {
          // sgn(h): the high index bits of w-M+c are all ones; in the bank-aware
          // order the slots of sign -1 are the second half of the steps
          const bool neg = sgf >= 0 ? sgf == 1 : (banked ? (h0 + hh >= (a.nhi >> 1)) : (__popc(h0 + hh) & 1));
          const real sg = neg ? -sgl : sgl;
          if constexpr (E >= 4) {
            gather_step4<real, E, CB>(reinterpret_cast<const unsigned char*>(zs), tb[hh], sg, v);
          } else {
            const ushort4 r4 = tb[hh][0];
            const unsigned short rr4[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
            for (int q = 0; q < Q; ++q) {
              real zz[CB];
              vload<real, CB>(zs + (size_t)rr4[q] * CB, zz);
#pragma unroll
              for (int c = 0; c < CB; ++c) v[c][q] = fma(zz[c], sg, v[c][q]);
            }
          }
        }
      }
      if (more) {
#pragma unroll
        for (int hh = 0; hh < KH; ++hh)
#pragma unroll
          for (int j = 0; j < NQ; ++j) tb[hh][j] = tn[hh][j];
      }
    };
    const int half = a.nhi >> 1;
    // (the 16-byte-row configurations up to M = 512: elsewhere the duplicated
    // loop body spilled)
    constexpr bool GS = SA_GSIGN && CB * sizeof(real) == 16 && E <= 8;
    if (GS && banked && half > 0 && half % KH == 0) {
      // the bank-aware order: the +1 steps, then the -1 steps; the sign is a
      // constant of each loop (the same fmas with the same signs).  Each half
      // holds its occupied slots in its first s0 / s1 steps (build_invb: the
      // section's largest column count, a multiple of KH): the rest, empty
      // for every column, is skipped
      int s0 = half, s1 = half;
      if (a.hs) {
        const unsigned v = a.hs[__builtin_amdgcn_readfirstlane(lc)];
        s0 = (int)(v & 0xffffu);
        s1 = (int)(v >> 16);
      }
      for (int h0 = 0; h0 < s0; h0 += KH) block(h0, 0, h0 + KH < s0 ? h0 + KH : (s1 > 0 ? half : -1));
      for (int h0 = half; h0 < half + s1; h0 += KH) block(h0, 1, h0 + KH < half + s1 ? h0 + KH : -1);
    } else {
      for (int h0 = 0; h0 < a.nhi; h0 += KH) block(h0, -1, h0 + KH < a.nhi ? h0 + KH : -1);
    }
  }
  if constexpr (LATE_F) load_f();
  if constexpr (LATE_B) load_section_nt<real, E>(a.beta + (size_t)bc[0] * LM + (size_t)lc * M, bprev[0], lpos, M);
  if (SA_GATHER_PRIO) __builtin_amdgcn_s_setprio(0);
  STAMP(3);
  // denoiser eta (sparc_ldpc.py:213-219, as denoise_section) of the CB
  // codewords with their section max / sums reduced together (wave_reduce_cb)
  const int ml = E >= 2 ? 64 : mlanes;  // E >= 2: M = 64 E fills every lane
  auto fwht_sec = [&](real (&x)[E]) {
    if constexpr (SGN) fwht_wave_sgn<E>(x, s1, s2);
    else fwht_wave<real, E>(x, lane, ml);
  };
  // binary32 codeword pairs: the two transforms of a pair interleaved
  constexpr bool FP = SA_FWHT_PAIR && SGN && CB % 2 == 0 && E >= 2;
  auto fwht_all = [&]() {
    if constexpr (FP) {
#pragma unroll
      for (int c = 0; c < CB; c += 2) fwht_wave_sgn_pair<E>(v[c], v[c + 1], s1, s2);
    }
  };
  fwht_all();
  const real inv_sn = (real)1 / a.sqrt_n;
  real bbl[CB], mx[CB], S[CB], S2[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    if constexpr (!PB) {
      if (c + 1 < CB)
        load_section_nt<real, E>(a.beta + (size_t)bc[c + 1] * LM + (size_t)lc * M, bprev[(c + 1) & 1], lpos, M);
    }
    if constexpr (!FP) fwht_sec(v[c]);
    const real k = cl[c] / tau2[c];
    real m = neg_inf<real>();
#pragma unroll
    for (int i = 0; i < E; ++i) {
      // :213, :215.  The exponent argument below, u - max, is contracted to
      // fma(s, k, -max) (one rounding where the reference rounds u first:
      // <= 1 ulp of u, inside the parity bounds; 4 % faster at c3)
      const real u = fma(v[c][i], inv_sn, bprev[PB ? c : (c & 1)][i]) * k;
      v[c][i] = (E >= 2 || elem_index<E>(lane, i) < M) ? u : neg_inf<real>();
      m = max_raw(m, v[c][i]);  // one v_max (operands finite or -inf)
    }
    mx[c] = m;
  }
  wave_reduce_cb<true, CB>(mx);  // :216 (per section)
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    real s = 0, s2 = 0;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if constexpr (XT)
        v[c][i] = (real)exp_neg_tab((double)(v[c][i] - mx[c]), xtab);  // :217
      else
        v[c][i] = dexp<real>(v[c][i] - mx[c]);  // :217; exp(-inf) = 0 on idle lanes
      s += v[c][i];
      s2 += v[c][i] * v[c][i];
    }
    S[c] = s;
    S2[c] = s2;
  }
  wave_reduce_cb<false, CB>(S);   // :218
  wave_reduce_cb<false, CB>(S2);  // sum(beta^2)
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const real scale = cl[c] / S[c];  // :219
#pragma unroll
    for (int i = 0; i < E; ++i) v[c][i] *= scale;
    if (have && live[c]) store_section_nt<real, E>(a.beta + (size_t)bc[c] * LM + (size_t)lc * M, v[c], lpos, M);
    if (have) {
      bbl[c] = S2[c] * scale * scale;
      if constexpr (!FP) fwht_sec(v[c]);  // T_l = H_M beta_l (natural positions)
    } else {
      bbl[c] = 0;
#pragma unroll
      for (int i = 0; i < E; ++i) v[c][i] = 0;
    }
  }
  if (have) fwht_all();  // (FP) the T transforms of the codeword pairs
  STAMP(4);
  __syncthreads();  // every wave is done with z before T overwrites it
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = elem_index<E>(lane, i);
    if (e < M) {
      real o[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) o[c] = v[c][i];
      // staged at t_pos(e): consecutive lanes write consecutive rows (in
      // natural order a lane's Q elements are adjacent, and the store of one
      // register by 64 lanes has a Q-row stride: a Q-way bank conflict)
      constexpr int Q = E < 4 ? E : 4;
      vstore<real, CB>(ts + ((size_t)wv * M + (i / Q) * 64 * Q + (i % Q) * 64 + lane) * CB, o);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < CB; ++c) bbw[wv * CB + c] = bbl[c];
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    if (tid == c && live[c]) {
      real t = 0;
      for (int w2 = 0; w2 < W; ++w2) t += bbw[w2 * CB + c];
      a.bbp[(size_t)bc[c] * a.G + g] = t;
    }
  }
  STAMP(5);
  // ---- Ab partial of the workgroup's W sections for every row ---------------
  // (each row's W table entries in its own bank-aware order, build_fwdb: the
  // entry holds the staged T element s * M + k itself)
  constexpr int SHB = ilog2c<CB * (int)sizeof(real)>();      // T element k -> byte k << SHB
  for (int r0 = 0; r0 < n; r0 += KR * NT) {
    ushort4 fn[KR][W4];
    const bool more = r0 + KR * NT < n;
    if (more) {
#pragma unroll
      for (int u = 0; u < KR; ++u) {
        const int r = r0 + KR * NT + u * NT + tid;
#pragma unroll
        for (int q = 0; q < W4; ++q) fn[u][q] = fw[(size_t)q * npad + (r < npad ? r : 0)];
      }
    }
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      const int r = r0 + u * NT + tid;
      real acc[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) acc[c] = 0;
#pragma unroll
      for (int q = 0; q < W4; ++q) {
        const uint2 w = *reinterpret_cast<const uint2*>(&f[u][q]);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          // entry = k | sign << 15: T element k of section q*4+s4, sign -> +-1.0
          const unsigned wd = s4 < 2 ? w.x : w.y;
          const bool up = s4 & 1;
          real t[CB];
          real sg;
          if constexpr (sizeof(real) == 4) {
            // binary32: k and the LDS byte address in two ops, the sign
            // bit ORed into 1.0f (one op for the upper half-word)
            const unsigned k = up ? __builtin_amdgcn_ubfe(wd, 16, 15) : (wd & 0x7fffu);
            const unsigned sb = (up ? wd : wd << 16) & 0x80000000u;
            sg = __uint_as_float(sb | 0x3f800000u);
            using V = real __attribute__((ext_vector_type(CB)));
            using lds_v = __attribute__((address_space(3))) const V;
            // ts is LDS address 0 (the dynamic region, no static LDS)
#ifdef SA_DIAG_ROWS_NOCONF
            const V x = *reinterpret_cast<lds_v*>((size_t)((((k >> 9) << 9) + (threadIdx.x & 15)) << SHB));
#else
            const V x = *reinterpret_cast<lds_v*>((size_t)(k << SHB));
#endif
#pragma unroll
            for (int c = 0; c < CB; ++c) t[c] = x[c];
          } else {
            const unsigned hw = up ? wd >> 16 : wd;
            const unsigned k = __builtin_amdgcn_ubfe(hw, 0, 15);
            sg = (hw & 0x8000u) ? (real)-1 : (real)1;
            vload<real, CB>(ts + (size_t)k * CB, t);
          }
#pragma unroll
          for (int c = 0; c < CB; ++c) acc[c] = fma(t[c], sg, acc[c]);
        }
      }
      if (r < n) {
        if (zil) {  // one 16-byte vector of the CB codewords ([NC][G][n][CB])
          using V = real __attribute__((ext_vector_type(CB)));
          V pv;
#pragma unroll
          for (int c = 0; c < CB; ++c) pv[c] = acc[c];
          __builtin_nontemporal_store(pv, reinterpret_cast<V*>(a.abp) + ((size_t)chunk * a.G + g) * n + r);
        } else {
#pragma unroll
          for (int c = 0; c < CB; ++c)
            if (live[c]) st_part(&a.abp[((size_t)bc[c] * a.G + g) * n + r], acc[c]);
        }
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < KR; ++u)
#pragma unroll
        for (int q = 0; q < W4; ++q) f[u][q] = fn[u][q];
    }
  }
#ifdef SA_STAMPS
  STAMP(6);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(7);
#endif
}


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
  int bc[CB];
  bool valid[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int b = chunk * CB + c;
    valid[c] = b < B;
    bc[c] = valid[c] ? b : B - 1;
  }
  // wave 0's operands that do not depend on the partials, loaded with them
  real tau[CB], last[CB], yv[RPL][CB], bbv[CB][2];
  V zo[RPL] = {};
  if (wv == 0) {
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      tau[c] = 1;
      last[c] = 0;
      if (a.mode == ROW_AMP) {
        tau[c] = ld_vmem(a.tau + (size_t)bc[c] * a.T1 + a.t);
        last[c] = a.t > 0 ? ld_vmem(a.tau + (size_t)bc[c] * a.T1 + a.t - 1) : (real)0;
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
constexpr int kRow2Rows = 32;  // one 128-B line of a partial per row block
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
__global__ void __launch_bounds__(256) k_decide(const real* beta, int32_t* idx, int L, int M) {
  const int lane = threadIdx.x & 63;
  const int l = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y;
  if (l >= L) return;
  const real* bl = beta + ((size_t)b * L + l) * M;
  real best = neg_inf<real>();
  int bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = elem_index<E>(lane, i);
    if (e < M) {
      const real x = bl[e];
      if (x > best || (x == best && e < bi)) { best = x; bi = e; }
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const real ob = __shfl_xor(best, m);
    const int oi = __shfl_xor(bi, m);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) idx[(size_t)b * L + l] = bi == 0x7fffffff ? 0 : bi;
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

#include "dense_i8.hip"
#include "dense_mfma.hip"

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

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------

int ilog2(int x) {
  int r = 0;
  while ((1 << r) < x) ++r;
  return r;
}

}  // namespace

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

// Launch of a loop kernel on the context's stream, timed as sa_profile asks
// (plain launch when no profile is running).
template <typename F, typename... Args>
void plaunch(sa_ctx* c, F kernel, dim3 grid, dim3 block, size_t lds, Args... args);

struct sa_ctx {
  Prof* prof = nullptr;
  int L = 0, M = 0, n = 0, w = 0, nhi = 0, backend = 0, prec = 0, device = 0;
  int plan = 0;       // SA_PLAN_* options of sa_create_ex (0: every choice by the built-in rules)
  bool pow2 = true;  // M a power of two (the Hadamard kernels, bit-level glue)
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
};

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

namespace {

size_t rsz(const sa_ctx* c) { return c->prec == SA_PREC_F64 ? 8 : 4; }

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

// ---- int8 matrix-core dense path (dense_i8.hip) -------------------------
constexpr int kI8MinB = 4;    // batches at least this large take the GEMM path
constexpr int kI8MaxS = 16;   // K splits of the A beta GEMM (its Ab partials)

bool use_i8(const sa_ctx* c, int B) {
  return c->backend == SA_BACKEND_DENSE && B >= kI8MinB;
}

// the dense backends: a materialised n x (L*M) matrix streamed by GEMVs
// (the Hadamard design's, or a caller's own: SA_BACKEND_MATRIX)
bool is_dense(const sa_ctx* c) { return c->backend == SA_BACKEND_DENSE || c->backend == SA_BACKEND_MATRIX; }

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
  return a;
}

// Row splits for small batches: enough workgroups to cover every CU.
int row_splits(const sa_ctx* c, int B) {
  const int wgs = c->G * B;
  int rs = (c->n_cus + wgs - 1) / wgs;
  return rs < 1 ? 1 : (rs > 4 ? 4 : rs);
}

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

bool zil_for(const sa_ctx* c, int B);

// Batched section kernel: grid = Gb groups x ceil(B / CB) chunks (1-D, XCD-grouped).
template <typename real, int E, int CB>
void launch_secb_e(sa_ctx* c, int B, SecArgs<real> a) {
  a.G = c->Gb;
  a.B = B;
  a.NC = (B + CB - 1) / CB;
  a.zil = zil_for(c, B) ? 1 : 0;
  a.gpx = c->gpx;
  if (c->prof) c->prof->begin(c->stream, K_SEC);
  const dim3 grid(c->Gb * a.NC);
  bool done = false;
  if constexpr (CB * sizeof(real) == 16) {
    if (a.zil) {
      if (c->WB == kWB16)
        plaunch(c, k_secb<real, E, CB, kWB16, true>, grid, kWB16 * 64, c->secb_lds, a);
      else
        plaunch(c, k_secb<real, E, CB, kWB, true>, grid, kWB * 64, c->secb_lds, a);
      done = true;
    }
  }
  if (!done) {
    if (c->WB == kWB16)
      plaunch(c, k_secb<real, E, CB, kWB16>, grid, kWB16 * 64, c->secb_lds, a);
    else
      plaunch(c, k_secb<real, E, CB, kWB>, grid, kWB * 64, c->secb_lds, a);
  }
  if (c->prof) c->prof->end(c->stream);
}

template <typename real, int CB>
int launch_secb_cb(sa_ctx* c, int B, const SecArgs<real>& a) {
  switch (c->E) {
    case 1: launch_secb_e<real, 1, CB>(c, B, a); break;
    case 2: launch_secb_e<real, 2, CB>(c, B, a); break;
    case 4: launch_secb_e<real, 4, CB>(c, B, a); break;
    case 8: launch_secb_e<real, 8, CB>(c, B, a); break;
    case 16: launch_secb_e<real, 16, CB>(c, B, a); break;
    default: return fail(SA_ERR_UNSUPPORTED, "batched kernel: M > 1024");
  }
  return SA_OK;
}

template <typename real>
int launch_secb(sa_ctx* c, int B, int t, int es) {
  SecArgs<real> a = sec_args<real>(c, SEC_AMP, t, es);
  int rc;
  if constexpr (sizeof(real) == 4) {
    if (c->CB == 4) {
      rc = launch_secb_cb<real, 4>(c, B, a);
      if (rc) return rc;
      HIP_TRY(hipGetLastError());
      return SA_OK;
    }
  }
  if (c->CB == 2) rc = launch_secb_cb<real, 2>(c, B, a);
  else rc = launch_secb_cb<real, 1>(c, B, a);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  return SA_OK;
}

bool use_batched(const sa_ctx* c, int B) { return c->CB > 0 && B >= 4; }

// Two-waves-per-section kernel for the unbatched path when its G2 x B
// workgroups fill at least half of the CUs (otherwise k_sec's row splits do).
bool use_sec2(const sa_ctx* c, int B) {
  return c->backend == SA_BACKEND_HADAMARD && !use_batched(c, B) && c->G2 > 0 && c->G2 * B * 2 >= c->n_cus;
}

// Ab / beta^2 partials per codeword of the unbatched multi-wave section kernels
int sec2_parts(const sa_ctx* c) { return c->sec3 ? c->G3 : c->G2; }

template <typename real>
int launch_sec2(sa_ctx* c, int B, int t, int es, void* bin, void* bout, int pt = 0) {
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

int row_kind_for(const sa_ctx* c, int B);
// Ab partial layout between the pair / triple kernels and k_row2 (SecArgs::pt):
// rows per row-major block, 0 for the [G][n] layout
int pt_for(const sa_ctx* c, int B, bool sec2) {
  const int rk = row_kind_for(c, B);
  return (sec2 && (c->sec3 || c->sec4) && (rk == 1 || rk == 4) && c->pt_on) ? (rk == 4 ? 16 : kRow2Rows) : 0;
}

template <typename real>
int launch_sec(sa_ctx* c, int B, int mode, int t, int es, void* bin = nullptr, void* bout = nullptr) {
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

// Row kernel for B codewords: k_row2 (32-row blocks) while B * ceil(n/64) <
// 4 CUs, else in binary32 k_rowv<4> (n % 4 == 0) or k_rowv<2> (n even) when
// their blocks cover the CUs twice, else k_row (64 rows).
// The batched decode with z and the Ab partials interleaved by codeword chunk
// (SecArgs::zil, 16-byte rows of CB codewords: binary32 CB = 4, binary64
// CB = 2), row kernel k_rowc.  The default in binary32 (C3 +1.7 %, C4
// +4.7 %) and, since the binary64 k_secb no longer spills (round 4: one
// bucket h-step in flight, 16-byte non-temporal beta), in binary64 too (C3
// 6.30 k -> 6.44 k, C4 3.09-3.12 k -> 3.19 k cw/s; round 3's spilling kernel
// lost 1.6 %); SA_PLAN_NO_ZIL keeps [B][n]
bool zil_for(const sa_ctx* c, int B) {
  const bool on = (c->plan & SA_PLAN_NO_ZIL) ? false : true;
  return on && c->backend == SA_BACKEND_HADAMARD && use_batched(c, B) && c->CB * (int)rsz(c) == 16;
}

int row_kind_for(const sa_ctx* c, int B) {
  if (zil_for(c, B)) return 5;
  if ((long long)B * c->NZ < 4LL * c->n_cus) return (c->row16 && B == 1) ? 4 : 1;
  const bool f32 = c->prec == SA_PREC_F32;
  // 16-byte rows: binary32 n % 4 == 0 (256-row blocks) or binary64 n even (128)
  if (c->n % (f32 ? 4 : 2) == 0 && (long long)B * (f32 ? c->NZ4 : c->NZ2) >= 2LL * c->n_cus) return 2;
  if (f32 && c->n % 2 == 0 && (long long)B * c->NZ2 >= 2LL * c->n_cus) return 3;  // 8-byte rows
  return 0;
}
int nz_for(const sa_ctx* c, int kind) {
  const bool f32 = c->prec == SA_PREC_F32;
  if (kind == 4) return c->NZh;
  if (kind == 5) return c->NZ2;  // k_rowc: 128-row blocks
  return kind == 1 ? c->NZ16 : (kind == 2 ? (f32 ? c->NZ4 : c->NZ2) : (kind == 3 ? c->NZ2 : c->NZ));
}
void pick_row(sa_ctx* c, int B) {
  c->row_kind = row_kind_for(c, B);
  c->nz_cur = nz_for(c, c->row_kind);  // z^2 partials per codeword
}

template <typename real>
int launch_row(sa_ctx* c, int B, int mode, int t, int es, int G, int Gb, int pt = 0, void* zin = nullptr,
               void* zout = nullptr) {
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
    if (SA_ROWC_U12 && (a.G + 3) / 4 > 8 && (a.G + 3) / 4 <= 12)
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
template <typename real = float>
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
bool use_fgemm(const sa_ctx* c, int B) { return c->backend == SA_BACKEND_MATRIX && B >= kFMinB; }

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

// ---- composite sequences (all asynchronous on c->stream) ----------------

// Ab of the batch staged in d_beta -> d_out  (B x n)
template <typename real>
int seq_ab(sa_ctx* c, int B) {
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
  if (is_dense(c)) {
    if ((rc = launch_dense_ab<real>(c, B, 0, 0, 1))) return rc;
    return launch_row<real>(c, B, ROW_ABOUT, 0, 0, c->KS, c->Gd);
  }
  if ((rc = launch_sec<real>(c, B, SEC_AB, 0, 0))) return rc;
  return launch_row<real>(c, B, ROW_ABOUT, 0, 0, c->G, c->G);
}

// Az of the batch staged in d_z -> d_out  (B x L*M)

template <typename real>
int seq_az(sa_ctx* c, int B) {
  if constexpr (sizeof(real) == 4)
    if (use_i8(c, B)) return i8_az(c, B, (float*)c->d_out, (long long)c->L * c->M);
  if (use_fgemm(c, B)) return fgemm_az<real>(c, B, (real*)c->d_out, (long long)c->L * c->M);
  if (is_dense(c)) {
    int rc = launch_dense_az<real>(c, B, 0, 0, 1);
    if (rc) return rc;
    // the RS row-split partials into d_out
    k_dense_az_reduce<real><<<4096, 256, 0, c->stream>>>((const real*)c->d_azp, (real*)c->d_out, c->RS, c->lda,
                                                         (size_t)c->L * c->M, B);
    HIP_TRY(hipGetLastError());
    return SA_OK;
  }
  return launch_sec<real>(c, B, SEC_AZ, 0, 0);
}

// Whole AMP decode of the staged batch: y in d_y, beta0 in d_beta if has_b0.
template <typename real>
int seq_amp(sa_ctx* c, int B, int T, int flags, int has_b0) {
  const int es = (flags & SA_FLAG_NO_EARLY_STOP) ? 0 : 1;
  const bool dense = is_dense(c);
  const bool i8 = use_i8(c, B);
  const bool fg = use_fgemm(c, B);
  const int S8 = i8 ? i8_splits(c, B) : (fg ? fgemm_splits(c, B) : 0);
  const bool batched = !dense && use_batched(c, B);
  const bool sec2 = use_sec2(c, B);
  pick_row(c, B);  // row kernel and its z^2 partial count
  c->zil_last = zil_for(c, B);
  // Ab partials row-block major between the pair / triple kernels and k_row2
  const int pt = pt_for(c, B, sec2);
  // partial counts of the producer of abp (Ab) and bbp (beta^2)
  const int G = (i8 || fg) ? S8 : (dense ? c->KS : (batched ? c->Gb : (sec2 ? sec2_parts(c) : c->G)));
  const int Gb = dense ? c->Gd : (batched ? c->Gb : (sec2 ? sec2_parts(c) : c->G));
  int rc;
  k_fill32<<<(B + 255) / 256, 256, 0, c->stream>>>((uint32_t*)c->d_iters, 0xffffffffu, (size_t)B);
  if (has_b0) {
    if (i8) {
      if ((rc = i8_ab_any(c, B, S8))) return rc;
      if ((rc = launch_row<real>(c, B, ROW_INIT, 0, 0, S8, c->Gd))) return rc;
    } else if (fg) {
      if ((rc = fgemm_ab<real>(c, B, S8))) return rc;
      if ((rc = launch_row<real>(c, B, ROW_INIT, 0, 0, S8, c->Gd))) return rc;
    } else if (dense) {
      if ((rc = launch_dense_ab<real>(c, B, 0, 0, 1))) return rc;
      if ((rc = launch_row<real>(c, B, ROW_INIT, 0, 0, c->KS, c->Gd))) return rc;
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
    if (i8) {
      // z -> digit planes -> Az GEMM (into the dense Az buffer, one partial)
      // -> denoiser (+ beta digit planes) -> A beta GEMM (S8 partials)
      if ((rc = i8_az(c, B, (float*)c->d_azp, (long long)c->lda))) return rc;
      if ((rc = launch_dense_den(c, B, t, es, true))) return rc;
      if ((rc = launch_gemm_i8<kI8NPB>(c, B, c->d_bq, c->LMp8, c->d_A8, c->np8, c->n, (float*)c->d_abp,
                               (long long)S8 * c->n, c->n, S8, c->d_bfix + 1, 0, K_DAB)))
        return rc;
    } else if (fg) {
      // z -> Az GEMM (one partial) -> denoiser -> A beta GEMM (S8 partials);
      // the GEMMs skip nothing for a stopped codeword: the row kernel keeps
      // its residual and the denoiser its estimate
      if ((rc = fgemm_az<real>(c, B, (real*)c->d_azp, (long long)c->lda))) return rc;
      if ((rc = launch_dense_den<real>(c, B, t, es, false, true))) return rc;
      if ((rc = fgemm_ab<real>(c, B, S8))) return rc;
    } else if (dense) {
      if ((rc = launch_dense_az<real>(c, B, t, es, 0))) return rc;
      if ((rc = launch_dense_den<real>(c, B, t, es))) return rc;
      if ((rc = launch_dense_ab<real>(c, B, t, es, 0))) return rc;
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
  for (int l = 0; l < L; ++l) {
    const uint32_t* o = c->ordering.data() + (size_t)l * n;
    uint16_t* il = inv.data() + (size_t)l * w;
    for (int r = 0; r < n; ++r) {
      const uint32_t v = o[r];
      if (v == 0 || v >= (uint32_t)w)
        return fail(SA_ERR_ORDERING, "ordering[" + std::to_string(l) + "," + std::to_string(r) +
                                         "] = " + std::to_string(v) + " outside [1, w=" + std::to_string(w) + ")");
      if (il[v] != (uint16_t)n)
        return fail(SA_ERR_ORDERING, "ordering row " + std::to_string(l) + " repeats value " + std::to_string(v));
      il[v] = (uint16_t)r;
      const uint32_t hi = v >> lgM;
      const uint16_t e = (uint16_t)((v & (uint32_t)(M - 1)) | ((__builtin_popcount(hi) & 1u) << 15));
      fwd[((size_t)(l / kSpw) * n + r) * kSpw + (l % kSpw)] = e;
      fwd2[(size_t)(l / 2) * n + r] |= (uint32_t)e << (16 * (l & 1));
      if (c->sec3)  // M <= 512: k in 9 bits, the sign in bit 9 of a 10-bit field
        fwd3[(size_t)(l / 3) * n + r] |= (uint32_t)((e & 0x1ffu) | ((e >> 15) << 9)) << (10 * (l % 3));
    }
  }
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
  std::vector<uint16_t> inv((size_t)L * w, (uint16_t)n), out((size_t)L * w, 0);
  std::vector<uint32_t> hs((size_t)L, 0);
  for (int l = 0; l < L; ++l)
    for (int r = 0; r < n; ++r) inv[(size_t)l * w + c->ordering[(size_t)l * n + r]] = (uint16_t)r;
  unsigned nth = std::thread::hardware_concurrency();
  nth = nth == 0 ? 1 : (nth > 16 ? 16 : nth);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nth; ++t)
    th.emplace_back([&, t]() {
      for (int l = (int)t; l < L; l += (int)nth)
        banked_section(c, l, inv.data() + (size_t)l * w, out.data() + (size_t)l * w, sets, gsize, nbank,
                       hs.data(), kh);
    });
  for (auto& x : th) x.join();
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
        for (int it = 0; it < 64 * W; ++it) {
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
  std::vector<uint16_t> fwd((size_t)G * n * kSpw, 0);
  for (int l = 0; l < c->L; ++l)
    for (int r = 0; r < n; ++r) {
      const uint32_t v = c->ordering[(size_t)l * n + r];
      fwd[((size_t)(l / kSpw) * n + r) * kSpw + (l % kSpw)] =
          (uint16_t)((v & (uint32_t)(c->M - 1)) | ((__builtin_popcount(v >> lgM) & 1u) << 15));
    }
  std::vector<uint16_t> out((size_t)Gb * W * npad, 0);
  unsigned nth = std::thread::hardware_concurrency();
  nth = nth == 0 ? 1 : (nth > 16 ? 16 : nth);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nth; ++t)
    th.emplace_back([&, t]() {
      for (int g = (int)t; g < Gb; g += (int)nth) fwdb_group(c, g, fwd.data(), npad, out.data());
    });
  for (auto& x : th) x.join();
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
    // (the kernel's h-steps per table block: SA_F64_KH in binary64, SA_F32_KH at CB = 4)
    const int kh = SA_SECB_COMPACT ? (sgn ? SA_F32_KH : SA_F64_KH) : c->nhi / 2;
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
  return SA_OK;
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

// Allow every section-kernel instantiation the full 160 KB LDS (once per process).
template <typename real>
hipError_t lds_attr_all() {
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
  SA_A((k_secb<real, 1, 1, kWB>)) SA_A((k_secb<real, 2, 1, kWB>)) SA_A((k_secb<real, 4, 1, kWB>))
  SA_A((k_secb<real, 8, 1, kWB>)) SA_A((k_secb<real, 16, 1, kWB>))
  SA_A((k_secb<real, 1, 2, kWB>)) SA_A((k_secb<real, 2, 2, kWB>)) SA_A((k_secb<real, 4, 2, kWB>))
  SA_A((k_secb<real, 8, 2, kWB>)) SA_A((k_secb<real, 16, 2, kWB>))
  SA_A((k_secb<real, 1, 1, kWB16>)) SA_A((k_secb<real, 2, 1, kWB16>)) SA_A((k_secb<real, 4, 1, kWB16>))
  SA_A((k_secb<real, 8, 1, kWB16>)) SA_A((k_secb<real, 16, 1, kWB16>))
  SA_A((k_secb<real, 1, 2, kWB16>)) SA_A((k_secb<real, 2, 2, kWB16>)) SA_A((k_secb<real, 4, 2, kWB16>))
  SA_A((k_secb<real, 8, 2, kWB16>)) SA_A((k_secb<real, 16, 2, kWB16>))
  if constexpr (sizeof(real) == 8) {  // codeword-interleaved (16-byte rows: CB = 2)
    SA_A((k_secb<real, 1, 2, kWB, true>)) SA_A((k_secb<real, 2, 2, kWB, true>)) SA_A((k_secb<real, 4, 2, kWB, true>))
    SA_A((k_secb<real, 8, 2, kWB, true>)) SA_A((k_secb<real, 16, 2, kWB, true>))
    SA_A((k_secb<real, 1, 2, kWB16, true>)) SA_A((k_secb<real, 2, 2, kWB16, true>))
    SA_A((k_secb<real, 4, 2, kWB16, true>)) SA_A((k_secb<real, 8, 2, kWB16, true>))
    SA_A((k_secb<real, 16, 2, kWB16, true>))
  }
  if constexpr (sizeof(real) == 4) {
    SA_A((k_secb<real, 1, 4, kWB>)) SA_A((k_secb<real, 2, 4, kWB>)) SA_A((k_secb<real, 4, 4, kWB>))
    SA_A((k_secb<real, 8, 4, kWB>)) SA_A((k_secb<real, 16, 4, kWB>))
    SA_A((k_secb<real, 1, 4, kWB16>)) SA_A((k_secb<real, 2, 4, kWB16>)) SA_A((k_secb<real, 4, 4, kWB16>))
    SA_A((k_secb<real, 8, 4, kWB16>)) SA_A((k_secb<real, 16, 4, kWB16>))
    SA_A((k_secb<real, 1, 4, kWB, true>)) SA_A((k_secb<real, 2, 4, kWB, true>)) SA_A((k_secb<real, 4, 4, kWB, true>))
    SA_A((k_secb<real, 8, 4, kWB, true>)) SA_A((k_secb<real, 16, 4, kWB, true>))
    SA_A((k_secb<real, 1, 4, kWB16, true>)) SA_A((k_secb<real, 2, 4, kWB16, true>))
    SA_A((k_secb<real, 4, 4, kWB16, true>)) SA_A((k_secb<real, 8, 4, kWB16, true>))
    SA_A((k_secb<real, 16, 4, kWB16, true>))
  }
#undef SA_A
  return e;
}

// gather_step4 addresses LDS absolutely: the batched kernel must have no
// static LDS in front of its dynamic region.
template <typename real>
bool secb_no_static_lds() {
  hipFuncAttributes at;
  const void* fs[] = {(const void*)k_secb<real, 4, 1, kWB>, (const void*)k_secb<real, 8, 1, kWB>,
                      (const void*)k_secb<real, 16, 1, kWB>, (const void*)k_secb<real, 8, 2, kWB>,
                      (const void*)k_secb<real, 16, 2, kWB>, (const void*)k_secb<real, 8, 2, kWB16>,
                      (const void*)k_secb<real, 16, 2, kWB16>, (const void*)k_secb<real, 8, 1, kWB16>};
  for (const void* f : fs)
    if (hipFuncGetAttributes(&at, f) != hipSuccess || at.sharedSizeBytes != 0) return false;
  return true;
}

int set_lds_limits() {
  static int done = 0;
  if (done) return SA_OK;
  if (!secb_no_static_lds<float>() || !secb_no_static_lds<double>())
    return fail(SA_ERR_HIP, "k_secb has static LDS: absolute LDS addressing in gather_step4 is invalid");
  hipError_t e = lds_attr_all<float>();
  if (e == hipSuccess) e = lds_attr_all<double>();
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_gemm_i8<kI8NPZ>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            I8Tile<kI8NPZ>::Lds);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_gemm_i8<kI8NPB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            I8Tile<kI8NPB>::Lds);
  {
    const void* fs[] = {(const void*)k_gemm_f<float, 0>, (const void*)k_gemm_f<float, 1>,
                        (const void*)k_gemm_f<double, 0>, (const void*)k_gemm_f<double, 1>};
    for (const void* f : fs)
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kFLds);
  }
  if (e != hipSuccess) return fail(SA_ERR_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  done = 1;
  return SA_OK;
}

int create_impl(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int prec,
                int device, int plan, const sa_ctx* share = nullptr) {
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
  if (!pow2 && backend == SA_BACKEND_HADAMARD)
    return fail(SA_ERR_UNSUPPORTED, "the matrix-free Hadamard operator needs M a power of two "
                                    "(the dense and host-operator backends take any M)");
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
  const int mx = (M + 1) > (n + 1) ? (M + 1) : (n + 1);
  c->w = 1 << ilog2(mx);  // 2^ceil(log2(max(M+1, n+1))), sparc_ldpc.py:52/:110
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
  if (c->sec_lds > 160 * 1024) {
    delete c;
    return fail(SA_ERR_UNSUPPORTED, "section kernel does not fit in LDS (n and M too large for this precision)");
  }
  c->G = (L + kSpw - 1) / kSpw;
  c->Gb = (L + kWB - 1) / kWB;  // (re-set after the batched width is chosen)
  if (M >= 128 && M <= 4096 && !c->big) {  // k_sec2: z + 2 sections' T + top-bit exchange + reductions
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
        const size_t need = (zb > tb ? zb : tb) + (size_t)W * cb * s + (s == 8 && SA_F64_EXPTAB ? 64 * 8 : 0);
        if (need <= (cb == 1 || W > kWB ? 160 : 80) * 1024) return {cb, need};
      }
      return {0, 0};
    };
    const auto c8 = c->big ? std::pair<int, size_t>{0, 0} : cb_for(kWB);
    const auto c16 = c->big ? std::pair<int, size_t>{0, 0} : cb_for(kWB16);
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
    // the caller's matrix, uploaded by sa_create_matrix: rows of whole GEMM K
    // stages (128 B), padded to whole 256-row tiles, zero padding
    c->RS = 8;
    c->KS = 8;
    const long long ks = kFKB / (long long)s;
    c->lda = (size_t)(((long long)L * M + ks - 1) / ks * ks);
    c->np = ((long long)n + kFTY - 1) / kFTY * kFTY;
    c->nk = ((long long)n + ks - 1) / ks * ks;
    c->LMy = ((long long)L * M + kFTY - 1) / kFTY * kFTY;
    rc = dev_alloc(c, &c->d_A, (size_t)c->np * c->lda * s);
    if (!rc) {
      hipError_t e = hipMemsetAsync(c->d_A, 0, (size_t)c->np * c->lda * s, c->stream);
      if (e != hipSuccess) rc = fail(SA_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
    }
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

}  // namespace


// ---------------------------------------------------------------------------
// SPARC <-> LDPC glue of the joint decoder (sparc_ldpc.py:257-314, 359-712)
// ---------------------------------------------------------------------------
// All of it runs on the device in binary64 on the B codewords of the batch;
// the LLR / app arrays are handed to and from the LDPC decoder
// (libldpc_bp.so) as device pointers, so a joint round never leaves HBM.
namespace {

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

}  // namespace

extern "C" {

int sa_create(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int precision,
              int device) {
  return create_impl(out, L, M, n, ordering, backend, precision, device, SA_PLAN_DEFAULT);
}

int sa_create_ex(sa_ctx** out, int L, int M, int n, const uint32_t* ordering, int backend, int precision,
                 int device, int plan) {
  return create_impl(out, L, M, n, ordering, backend, precision, device, plan);
}

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
  return create_impl(out, Ls, parent->M, parent->n, ord.data(), parent->backend, parent->prec, parent->device,
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
  return create_impl(out, src->L, src->M, src->n, src->ordering.data(), src->backend, src->prec, src->device,
                     src->plan, src);
}

void sa_destroy(sa_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  drop_graphs(c);
  free_workspace(c);
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
  const size_t LM = (size_t)c->L * c->M;
  if ((rc = upload(c, c->d_beta, beta, (size_t)B * LM))) return rc;
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
  const size_t LM = (size_t)c->L * c->M;
  if ((rc = upload(c, c->d_z, z, (size_t)B * c->n))) return rc;
  c->zil_last = false;  // d_z holds [B][n] now
  if (c->prec == SA_PREC_F64) {
    rc = seq_az<double>(c, B);
  } else {
    rc = seq_az<float>(c, B);
  }
  if (rc) return rc;
  if ((rc = download(c, out, c->d_out, (size_t)B * LM))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SA_OK;
}

int sa_reserve(sa_ctx* c, int B, int T) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || T < 0) return fail(SA_ERR_ARG, "sa_reserve: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  return ensure_workspace(c, B, T > 0 ? T : 1);
}

int sa_stage(sa_ctx* c, int B, const double* y, const double* Pl, const double* beta0) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0) return fail(SA_ERR_ARG, "sa_stage: bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_workspace(c, B, c->Tcap > 0 ? c->Tcap : 1);
  if (rc) return rc;
  if (Pl && (rc = set_power(c, Pl))) return rc;
  if (y && (rc = upload(c, c->d_y, y, (size_t)B * c->n))) return rc;  // NULL: keep the staged y
  if (beta0 && (rc = upload(c, c->d_beta, beta0, (size_t)B * c->L * c->M))) return rc;
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

int sa_fetch(sa_ctx* c, int B, double* beta_out, int* iters_out) {
  if (check_ctx(c)) return SA_ERR_ARG;
  if (B <= 0 || B > c->Bcap) return fail(SA_ERR_ARG, "sa_fetch: bad batch");
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  if (beta_out && (rc = download(c, beta_out, c->d_beta, (size_t)B * c->L * c->M))) return rc;
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

extern "C++" {
namespace {
int launch_decide(sa_ctx* c, int B) {
  dim3 grid((c->L + 3) / 4, B);
#define SA_DEC(EE)                                                                                             \
  case EE:                                                                                                     \
    if (c->prec == SA_PREC_F64)                                                                                \
      k_decide<double, EE><<<grid, 256, 0, c->stream>>>((const double*)c->d_beta, c->d_idx, c->L, c->M);      \
    else                                                                                                       \
      k_decide<float, EE><<<grid, 256, 0, c->stream>>>((const float*)c->d_beta, c->d_idx, c->L, c->M);        \
    break;
  switch (c->E) { SA_DEC(1) SA_DEC(2) SA_DEC(4) SA_DEC(8) SA_DEC(16) SA_DEC(32) SA_DEC(64) }
#undef SA_DEC
  HIP_TRY(hipGetLastError());
  return SA_OK;
}
}  // namespace
}  // extern "C++"

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

int sa_plan(sa_ctx* c, int B, int64_t* o) {
  if (check_ctx(c) || !o || B <= 0) return fail(SA_ERR_ARG, "sa_plan: bad arguments");
  const bool dense = is_dense(c);
  const bool batched = !dense && use_batched(c, B);
  const bool sec2 = use_sec2(c, B);
  const bool i8 = use_i8(c, B);
  const bool fg = use_fgemm(c, B);
  o[0] = i8 ? 6 : (fg ? 7 : (dense ? 3 : (batched ? 2 : (sec2 ? (c->sec3 ? 5 : (c->sec4 ? 4 : 1)) : (c->big ? 8 : 0)))));
  o[1] = i8 ? i8_splits(c, B)
            : (fg ? fgemm_splits(c, B) : (dense ? c->KS : (batched ? c->Gb : (sec2 ? sec2_parts(c) : c->G))));
  o[2] = (!dense && !batched && !sec2) ? row_splits(c, B) : 1;
  o[3] = batched ? c->CB : 1;
  o[4] = nz_for(c, row_kind_for(c, B));
  o[5] = c->w;
  o[6] = row_kind_for(c, B);
  o[7] = c->n_cus;
  return SA_OK;
}

int sa_info(const sa_ctx* c, int64_t* o) {
  if (check_ctx(c) || !o) return fail(SA_ERR_ARG, "sa_info: bad arguments");
  o[0] = c->L; o[1] = c->M; o[2] = c->n; o[3] = c->w; o[4] = c->backend; o[5] = c->prec;
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
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16 * 16));
  return SA_OK;
}
#endif

}  // extern "C"
