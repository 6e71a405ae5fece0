// sa_common.h — device-side building blocks shared by the AMP kernel units
// (sa_sec.hip, sa_secb.hip, sa_row.hip, sa_dense.hip, sa_glue.hip): cross-lane
// moves, the M-point FWHT, the section denoiser, loads / stores, the kernel
// argument blocks and the operator constants.  See sparc_amp.hip for the
// operator's factorisation.
#pragma once
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

namespace sa {

// last error message of the calling thread (sa_last_error)
extern thread_local std::string g_err;
int fail(int code, const std::string& msg);

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
static __constant__ double c_exp2_64[64] = {  // 2^(j/64), correctly rounded (generated with decimal, 80 digits)
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
                                                bool store = true, int dead = 0) {
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
    u[i] = (e < M && e >= dead) ? uu : neg_inf<real>();  // dead columns of a padded section: beta 0
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
  // Monte-Carlo stream (sa_mc_run): per-codeword iteration index t_b (slot_t),
  // -1 for an empty slot; null: every codeword is at iteration t
  const int* tb;
  int dead;  // leading dead columns of a padded section (sa_ctx::dead; k_sec only)
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
  const int* tb;  // k_rowc: per-codeword iteration index (SecArgs::tb), or null
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

#ifdef SA_STAMPS
// [wave][stamp]: every wave of the stamped workgroup records its own phases
static __device__ unsigned long long g_stamps[16 * 16];
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
// k_secb's bucket h-steps with table loads in flight per block (binary32 at
// CB = 4 or E = 16 / binary64); the bank-aware table (ensure_invb) pads each
// half's occupied steps to a multiple of it
constexpr int kSecbKH32 = 2, kSecbKH64 = 2;

template <int N>
constexpr int ilog2c() { return N <= 1 ? 0 : 1 + ilog2c<N / 2>(); }

// argmax of one section (one wave, lane's elements elem_index<E>), first index
// on ties as np.argmax (sparc_ldpc.py:452-455); uniform over the wave
template <typename real, int E>
__device__ __forceinline__ int section_argmax(const real* bl, int lane, int M, int dead = 0) {
  real best = neg_inf<real>();
  int bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const int e = elem_index<E>(lane, i);
    if (e < M && e >= dead) {
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
  return bi == 0x7fffffff ? 0 : bi - dead;  // the caller's column (a padded section's dead columns first)
}

constexpr int kRow2Rows = 32;  // k_row2: one 128-B line of a partial per row block

inline int ilog2(int x) {
  int r = 0;
  while ((1 << r) < x) ++r;
  return r;
}

}  // namespace sa
