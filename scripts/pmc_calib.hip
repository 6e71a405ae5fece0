// PMC calibration probe (diagnostic, never part of the product).
//
// Question: how many bytes do rocprofv3's FETCH_SIZE / WRITE_SIZE report for
// each access width and cache policy the product kernels use?  The guide
// (MI355X_MICROARCH.md, HBM) calibrates only 16-B-per-lane streaming loads
// (FETCH_SIZE = 1/2 of the bytes) and 16-B stores (exact); other widths are
// "uncalibrated".  Each kernel below touches a 1 GiB buffer (past the 256 MiB
// Infinity Cache) exactly once with one pattern; the ratio counter / bytes is
// the correction factor for that pattern.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/pmc_calib scripts/pmc_calib.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -d DIR -o f --output-format csv -- ./scripts/pmc_calib
//   rocprofv3 --kernel-trace --pmc WRITE_SIZE -d DIR -o w --output-format csv -- ./scripts/pmc_calib
//   python3 scripts/pmc_calib.py DIR
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr size_t kBytes = size_t(1) << 30;

template <int W> struct VT;
template <> struct VT<2> { using t = unsigned short; };
template <> struct VT<4> { using t = unsigned; };
template <> struct VT<8> { using t = unsigned __attribute__((ext_vector_type(2))); };
template <> struct VT<16> { using t = unsigned __attribute__((ext_vector_type(4))); };

template <typename T> __device__ __forceinline__ unsigned fold(T v) {
  if constexpr (sizeof(T) <= 4) return (unsigned)v;
  else if constexpr (sizeof(T) == 8) return v.x ^ v.y;
  else return v.x ^ v.y ^ v.z ^ v.w;
}

// read every byte once, W bytes per lane, consecutive lanes consecutive
template <int W, bool NT>
__global__ void __launch_bounds__(256) rd(const char* __restrict__ p, unsigned* out) {
  using T = typename VT<W>::t;
  const T* q = reinterpret_cast<const T*>(p);
  const size_t n = kBytes / W;
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v = NT ? __builtin_nontemporal_load(q + i) : q[i];
    acc ^= fold(v);
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // practically never: keeps the loads
}

// write every byte once
template <int W, bool NT>
__global__ void __launch_bounds__(256) wr(char* __restrict__ p) {
  using T = typename VT<W>::t;
  T* q = reinterpret_cast<T*>(p);
  const size_t n = kBytes / W;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v = T(i);
    if (NT) __builtin_nontemporal_store(v, q + i);
    else q[i] = v;
  }
}

// LDS-DMA: 1 KiB per wave instruction (global_load_lds_dwordx4)
__global__ void __launch_bounds__(256) rd_dma(const char* __restrict__ p, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char buf[4][1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t nch = kBytes / 1024;
  for (size_t ch = blockIdx.x * 4 + wv; ch < nch; ch += (size_t)gridDim.x * 4) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(p + ch * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)(buf[wv]), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (buf[0][threadIdx.x] == 0x5a && out[0] == 0x12345678u) out[1] = 1;
}

int main() {
  char* d = nullptr;
  unsigned* o = nullptr;
  CK(hipMalloc(&d, kBytes));
  CK(hipMalloc(&o, 4096 * sizeof(unsigned)));
  CK(hipMemset(d, 1, kBytes));
  CK(hipMemset(o, 0, 4096 * sizeof(unsigned)));
  const int G = 4096;
  rd<16, false><<<G, 256>>>(d, o);
  rd<8, false><<<G, 256>>>(d, o);
  rd<4, false><<<G, 256>>>(d, o);
  rd<2, false><<<G, 256>>>(d, o);
  rd<16, true><<<G, 256>>>(d, o);
  rd<8, true><<<G, 256>>>(d, o);
  rd<4, true><<<G, 256>>>(d, o);
  rd_dma<<<G, 256>>>(d, o);
  wr<16, false><<<G, 256>>>(d);
  wr<8, false><<<G, 256>>>(d);
  wr<4, false><<<G, 256>>>(d);
  wr<16, true><<<G, 256>>>(d);
  wr<8, true><<<G, 256>>>(d);
  wr<4, true><<<G, 256>>>(d);
  CK(hipDeviceSynchronize());
  printf("pmc_calib: %zu bytes per kernel\n", kBytes);
  CK(hipFree(d));
  CK(hipFree(o));
  return 0;
}
