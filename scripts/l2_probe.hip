// L2-residency probe (diagnostic, never part of the product).
//
// Question: does a per-XCD table share stay in that XCD's L2 across kernel
// boundaries when every workgroup picks its share by the XCC it runs on
// (s_getreg HW_REG_XCC_ID + a per-XCD ticket), instead of by blockIdx (whose
// XCD may rotate from launch to launch)?
//
// 256 workgroups x 512 threads each read a 48 KB slice of an 8 x 1.5 MB table
// set (12 MB, the size of the c2 bucket + Ab tables) and write one sum.  Between
// table launches a "row" kernel streams 4.7 MB of other data (the Ab
// partials' size).  Reported per mode: mean table-kernel time (HIP events over
// 64 launches) and, under rocprofv3 --pmc FETCH_SIZE, the fetch per dispatch.
//
//   hipcc --offload-arch=gfx950 -O3 -o l2_probe scripts/l2_probe.hip
//   ./l2_probe            (modes: 0 blockIdx, 1 XCC-stable)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kWG = 256, kNT = 512;
constexpr size_t kSlice = 48 * 1024;           // bytes per workgroup
constexpr size_t kTable = kSlice * kWG;        // 12 MB

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

// mode 0: slice = blockIdx.x.  mode 1: slice = xcc * 32 + ticket, where the
// ticket comes from a per-XCD counter (work stealing from the next XCD's
// queue when this XCD got more than 32 workgroups); the last finisher resets.
__global__ void __launch_bounds__(kNT) k_table(const float4* __restrict__ tab, float* out, unsigned* tick,
                                               int mode) {
  __shared__ int s_slice;
  if (threadIdx.x == 0) {
    int s = blockIdx.x;
    if (mode == 1) {
      const int x = xcc_id();
      s = -1;
      for (int k = 0; k < 8 && s < 0; ++k) {
        const int q = (x + k) & 7;
        const unsigned r = atomicAdd(&tick[q], 1u);
        if (r < 32) s = q * 32 + (int)r;
      }
    }
    s_slice = s;
  }
  __syncthreads();
  const int s = s_slice;
  float acc = 0.f;
  if (s >= 0) {
    const float4* p = tab + (size_t)s * (kSlice / 16);
    for (size_t i = threadIdx.x; i < kSlice / 16; i += kNT) {
      const float4 v = p[i];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  for (int m = 32; m; m >>= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0) atomicAdd(&out[blockIdx.x], acc);
  if (mode == 1) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned d = atomicAdd(&tick[8], 1u);
      if (d == kWG - 1) {  // last finisher: reset for the next launch
        for (int q = 0; q < 9; ++q) atomicExch(&tick[q], 0u);
      }
    }
  }
}

// stand-in for the row kernel: streams `nb` bytes with non-temporal loads
__global__ void __launch_bounds__(256) k_stream(const float4* __restrict__ p, size_t n4, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p) + i);
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

int main(int argc, char** argv) {
  const int reps = 64;
  float4 *tab, *str;
  float* out;
  unsigned* tick;
  const size_t sbytes = 4718592;
  CK(hipMalloc(&tab, kTable));
  CK(hipMalloc(&str, sbytes));
  CK(hipMalloc(&out, kWG * sizeof(float)));
  CK(hipMalloc(&tick, 16 * sizeof(unsigned)));
  CK(hipMemset(tab, 0, kTable));
  CK(hipMemset(str, 0, sbytes));
  CK(hipMemset(tick, 0, 16 * sizeof(unsigned)));
  CK(hipMemset(out, 0, kWG * sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    for (int with_stream = 0; with_stream < 2; ++with_stream) {
      for (int w = 0; w < 4; ++w) k_table<<<kWG, kNT>>>(tab, out, tick, mode);
      CK(hipDeviceSynchronize());
      float tot = 0.f;
      for (int r = 0; r < reps; ++r) {
        if (with_stream) k_stream<<<512, 256>>>(str, sbytes / 16, out);
        CK(hipEventRecord(e0));
        k_table<<<kWG, kNT>>>(tab, out, tick, mode);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
      }
      std::vector<unsigned> t(16);
      CK(hipMemcpy(t.data(), tick, 16 * sizeof(unsigned), hipMemcpyDeviceToHost));
      printf("mode=%d (%s) stream_between=%d: table kernel %.2f us/launch (event-bracketed), tick[8]=%u\n",
             mode, mode ? "xcc-stable" : "blockIdx", with_stream, tot / reps * 1e3, t[8]);
    }
  }
  return 0;
}
