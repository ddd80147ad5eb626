// Does ds_read_b128 at 4-byte (not 16-byte) aligned LDS addresses return the
// right bytes on gfx950, and at what cost?  One workgroup per CU, each wave
// reads 16-B pieces at lane * 108 + 16 j + off (off = 0 or 8 bytes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1;} } while (0)

template <int MODE>  // 0: b128 at 4-B aligned, 1: 4 x b32, 2: b128 at 16-B aligned (wrong data, timing only)
__global__ void __launch_bounds__(512) k(uint32_t* out, int iters, int check) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 64 * 1024 / 4 * 8 / 8; i += blockDim.x) lds[i] = i * 2654435761u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t base = (uint32_t)wave * 7168u + (uint32_t)lane * 108u;
  uint32_t acc = 0, bad = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      uint32_t a = base + 16u * j + 4u * (uint32_t)(it & 1);
      if (MODE == 2) a &= ~15u;
      u32x4 v;
      if (MODE == 1) {
        v.x = *(const lds_u32*)(uintptr_t)(a);
        v.y = *(const lds_u32*)(uintptr_t)(a + 4);
        v.z = *(const lds_u32*)(uintptr_t)(a + 8);
        v.w = *(const lds_u32*)(uintptr_t)(a + 12);
      } else {
        v = *(const lds_u32x4*)(uintptr_t)a;
      }
      if (check) {
        const uint32_t w = a / 4;
        bad |= (v.x != w * 2654435761u) | (v.y != (w + 1) * 2654435761u) |
               (v.z != (w + 2) * 2654435761u) | (v.w != (w + 3) * 2654435761u);
      }
      acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
    }
  }
  if (check) atomicOr(out, bad);
  if (acc == 0x12345678u) out[1] = acc;
}

int main() {
  uint32_t* d;
  CK(hipMalloc(&d, 8));
  int ncu = 256;
  size_t lds = 64 * 1024;
  for (int mode = 0; mode < 3; ++mode) {
    CK(hipMemset(d, 0, 8));
    auto kern = mode == 0 ? k<0> : mode == 1 ? k<1> : k<2>;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(512), lds, 0, d, 4, 1);
    CK(hipDeviceSynchronize());
    uint32_t bad = 0;
    CK(hipMemcpy(&bad, d, 4, hipMemcpyDeviceToHost));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(ncu), dim3(512), lds, 0, d, 20000, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    // LDS instructions per CU: 8 waves * 20000 * 7 (x4 for mode 1)
    double ninst = 8.0 * 20000 * 7 * (mode == 1 ? 4 : 1);
    printf("mode %d (%s): data %s, %.3f ms, %.2f ns per LDS instr per CU\n", mode,
           mode == 0 ? "b128 @4B-aligned" : mode == 1 ? "4 x b32" : "b128 @16B-aligned",
           mode == 2 ? "n/a" : (bad ? "WRONG" : "ok"), ms, ms * 1e6 / ninst);
  }
  return 0;
}
