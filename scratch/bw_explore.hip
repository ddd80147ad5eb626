// Read-bandwidth microbenchmark on MI355X: which load style reaches the HBM ceiling?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int R, bool NT>
__global__ void __launch_bounds__(256) rd_gridstride(const u32x4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  const uint64_t gsz = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i + (R - 1) * gsz < n16; i += R * gsz) {
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = NT ? __builtin_nontemporal_load(p + i + r * gsz) : p[i + r * gsz];
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= v[r];
  }
  for (; i < n16; i += gsz) acc ^= p[i];
  uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9E3779B9u) sink[0] = x;
}

// each block sweeps a contiguous chunk
template <int R, bool NT>
__global__ void __launch_bounds__(1024) rd_chunk(const u32x4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = blockIdx.x * per, b1 = min(n16, b0 + per);
  u32x4 acc = {0, 0, 0, 0};
  uint64_t i = b0 + threadIdx.x;
  for (; i + (R - 1) * 1024 < b1; i += R * 1024) {
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = NT ? __builtin_nontemporal_load(p + i + r * 1024) : p[i + r * 1024];
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= v[r];
  }
  for (; i < b1; i += 1024) acc ^= p[i];
  uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9E3779B9u) sink[0] = x;
}

// LDS-DMA ring: each wave streams its own slice through a 4-slot ring of 1 KiB pieces x K
template <int K, int AUX>
__global__ void __launch_bounds__(1024) rd_ldsdma(const uint8_t* __restrict__ p, uint64_t nbytes, uint32_t* sink) {
  extern __shared__ uint32_t lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t nwaves = (uint64_t)gridDim.x * 16;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + wave;
  const uint64_t pieces = nbytes / 1024;
  uint32_t acc = 0;
  // wave-private LDS region: K slots x 1 KiB
  __attribute__((address_space(3))) uint32_t* base = (__attribute__((address_space(3))) uint32_t*)((uintptr_t)(wave * K * 1024));
  uint64_t pc = gw;
  for (; pc + (K - 1) * nwaves < pieces; pc += K * nwaves) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint8_t* src = p + (pc + k * nwaves) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(base + k * 256), 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < K; ++k) {
      u32x4 v = *(__attribute__((address_space(3))) u32x4*)(base + k * 256 + lane * 4);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
  const uint64_t bytes = 4341104640ull;  // cfg2 frame buffer
  uint8_t* d;
  uint32_t* sink;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(d, 0x5a, bytes));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-40s med %.3f ms  %.1f GB/s (best %.1f)\n", name, ts[3], bytes / ts[3] / 1e6, bytes / ts[0] / 1e6);
    fflush(stdout);
  };
  const uint64_t n16 = bytes / 16;
  const u32x4* p = (const u32x4*)d;
  for (int bpc : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, 64, "gridstride R8 plain bpc=%d", bpc);
    run(nm, [&] { hipLaunchKernelGGL((rd_gridstride<8, false>), dim3(cus * bpc), dim3(256), 0, 0, p, n16, sink); });
    snprintf(nm, 64, "gridstride R8 nt bpc=%d", bpc);
    run(nm, [&] { hipLaunchKernelGGL((rd_gridstride<8, true>), dim3(cus * bpc), dim3(256), 0, 0, p, n16, sink); });
  }
  run("gridstride R16 nt bpc=8", [&] { hipLaunchKernelGGL((rd_gridstride<16, true>), dim3(cus * 8), dim3(256), 0, 0, p, n16, sink); });
  run("chunk R8 plain 1/cu", [&] { hipLaunchKernelGGL((rd_chunk<8, false>), dim3(cus), dim3(1024), 0, 0, p, n16, sink); });
  run("chunk R8 nt 1/cu", [&] { hipLaunchKernelGGL((rd_chunk<8, true>), dim3(cus), dim3(1024), 0, 0, p, n16, sink); });
  run("chunk R8 plain 2/cu", [&] { hipLaunchKernelGGL((rd_chunk<8, false>), dim3(cus * 2), dim3(1024), 0, 0, p, n16, sink); });
  run("chunk R4 plain 1/cu", [&] { hipLaunchKernelGGL((rd_chunk<4, false>), dim3(cus), dim3(1024), 0, 0, p, n16, sink); });
  hipFuncSetAttribute((const void*)rd_ldsdma<4, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  hipFuncSetAttribute((const void*)rd_ldsdma<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  hipFuncSetAttribute((const void*)rd_ldsdma<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  run("ldsdma K4 aux0 1/cu", [&] { hipLaunchKernelGGL((rd_ldsdma<4, 0>), dim3(cus), dim3(1024), 65536, 0, d, bytes, sink); });
  run("ldsdma K4 nt 1/cu", [&] { hipLaunchKernelGGL((rd_ldsdma<4, 2>), dim3(cus), dim3(1024), 65536, 0, d, bytes, sink); });
  run("ldsdma K8 nt 1/cu", [&] { hipLaunchKernelGGL((rd_ldsdma<8, 2>), dim3(cus), dim3(1024), 131072, 0, d, bytes, sink); });
  return 0;
}
