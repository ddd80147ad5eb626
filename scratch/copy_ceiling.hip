// How fast can MI355X copy?  (The segmentation kernel runs at the rate of
// its own copy pattern, ~5.4 TB/s of read + write bytes; MI355X_MICROARCH.md
// quotes 6.29 TB/s for a float4 copy.)  Copy shapes over 2 GiB -> 2 GiB,
// GB/s = (read + written bytes) / median time.
// build: hipcc --offload-arch=gfx950 -O3 -o scratch/copy_ceiling scratch/copy_ceiling.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                    \
    }                                                             \
  } while (0)

// grid-stride, U float4 per thread per iteration; LP/SP: nt loads / stores
template <int U, bool LNT, bool SNT>
__global__ void gs_copy(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t k = i + u * stride;
      if (k < n16) v[u] = LNT ? __builtin_nontemporal_load(s + k) : s[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t k = i + u * stride;
      if (k < n16) {
        if (SNT)
          __builtin_nontemporal_store(v[u], d + k);
        else
          d[k] = v[u];
      }
    }
  }
}

// one workgroup per CU sweeping a contiguous chunk, R loads then R stores per lane
template <int R, bool SNT>
__global__ void cu_copy(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n16) {
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b = blockIdx.x * per, e = min(n16, b + per);
  for (uint64_t i = b + threadIdx.x; i < e; i += (uint64_t)blockDim.x * R) {
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t k = i + (uint64_t)r * blockDim.x;
      v[r] = k < e ? __builtin_nontemporal_load(s + k) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t k = i + (uint64_t)r * blockDim.x;
      if (k < e) {
        if (SNT)
          __builtin_nontemporal_store(v[r], d + k);
        else
          d[k] = v[r];
      }
    }
  }
}

int main() {
  const uint64_t bytes = 2ull << 30, n16 = bytes / 16;
  u32x4 *s, *d;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 0x5a, bytes));
  CK(hipMemset(d, 0, bytes));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 20; ++w) launch();
    std::vector<float> ts;
    for (int r = 0; r < 20; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"copy\": \"%s\", \"ms\": %.4f, \"GBps_rw\": %.1f}\n", name, ts[10], 2.0 * bytes / ts[10] / 1e6);
    fflush(stdout);
  };
#define GS(U, L, S, T, B) run("grid-stride U=" #U " ldnt=" #L " stnt=" #S " T=" #T " blocks=" #B "xCU", [&] { hipLaunchKernelGGL((gs_copy<U, L, S>), dim3(ncu * B), dim3(T), 0, 0, s, d, n16); });
#define CU(R, S, T) run("per-CU R=" #R " stnt=" #S " T=" #T, [&] { hipLaunchKernelGGL((cu_copy<R, S>), dim3(ncu), dim3(T), 0, 0, s, d, n16); });
  for (int rep = 0; rep < 2; ++rep) {
    GS(1, false, false, 256, 8)
    GS(1, false, false, 1024, 4)
    GS(4, false, false, 256, 8)
    GS(4, true, true, 256, 8)
    GS(4, true, false, 256, 8)
    GS(2, false, false, 512, 16)
    GS(1, false, false, 256, 64)
    CU(4, true, 1024)
    CU(4, false, 1024)
    CU(8, true, 512)
    CU(2, true, 1024)
    CU(8, true, 1024)
  }
  return 0;
}
