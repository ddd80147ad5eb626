// HBM fetch granularity: does a wave that touches only part of each 128-byte
// line move fewer bytes?  Every lane issues the same 16-byte loads; in kernel
// variant K the lanes of each 8-lane line group read chunks (lane & 7) & MASK
// of their line, so the touched bytes per line are 128 (MASK 7), 64 (3),
// 32 (1) or 16 (0).  If the time drops with the touched bytes, a partly used
// boundary line costs only its touched sectors.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int MASK>
__global__ void __launch_bounds__(1024) rd(const u32x4* __restrict__ p, uint64_t nlines, uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int chunk = (lane & 7) & MASK;
  const int line = lane >> 3;  // 8 lines per wave instruction
  u32x4 acc = {0, 0, 0, 0};
  // each wave: 4 instructions in flight, 32 lines, then the next block
  for (uint64_t b = wave * 32; b + 32 <= nlines; b += nwaves * 32) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[(b + 8 * u + line) * 8 + chunk];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <class F>
static float time_it(F f, int reps = 10) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

template <int MASK>
static void run(const u32x4* p, uint64_t nlines, uint32_t* sink, int cus) {
  const float ms = time_it([&] { hipLaunchKernelGGL(rd<MASK>, dim3(cus * 2), dim3(1024), 0, 0, p, nlines, sink); });
  const int touched = 16 * (MASK + 1);
  printf("{\"touched_bytes_per_line\": %d, \"ms\": %.4f, \"full_line_GBps\": %.1f, \"touched_GBps\": %.1f}\n", touched, ms,
         nlines * 128.0 / ms / 1e6, nlines * (double)touched / ms / 1e6);
  fflush(stdout);
}

int main() {
  const uint64_t bytes = 4ull << 30, nlines = bytes / 128;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4* p;
  uint32_t* sink;
  CK(hipMalloc(&p, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(p, 1, bytes));
  run<7>(p, nlines, sink, cus);
  run<3>(p, nlines, sink, cus);
  run<1>(p, nlines, sink, cus);
  run<0>(p, nlines, sink, cus);
  run<7>(p, nlines, sink, cus);
  CK(hipFree(p));
  CK(hipFree(sink));
  return 0;
}
