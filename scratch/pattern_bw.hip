// Pure-load replica of the ICRC kernel's access pattern: groups of G lanes read
// 16G-byte runs of packets at stride S; 64/G packets per wave; block-contiguous.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int LOG2G, int U>
__global__ void __launch_bounds__(1024, 1) pat(const uint8_t* base, uint64_t stride, int len, uint32_t n, int align_runs, uint32_t* sink) {
  constexpr int G = 1 << LOG2G, PPW = 64 / G, DPI = 4 * G;
  const int lane = threadIdx.x & 63, gl = lane & (G - 1), grp = lane >> LOG2G;
  const uint32_t nsets = (n + PPW - 1) / PPW;
  const uint32_t per = (nsets + gridDim.x - 1) / gridDim.x;
  const uint32_t s0 = blockIdx.x * per, s1 = min(nsets, s0 + per);
  uint32_t acc = 0;
  const int ndw = len / 4;
  const int J = (ndw + DPI - 1) / DPI;
  for (uint32_t set = s0 + (threadIdx.x >> 6); set < s1; set += 16) {
    const uint32_t pkt = set * PPW + grp;
    if (pkt >= n) continue;
    const uint8_t* fp = base + (uint64_t)pkt * stride;
    int pad = J * DPI - ndw;
    if (align_runs) { // grid aligned to absolute memory instead of the packet end
      pad = (int)(((uintptr_t)fp >> 2) & (DPI - 1));
    }
    for (int j = 0; j < J; j += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int kb = DPI * (j + u) + 4 * gl - pad;
        if (j + u < J && kb >= 0 && kb + 4 <= ndw) v[u] = __builtin_nontemporal_load((const u32x4*)(fp + 4 * (int64_t)kb));
        else v[u] = u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
  const uint32_t n = 1 << 20;
  const uint64_t bytes = (uint64_t)n * 4160 + 4096;
  uint8_t* d; uint32_t* sink;
  CK(hipMalloc(&d, bytes)); CK(hipMalloc(&sink, 64)); CK(hipMemset(d, 0x5a, bytes));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, double nbytes, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) { CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms); }
    std::sort(ts.begin(), ts.end());
    printf("%-44s med %.3f ms  %.1f GB/s\n", name, ts[3], nbytes / ts[3] / 1e6); fflush(stdout);
  };
  for (uint64_t S : {4096ull, 4140ull, 4160ull}) for (int al = 0; al < 2; ++al) {
    if (S == 4096 && al) continue;
    int len = (int)(S == 4160 ? 4136 : S - 4);
    double nb = (double)n * len;
    char nm[80];
#define RUNG(L) snprintf(nm, 80, "S=%llu G=%d align=%d", (unsigned long long)S, 1 << L, al); run(nm, nb, [&] { hipLaunchKernelGGL((pat<L, 4>), dim3(256), dim3(1024), 0, 0, d, S, len, n, al, sink); });
    RUNG(2) RUNG(3) RUNG(4) RUNG(5) RUNG(6)
  }
  return 0;
}
