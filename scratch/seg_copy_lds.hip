// Segmentation copy pattern with the MR loads going straight into LDS
// (LDS-DMA, global_load_lds_dwordx4) instead of into VGPRs: does holding
// more loads in flight per CU (no VGPRs per load, so more waves or a deeper
// prefetch beside the ~200-VGPR fold) lift the pattern's rate?  2^20 packets,
// 4096 MR bytes -> 4096 frame bytes in 4224-byte slots (dword-aligned MR
// reads: the replica in seg_copy.hip measured the 40-B header offset free),
// groups of 8 lanes per packet, 8 packets per wave set.  Per wave: two LDS
// buffers of U KiB (one KiB = one wave-instruction: 64 lanes x 16 B); block b
// + 1's loads are issued, block b is read back from LDS and stored (nt).
// GB/s = (MR bytes + frame bytes) / median time; the VGPR version beside it.
// build: hipcc --offload-arch=gfx950 -O3 -o scratch/seg_copy_lds scratch/seg_copy_lds.hip
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

constexpr uint32_t kMsg = 4096, kSlot = 4224;
constexpr int kJ = kMsg / 128;  // iterations per packet (128 B per group of 8)

// s_waitcnt with vmcnt = N (< 64), expcnt and lgkmcnt left open
#define WAIT_VM(N) __builtin_amdgcn_s_waitcnt(0x0F70 | ((N) & 0xF) | (((N) >> 4) << 14))

template <int U, int W>
__global__ void __launch_bounds__(64 * W, 1) segcopy_lds(const uint8_t* mr, uint8_t* out, uint32_t n) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];
  constexpr int NB = kJ / U;
  static_assert(kJ % U == 0, "whole blocks");
  const int lane = threadIdx.x & 63, gl = lane & 7, grp = lane >> 3;
  const uint32_t wave = threadIdx.x >> 6;
  uint8_t* buf = lds + wave * (2u * U * 1024u);
  const uint32_t nsets = n / 8;
  const uint32_t per = (nsets + gridDim.x - 1) / gridDim.x;
  const uint32_t s0 = blockIdx.x * per, s1 = min(nsets, s0 + per);
  for (uint32_t set = s0 + wave; set < s1; set += W) {
    const uint32_t pkt = set * 8 + grp;
    const uint8_t* src = mr + (uint64_t)pkt * kMsg + 16 * gl;
    uint8_t* dst = out + (uint64_t)pkt * kSlot + 16 * gl;
    auto issue = [&](int b) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(src + 128 * (b * U + u)),
            (__attribute__((address_space(3))) void*)(buf + ((b & 1) * U + u) * 1024u), 16, 0, 0);
    };
    issue(0);
    for (int b = 0; b < NB; ++b) {
      if (b + 1 < NB) {
        issue(b + 1);
        WAIT_VM(U);  // block b has landed (block b + 1's U loads stay in flight)
      } else {
        WAIT_VM(0);
      }
      __asm__ __volatile__("" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const u32x4 v = *(const u32x4*)(buf + ((b & 1) * U + u) * 1024u + 16u * lane);
        __builtin_nontemporal_store(v, (u32x4*)(dst + 128 * (b * U + u)));
      }
      __asm__ __volatile__("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): reads done before the buffer is refilled
    }
  }
}

template <int U, int W>
__global__ void __launch_bounds__(64 * W, 1) segcopy_vgpr(const uint8_t* mr, uint8_t* out, uint32_t n) {
  constexpr int NB = kJ / U;
  const int lane = threadIdx.x & 63, gl = lane & 7, grp = lane >> 3;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t nsets = n / 8;
  const uint32_t per = (nsets + gridDim.x - 1) / gridDim.x;
  const uint32_t s0 = blockIdx.x * per, s1 = min(nsets, s0 + per);
  for (uint32_t set = s0 + wave; set < s1; set += W) {
    const uint32_t pkt = set * 8 + grp;
    const u32x4* src = (const u32x4*)(mr + (uint64_t)pkt * kMsg + 16 * gl);
    u32x4* dst = (u32x4*)(out + (uint64_t)pkt * kSlot + 16 * gl);
    u32x4 X[U], Y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) X[u] = __builtin_nontemporal_load(src + 8 * u);
    for (int b = 0; b < NB; b += 2) {
      if (b + 1 < NB) {
#pragma unroll
        for (int u = 0; u < U; ++u) Y[u] = __builtin_nontemporal_load(src + 8 * ((b + 1) * U + u));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_nontemporal_store(X[u], dst + 8 * (b * U + u));
      if (b + 1 >= NB) break;
      if (b + 2 < NB) {
#pragma unroll
        for (int u = 0; u < U; ++u) X[u] = __builtin_nontemporal_load(src + 8 * ((b + 2) * U + u));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_nontemporal_store(Y[u], dst + 8 * ((b + 1) * U + u));
    }
  }
}

template <class F>
static float time_it(F f, int reps = 15) {
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

static const uint8_t* g_mr;
static uint8_t* g_out;
static uint32_t g_n;
static int g_cus;

template <int U, int W>
static void run_lds() {
  const size_t lds = (size_t)W * 2 * U * 1024;
  if (lds > 160 * 1024) return;
  CK(hipFuncSetAttribute((const void*)segcopy_lds<U, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  auto go = [&] { hipLaunchKernelGGL((segcopy_lds<U, W>), dim3(g_cus), dim3(64 * W), lds, 0, g_mr, g_out, g_n); };
  go();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const float ms = time_it(go);
  printf("{\"kernel\": \"lds-dma\", \"U\": %d, \"waves\": %d, \"lds_KiB\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", U, W,
         lds / 1024, ms, 2.0 * g_n * kMsg / ms / 1e6);
  fflush(stdout);
}

template <int U, int W>
static void run_vgpr() {
  auto go = [&] { hipLaunchKernelGGL((segcopy_vgpr<U, W>), dim3(g_cus), dim3(64 * W), 0, 0, g_mr, g_out, g_n); };
  go();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const float ms = time_it(go);
  printf("{\"kernel\": \"vgpr\", \"U\": %d, \"waves\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", U, W, ms,
         2.0 * g_n * kMsg / ms / 1e6);
  fflush(stdout);
}

int main() {
  g_n = 1u << 20;
  CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *mr, *out;
  CK(hipMalloc(&mr, (size_t)g_n * kMsg));
  CK(hipMalloc(&out, (size_t)g_n * kSlot));
  CK(hipMemset(mr, 0x5A, (size_t)g_n * kMsg));
  CK(hipMemset(out, 0, (size_t)g_n * kSlot));
  g_mr = mr;
  g_out = out;
  // correctness of the LDS path once: every frame byte equals its MR byte
  {
    CK(hipMemset(out, 0, (size_t)g_n * kSlot));
    std::vector<uint8_t> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
    CK(hipMemcpy(mr + (size_t)12345 * kMsg, h.data(), 4096, hipMemcpyHostToDevice));
    run_lds<4, 8>();
    std::vector<uint8_t> g(4096);
    CK(hipMemcpy(g.data(), out + (size_t)12345 * kSlot, 4096, hipMemcpyDeviceToHost));
    printf("{\"lds_copy_bit_exact\": %s}\n", g == h ? "true" : "false");
  }
  for (int rep = 0; rep < 2; ++rep) {
    run_vgpr<4, 8>();
    run_vgpr<4, 16>();
    run_lds<4, 8>();
    run_lds<8, 8>();
    run_lds<4, 12>();
    run_lds<4, 16>();
    run_lds<2, 16>();
    run_lds<8, 4>();
    run_lds<16, 4>();
  }
  CK(hipFree(mr));
  CK(hipFree(out));
  return 0;
}
