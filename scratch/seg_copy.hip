// Copy-only replica of the segmentation kernel's memory pattern (no CRC, no
// headers): 2^20 packets, each 4096 MR bytes -> a 4140-byte frame (payload at
// frame byte 40) in a 4352-byte slot.  Groups of G lanes per packet, 64/G
// packets per wave set; iteration j of lane i reads the 16 MR bytes at
// frame dword 4(Gj + i) - 10 (unaligned by the 40-B header) and writes frame
// bytes 16(Gj + i) with one aligned 16-B store; U iterations per block, two
// blocks in flight (ping-pong), W waves per CU.  Question: does the width of
// a packet's contiguous write (16G bytes per instruction) decide the rate?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t kMsg = 4096;

template <int LOG2G, int U, int W, int POL>
__global__ void __launch_bounds__(64 * W, 1) segcopy(const uint8_t* mr, uint8_t* out, uint32_t n, int kHdr, int kFrame,
                                                        uint32_t kSlot) {
  constexpr int G = 1 << LOG2G, PPW = 64 / G, DPI = 16 * G;  // bytes per iteration per packet
  const int J = (kFrame + DPI - 1) / DPI;
  const int NB = (J + U - 1) / U;
  const int lane = threadIdx.x & 63, gl = lane & (G - 1), grp = lane >> LOG2G;
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t nsets = (n + PPW - 1) / PPW;
  const uint32_t per = (nsets + gridDim.x - 1) / gridDim.x;
  const uint32_t s0 = blockIdx.x * per, s1 = min(nsets, s0 + per);
  for (uint32_t set = s0 + wave; set < s1; set += W) {
    const uint32_t pkt = min(set * PPW + grp, n - 1);
    const uint8_t* src = mr + (uint64_t)pkt * kMsg;
    uint8_t* dst = out + (uint64_t)pkt * kSlot;
    auto ld = [&](int j) -> u32x4 {
      const int jj = min(j, J - 1);
      int o = DPI * jj + 16 * gl - kHdr;
      o = max(0, min(o, (int)kMsg - 16));
      return *(const u32x4_u*)(src + o);
    };
    auto st = [&](int j, const u32x4& v) {
      const int o = DPI * j + 16 * gl;
      if (j < J && o < kFrame) {
        if (POL == 2)
          __builtin_nontemporal_store(v, (u32x4*)(dst + o));
        else
          *(u32x4*)(dst + o) = v;
      }
    };
    u32x4 X[U], Y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) Y[u] = ld(u);
#pragma unroll
    for (int u = 0; u < U; ++u) X[u] = ld(U + u);
#pragma unroll
    for (int u = 0; u < U; ++u) st(u, Y[u]);
    for (int b = 1; b < NB; b += 2) {
#pragma unroll
      for (int u = 0; u < U; ++u) Y[u] = ld((b + 1) * U + u);
#pragma unroll
      for (int u = 0; u < U; ++u) st(b * U + u, X[u]);
      if (b + 1 >= NB) break;
#pragma unroll
      for (int u = 0; u < U; ++u) X[u] = ld((b + 2) * U + u);
#pragma unroll
      for (int u = 0; u < U; ++u) st((b + 1) * U + u, Y[u]);
    }
  }
}

// Plain stream copy of the same byte count, for the ceiling.
__global__ void __launch_bounds__(1024) stream_copy(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    __builtin_nontemporal_store(a, d + i);
    __builtin_nontemporal_store(b, d + i + stride);
    __builtin_nontemporal_store(c, d + i + 2 * stride);
    __builtin_nontemporal_store(e, d + i + 3 * stride);
  }
  for (; i < n16; i += stride) d[i] = s[i];
}

// One event pair around `reps` launches (a pair per launch drains each
// launch's writes at the release, round 5), mean ms per launch.
template <class F>
static float time_it(F f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

// Round 6: one packet per wave at a time, streamed: a wave owns a contiguous
// range of packets and walks its (packet, 1-KiB chunk) sequence with loads U
// chunks ahead across packet boundaries (no per-set restart); chunk j of
// packet p: lane i reads MR bytes 1024 j + 16 i - hdr of the packet (clamped
// into the packet) and writes slot bytes 1024 j + 16 i while < the frame
// rounded up to 128 B.
template <int U, int W>
__global__ void __launch_bounds__(64 * W, 1) segstream(const uint8_t* mr, uint8_t* out, uint32_t n, int kHdr,
                                                          int kFrame, uint32_t kSlot) {
  const int lane = threadIdx.x & 63;
  const int C = (kFrame + 1023) / 1024;          // chunks per packet
  const int fr = (kFrame + 127) & ~127;          // bytes written per packet
  const uint32_t nw = gridDim.x * W;
  const uint32_t wid = blockIdx.x * W + (threadIdx.x >> 6);
  const uint32_t per = (n + nw - 1) / nw;
  const uint32_t p0 = wid * per, p1 = min(n, p0 + per);
  if (p0 >= p1) return;
  const uint32_t T = (p1 - p0) * C;
  auto ld = [&](uint32_t t) -> u32x4 {
    t = min(t, T - 1);
    const uint32_t p = p0 + t / C, j = t % C;
    int o = 1024 * (int)j + 16 * lane - kHdr;
    o = max(0, min(o, (int)kMsg - 16));
    return *(const u32x4_u*)(mr + (uint64_t)p * kMsg + o);
  };
  u32x4 R[U];
#pragma unroll
  for (int u = 0; u < U; ++u) R[u] = ld(u);
  for (uint32_t t = 0; t < T; t += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t tt = t + u;
      const u32x4 v = R[u];
      R[u] = ld(tt + U);
      if (tt < T) {
        const uint32_t p = p0 + tt / C, j = tt % C;
        const int o = 1024 * (int)j + 16 * lane;
        if (o < fr) __builtin_nontemporal_store(v, (u32x4*)(out + (uint64_t)p * kSlot + o));
      }
    }
  }
}

template <int U, int W>
static void run_stream(const uint8_t* mr, uint8_t* out, uint32_t n, int cus, int hdr, int frame, uint32_t slot) {
  auto go = [&] { hipLaunchKernelGGL((segstream<U, W>), dim3(cus), dim3(64 * W), 0, 0, mr, out, n, hdr, frame, slot); };
  go();
  CK(hipGetLastError());
  const float ms = time_it(go);
  const double bytes = (double)n * kMsg + (double)n * frame;
  printf("{\"kernel\": \"segstream\", \"hdr\": %d, \"frame\": %d, \"slot\": %u, \"U\": %d, \"waves\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
         hdr, frame, slot, U, W, ms, bytes / ms / 1e6);
  fflush(stdout);
}

template <int LOG2G, int U, int W, int POL>
static void run(const uint8_t* mr, uint8_t* out, uint32_t n, int cus, int hdr, int frame, uint32_t slot) {
  hipLaunchKernelGGL((segcopy<LOG2G, U, W, POL>), dim3(cus), dim3(64 * W), 0, 0, mr, out, n, hdr, frame, slot);  // warm + check launch
  CK(hipGetLastError());
  const float ms = time_it([&] { hipLaunchKernelGGL((segcopy<LOG2G, U, W, POL>), dim3(cus), dim3(64 * W), 0, 0, mr, out, n, hdr, frame, slot); });
  const double bytes = (double)n * kMsg + (double)n * frame;
  printf("{\"kernel\": \"segcopy\", \"hdr\": %d, \"frame\": %d, \"slot\": %u, \"G\": %d, \"U\": %d, \"waves\": %d, \"pol\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
         hdr, frame, slot, 1 << LOG2G, U, W, POL, ms, bytes / ms / 1e6);
  fflush(stdout);
}

int main() {
  const uint32_t n = 1u << 20;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *mr, *out;
  CK(hipMalloc(&mr, (size_t)n * kMsg));
  CK(hipMalloc(&out, (size_t)n * 4352));
  CK(hipMemset(mr, 0x5A, (size_t)n * kMsg));
  CK(hipMemset(out, 0, (size_t)n * 4352));
  const uint64_t n16 = (uint64_t)n * kMsg / 16;
  const float sc = time_it([&] { hipLaunchKernelGGL(stream_copy, dim3(cus), dim3(1024), 0, 0, (const u32x4*)mr, (u32x4*)out, n16); });
  printf("{\"kernel\": \"stream_copy\", \"ms\": %.4f, \"GBps\": %.1f}\n", sc, 2.0 * n16 * 16 / sc / 1e6);
  // round 6: loads in flight per lane (U) x waves per CU at the shipped
  // geometry (40-B header, 4140-B frames, 4224-B slots), 3 rounds
  for (int r = 0; r < 3; ++r) {
    run<3, 4, 8, 2>(mr, out, n, cus, 40, 4140, 4224);
    run<3, 4, 8, 2>(mr, out, n, cus, 0, 4096, 4096);
    run_stream<4, 8>(mr, out, n, cus, 40, 4140, 4224);
    run_stream<8, 8>(mr, out, n, cus, 40, 4140, 4224);
    run_stream<4, 16>(mr, out, n, cus, 40, 4140, 4224);
    run_stream<8, 16>(mr, out, n, cus, 40, 4140, 4224);
    run_stream<4, 8>(mr, out, n, cus, 0, 4096, 4096);
    run_stream<8, 16>(mr, out, n, cus, 0, 4096, 4096);
  }
  CK(hipFree(mr));
  CK(hipFree(out));
  return 0;
}
