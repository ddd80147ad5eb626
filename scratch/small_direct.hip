// cfg5 (2^24 frames of 108 B): can the small-frame kernel drop its LDS
// staging slots (83 KB at 12 waves) so the output ring can hold 3x more
// rounds?  Replica of the kernel's read pattern with the CRC removed:
//   mode 0: coalesced 16-byte loads of a 64-frame batch (kernel today), read only
//   mode 1: "direct": lane f loads its own frame with 7 16-byte loads
//           (4-byte-aligned, 108 B apart across the wave), read only
//   mode 2: coalesced loads + the 4-byte words through an LDS ring of RING
//           rounds flushed between barriers (policy SPOL)
//   mode 3: direct loads + the same ring
// plus a write-only kernel over the 64 MiB of outputs.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/small_direct scratch/small_direct.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                   \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int C = 7;  // 16-byte chunks per lane per 64-frame batch of 108-B frames

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int MODE, int NW, int RING, int LPOL, int SPOL, int BF = 64, int VR = 0>
__global__ void __launch_bounds__(64 * NW, 1) rw(const uint8_t* frames, uint32_t S, uint32_t n,
                                                 uint32_t* out, uint32_t* sink) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int CB = (BF * 108 + 1023) / 1024;  // loads per lane per batch (108-B frames)
  const uint32_t nchunk = BF * S / 16;
  const uint32_t nb = (n + BF - 1) / BF;
  const uint32_t per_block = (nb + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = blockIdx.x * per_block, b1 = min(nb, b0 + per_block);
  const uint32_t nrounds = b1 > b0 ? (b1 - b0 + NW - 1) / NW : 0;
  const auto fr = rsrc(frames, (uint32_t)min<uint64_t>((uint64_t)n * S, 0xFFFFFFF0u));
  constexpr bool kDirect = MODE == 1 || MODE == 3;
  constexpr bool kRing = MODE >= 2;
  auto load = [&](uint32_t b, u32x4* R) {
    b = min(b, b1 - 1);
    if constexpr (kDirect) {
      const uint32_t f = (b * 64u + lane) * S;
#pragma unroll
      for (int t = 0; t < C; ++t)
        R[t] = __builtin_amdgcn_raw_buffer_load_b128(fr, f + 16u * t, 0, LPOL);
    } else {
      const uint32_t base = b * (uint32_t)BF * S;
#pragma unroll
      for (int t = 0; t < CB; ++t)
        R[t] = __builtin_amdgcn_raw_buffer_load_b128(fr, base + 16u * min((uint32_t)(lane + 64 * t), nchunk - 1), 0,
                                                     LPOL);
    }
  };
  uint32_t acc = 0, in_ring = 0, rbase = b0;
  uint32_t vr[VR > 0 ? VR : 1];  // mode 4: the last VR rounds of a window in VGPRs (vr[0] newest)
  const auto orr = rsrc(out, n * 4u);
  auto flush = [&]() {
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    __asm__ __volatile__("" ::: "memory");
    const uint32_t lds_rounds = min(in_ring, (uint32_t)RING);
    const uint32_t words = min(lds_rounds * NW, b1 - rbase) * (uint32_t)BF;
    if constexpr (VR > 0) {  // rounds RING .. in_ring - 1 from the registers, 256 B per store
#pragma unroll
      for (int k = 0; k < VR; ++k) {
        const uint32_t r = in_ring - 1u - (uint32_t)k;
        const uint32_t bb = rbase + r * NW + wave;
        if (r >= (uint32_t)RING && r < in_ring && bb < b1)
          __builtin_amdgcn_raw_buffer_store_b32(vr[k], orr, 4u * (bb * 64u + lane), 0, SPOL);
      }
    }
    for (uint32_t i = tid; i < words / 4; i += NW * 64)
      __builtin_amdgcn_raw_buffer_store_b128(*(const lds_u32x4*)(uintptr_t)(16u * i), orr, 4u * (rbase * (uint32_t)BF) + 16u * i, 0,
                                             SPOL);
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    __asm__ __volatile__("" ::: "memory");
    rbase += in_ring * NW;
    in_ring = 0;
  };
  auto consume = [&](uint32_t r, u32x4* R) {
    u32x4 v = R[0];
#pragma unroll
    for (int t = 1; t < (kDirect ? C : CB); ++t) v ^= R[t];
    const uint32_t w = v.x ^ v.y ^ v.z ^ v.w;
    const uint32_t b = b0 + r * NW + wave;
    load(b + 2 * NW, R);
    if constexpr (!kRing) {
      acc ^= w;
    } else {
      if constexpr (VR > 0) {
        if (in_ring < (uint32_t)RING) {
          *(lds_u32*)(uintptr_t)(4u * (in_ring * NW * BF + wave * BF + lane)) = w;
        } else {
#pragma unroll
          for (int k = VR - 1; k > 0; --k) vr[k] = vr[k - 1];
          vr[0] = w;
        }
        if (++in_ring == RING + VR) flush();
      } else {
        if (lane < BF) *(lds_u32*)(uintptr_t)(4u * (in_ring * NW * BF + wave * BF + lane)) = w;
        if (++in_ring == RING) flush();
      }
    }
  };
  if (nrounds) {
    u32x4 X[C], Y[C];
    load(b0 + wave, X);
    load(b0 + wave + NW, Y);
    for (uint32_t r = 0; r < nrounds; r += 2) {
      consume(r, X);
      if (r + 1 < nrounds) consume(r + 1, Y);
    }
    if (kRing && in_ring) flush();
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void __launch_bounds__(1024) write_only(uint32_t* out, uint64_t nw4) {
  const uint64_t per = (nw4 + gridDim.x - 1) / gridDim.x;
  const uint64_t b = blockIdx.x * per, e = min(nw4, b + per);
  for (uint64_t i = b + threadIdx.x; i < e; i += 1024) ((u32x4*)out)[i] = u32x4{(uint32_t)i, 1, 2, 3};
}

int main() {
  const uint32_t n = 1u << 24, S = 108;
  const uint64_t bytes = (uint64_t)n * S;
  uint8_t* d;
  uint32_t *out, *sink;
  CK(hipMalloc(&d, bytes + 4096));
  CK(hipMalloc(&out, (size_t)n * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(d, 0x5a, bytes));
  CK(hipMemset(out, 0, (size_t)n * 4));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double rb = (double)bytes + 4.0 * n;
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 40; ++w) launch();
    std::vector<float> ts;
    for (int r = 0; r < 30; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-48s med %.4f ms  min %.4f  %.1f GB/s alg\n", name, ts[15], ts[0], rb / ts[15] / 1e6);
    fflush(stdout);
  };
#define RUN(M, W, RG, LP, SP, NAME, BF, ...)                                                            \
  {                                                                                                 \
    auto kf = rw<M, W, RG, LP, SP, BF, ##__VA_ARGS__>;                                                             \
    const size_t lds = (size_t)(RG > 0 ? RG : 1) * W * BF * 4;                                      \
    CK(hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    run(NAME, [&] { hipLaunchKernelGGL(kf, dim3(ncu), dim3(64 * W), lds, 0, d, S, n, out, sink); }); \
  }
  for (int rep = 0; rep < 2; ++rep) {
    RUN(0, 12, 0, 2, 16, "coalesced read-only 12w nt", 64)
    RUN(2, 12, 13, 2, 16, "coalesced + ring 13 sc1 12w", 64)
    RUN(2, 12, 27, 2, 16, "coalesced + ring 27 sc1 12w", 64)
    RUN(2, 12, 13, 2, 16, "coalesced + ring 13 + 8 vgpr sc1 12w", 64, 8)
    RUN(2, 12, 13, 2, 16, "coalesced + ring 13 + 14 vgpr sc1 12w", 64, 14)
    RUN(2, 12, 13, 2, 2, "coalesced + ring 13 + 14 vgpr nt 12w", 64, 14)
    RUN(2, 12, 13, 2, 0, "coalesced + ring 13 + 14 vgpr plain 12w", 64, 14)
  }
  return 0;
}
