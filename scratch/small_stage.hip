// cfg5 (2^24 frames of 108 B): does staging the 64-frame batches into LDS
// with LDS-DMA (global_load_lds_dwordx4, no ds_write and no prefetch
// registers) beat today's loads-into-VGPRs-then-ds_write staging?  Replica of
// the small kernel's memory pattern with the CRC replaced by an XOR of each
// lane's 27 frame dwords read from LDS, the 4-byte words collected in an LDS
// ring of RING rounds and flushed between barriers with sc1 stores (as the
// kernel does):
//   mode 0: VGPR staging, one slot per wave, two batches prefetched in VGPRs
//   mode 1: LDS-DMA staging, two slots per wave (batch b + 1 in flight while
//           batch b is read)
// build: hipcc --offload-arch=gfx950 -O3 -o scratch/small_stage scratch/small_stage.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                    \
    }                                                             \
  } while (0)

constexpr uint32_t S = 108, kBatch = 64 * S, kChunks = kBatch / 16;  // 432 chunks
constexpr int C = 7;                                                 // loads per lane per batch
constexpr uint32_t kSlot = C * 1024;                                 // 7 KiB per staging slot
#define WAIT_VM(N) __builtin_amdgcn_s_waitcnt(0x0F70 | ((N) & 0xF) | (((N) >> 4) << 14))

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// LDS: [tables: 32 KiB if LK][slots: NW * NS * 7 KiB][ring: RING rounds * NW * 256 B]
//   mode 2 (round 4): ONE slot per wave filled by LDS-DMA; a round reads its
//   lane's 27 frame dwords into VGPRs, then refills the slot with the next
//   batch (in flight during the fold), then folds from the registers.
//   LK: table lookups per dword emulating the fold (4 chains, conflict-free
//   32-copy addressing); 0 = a plain XOR.
template <int MODE, int NW, int RING, int LK = 0>
__global__ void __launch_bounds__(64 * NW, 1) stage(const uint8_t* frames, uint32_t n, uint32_t* out) {
  constexpr int NS = MODE == 1 ? 2 : 1;
  constexpr uint32_t kTab = LK ? 32768u : 0u;
  constexpr uint32_t kRing = kTab + NW * NS * kSlot;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t nb = n / 64;
  const uint32_t per = (nb + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = blockIdx.x * per, b1 = min(nb, b0 + per);
  const uint32_t nrounds = b1 > b0 ? (b1 - b0 + NW - 1) / NW : 0;
  const auto fr = rsrc(frames, (uint32_t)min<uint64_t>((uint64_t)n * S, 0xFFFFFFF0u));
  const auto orr = rsrc(out, n * 4u);
  const uint32_t slot0 = kTab + (uint32_t)wave * NS * kSlot;
  if constexpr (LK > 0) {  // table (byte e, copy c) = e * 128 + c * 4: any value
    for (uint32_t i = tid; i < 8192u; i += NW * 64) *(lds_u32*)(uintptr_t)(4u * i) = i * 2654435761u;
    __syncthreads();
  }
  const uint32_t kc = (uint32_t)(lane & 31) * 4u;
  // the emulated fold of dword w into chain register x
  auto absorb = [&](uint32_t x, uint32_t w) {
    x ^= w;
    if constexpr (LK == 0) return x;
    uint32_t y = 0;
#pragma unroll
    for (int q = 0; q < LK; ++q) y ^= *(const lds_u32*)(uintptr_t)(((x >> (8 * q)) & 0xFFu) * 128u + kc);
    return y;
  };
  // chunk t of lane: batch chunk lane + 64 t (clamped to the batch's last)
  auto chunk_off = [&](uint32_t b, int t) { return b * kBatch + 16u * min((uint32_t)(lane + 64 * t), kChunks - 1); };
  uint32_t in_ring = 0, rbase = b0;
  auto flush = [&]() {
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    __asm__ __volatile__("" ::: "memory");
    const uint32_t words = min(in_ring * NW, b1 - rbase) * 64u;
    for (uint32_t i = tid; i < words / 4; i += NW * 64)
      __builtin_amdgcn_raw_buffer_store_b128(*(const lds_u32x4*)(uintptr_t)(kRing + 16u * i), orr,
                                             4u * (rbase * 64u) + 16u * i, 0, 16);
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    __asm__ __volatile__("" ::: "memory");
    rbase += in_ring * NW;
    in_ring = 0;
  };
  // the "fold": lane f XORs its frame's 27 dwords from the slot
  auto fold_regs = [&](const uint32_t* d) {
    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < (int)(S / 4); ++k) c[k & 3] = absorb(c[k & 3], d[k]);
    const uint32_t w = c[0] ^ c[1] ^ c[2] ^ c[3];
    *(lds_u32*)(uintptr_t)(kRing + 4u * (in_ring * NW * 64u + wave * 64u + lane)) = w;
    if (++in_ring == RING) flush();
  };
  auto fold = [&](uint32_t slot, uint32_t r) {
    uint32_t d[S / 4];
#pragma unroll
    for (int k = 0; k < (int)(S / 4); ++k) d[k] = *(const lds_u32*)(uintptr_t)(slot + S * lane + 4u * k);
    fold_regs(d);
  };
  if (nrounds == 0) return;  // (the whole workgroup: b0 >= b1 for every wave)
  if constexpr (MODE == 0) {
    u32x4 X[C], Y[C];
    auto load = [&](uint32_t b, u32x4* R) {
      b = min(b, b1 - 1);
#pragma unroll
      for (int t = 0; t < C; ++t) R[t] = __builtin_amdgcn_raw_buffer_load_b128(fr, chunk_off(b, t), 0, 2);
    };
    auto put = [&](const u32x4* R) {
#pragma unroll
      for (int t = 0; t < C; ++t) *(lds_u32x4*)(uintptr_t)(slot0 + 1024u * t + 16u * lane) = R[t];
    };
    load(b0 + wave, X);
    load(b0 + wave + NW, Y);
    for (uint32_t r = 0; r < nrounds; r += 2) {
      put(X);
      load(b0 + (r + 2) * NW + wave, X);
      fold(slot0, r);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (r + 1 < nrounds) {
        put(Y);
        load(b0 + (r + 3) * NW + wave, Y);
        fold(slot0, r + 1);
        __builtin_amdgcn_s_waitcnt(0xC07F);
      }
    }
  } else if constexpr (MODE == 2) {
    auto issue = [&](uint32_t b) {
      b = min(b, b1 - 1);
#pragma unroll
      for (int t = 0; t < C; ++t)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(frames + chunk_off(b, t)),
                                         (__attribute__((address_space(3))) void*)(uintptr_t)(slot0 + 1024u * t), 16, 0,
                                         0);
    };
    issue(b0 + wave);
    for (uint32_t r = 0; r < nrounds; ++r) {
      WAIT_VM(0);  // batch r has landed in the slot
      __asm__ __volatile__("" ::: "memory");
      uint32_t d[S / 4];
#pragma unroll
      for (int k = 0; k < (int)(S / 4); ++k) d[k] = *(const lds_u32*)(uintptr_t)(slot0 + S * lane + 4u * k);
      __asm__ __volatile__("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0xC07F);  // the slot is read: refill it
      __asm__ __volatile__("" ::: "memory");
      issue(b0 + (r + 1) * NW + wave);
      fold_regs(d);
    }
    WAIT_VM(0);
  } else {
    // batch chunk lane + 64 t lands at slot + 1024 t + 16 lane (the DMA's
    // per-lane LDS address); frame f's bytes therefore sit at slot + 108 f
    auto issue = [&](uint32_t b, uint32_t slot) {
      b = min(b, b1 - 1);
#pragma unroll
      for (int t = 0; t < C; ++t)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(frames + chunk_off(b, t)),
                                         (__attribute__((address_space(3))) void*)(uintptr_t)(slot + 1024u * t), 16, 0,
                                         0);
    };
    issue(b0 + wave, slot0);
    for (uint32_t r = 0; r < nrounds; ++r) {
      const uint32_t cur = slot0 + (r & 1u) * kSlot, nxt = slot0 + ((r + 1) & 1u) * kSlot;
      if (r + 1 < nrounds) {
        issue(b0 + (r + 1) * NW + wave, nxt);
        WAIT_VM(C);  // batch r has landed; batch r + 1 stays in flight
      } else {
        WAIT_VM(0);
      }
      __asm__ __volatile__("" ::: "memory");
      fold(cur, r);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // slot `cur` read before it is refilled
      __asm__ __volatile__("" ::: "memory");
    }
  }
  if (in_ring) flush();
}

int main() {
  const uint32_t n = 1u << 24;
  const uint64_t bytes = (uint64_t)n * S;
  uint8_t* d;
  uint32_t *out, *ref;
  CK(hipMalloc(&d, bytes + 4096));
  CK(hipMalloc(&out, (size_t)n * 4));
  CK(hipMalloc(&ref, (size_t)n * 4));
  {
    std::vector<uint32_t> h(bytes / 4);
    uint32_t x = 1;
    for (auto& v : h) v = x = x * 1664525u + 1013904223u;
    CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
  }
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double rb = (double)bytes + 4.0 * n;
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 20; ++w) launch();
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
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"min_ms\": %.4f, \"GBps_alg\": %.1f}\n", name, ts[15], ts[0],
           rb / ts[15] / 1e6);
    fflush(stdout);
  };
#define RUN(M, W, RG, NAME, DST) RUNL(M, W, RG, 0, NAME, DST)
#define RUNL(M, W, RG, LK, NAME, DST)                                                                     \
  {                                                                                                       \
    auto kf = stage<M, W, RG, LK>;                                                                        \
    const size_t lds = (LK ? 32768 : 0) + (size_t)W * (M == 1 ? 2 : 1) * kSlot + (size_t)RG * W * 256;    \
    if (lds <= 160 * 1024) {                                                                              \
      CK(hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));     \
      run(NAME, [&] { hipLaunchKernelGGL(kf, dim3(ncu), dim3(64 * W), lds, 0, d, n, DST); });              \
    }                                                                                                     \
  }
  // the two modes must produce the same words
  RUN(0, 12, 13, "vgpr staging 12w ring 13", ref)
  RUN(1, 8, 24, "lds-dma staging 8w 2 slots ring 24", out)
  {
    std::vector<uint32_t> x(n), y(n);
    CK(hipMemcpy(x.data(), ref, (size_t)n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
    printf("{\"words_equal\": %s}\n", x == y ? "true" : "false");
  }
  // round 4: DMA into one slot per wave, frames read to VGPRs before the refill
  RUN(2, 12, 13, "lds-dma one slot 12w ring 13", out)
  {
    std::vector<uint32_t> x(n), y(n);
    CK(hipMemcpy(x.data(), ref, (size_t)n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
    printf("{\"words_equal_mode2\": %s}\n", x == y ? "true" : "false");
  }
  RUNL(0, 12, 12, 4, "fold-emulated vgpr staging 12w ring 12", ref)
  RUNL(2, 12, 12, 4, "fold-emulated lds-dma one slot 12w ring 12", out)
  {
    std::vector<uint32_t> x(n), y(n);
    CK(hipMemcpy(x.data(), ref, (size_t)n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), out, (size_t)n * 4, hipMemcpyDeviceToHost));
    printf("{\"words_equal_fold\": %s}\n", x == y ? "true" : "false");
  }
  for (int rep = 0; rep < 2; ++rep) {
    RUNL(0, 12, 12, 4, "fold-emulated vgpr staging 12w ring 12", out)
    RUNL(2, 12, 12, 4, "fold-emulated lds-dma one slot 12w ring 12", out)
    RUNL(2, 14, 5, 4, "fold-emulated lds-dma one slot 14w ring 5", out)
    RUNL(2, 10, 20, 4, "fold-emulated lds-dma one slot 10w ring 20", out)
    RUN(2, 12, 13, "lds-dma one slot 12w ring 13", out)
    RUN(2, 16, 8, "lds-dma one slot 16w ring 8", out)
  }
  for (int rep = 0; rep < 2; ++rep) {
    RUN(0, 12, 13, "vgpr staging 12w ring 13", out)
    RUN(0, 8, 24, "vgpr staging 8w ring 24", out)
    RUN(1, 8, 24, "lds-dma staging 8w 2 slots ring 24", out)
    RUN(1, 8, 16, "lds-dma staging 8w 2 slots ring 16", out)
    RUN(1, 10, 10, "lds-dma staging 10w 2 slots ring 10", out)
    RUN(1, 6, 40, "lds-dma staging 6w 2 slots ring 40", out)
  }
  return 0;
}
