// ICRC fault injection for batches of wire frames (gfx950).
//
// The reference corrupts single packets from Python hooks registered through
// SideServicer.SetHook (src/sanity_side.py:345-364; the hook functions live in
// src/hooks.py:10-138 and mutate BTH / RETH / AETH fields or the payload
// before the packet is built).  It has no ICRC error case because it never
// checks the ICRC on receive.  This kernel provides that case at batch scale:
// a seed-determined subset of frames is corrupted in place so that the verify
// path (ricrc_verify_batch[_dev]) can be exercised on millions of frames with
// a known expected outcome per frame.
//
// One thread per packet; a few bytes per packet are touched, so the kernel is
// bound by the per-packet descriptor loads, not by HBM bandwidth.
#include "icrc_internal.hpp"
#include "roce_icrc.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ricrc {

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Masked byte positions of the ICRC rule (src/roce.py:204-211) for IHL `ihl`.
__device__ __forceinline__ bool masked_byte(uint32_t pos, uint32_t u) {
  return pos == 1 || pos == 8 || pos == 10 || pos == 11 || pos == u + 6 || pos == u + 7 ||
         pos == u + 12;
}

__global__ void __launch_bounds__(256) fault_kernel(FaultArgs a) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
    const uint64_t h = splitmix64(a.seed ^ ((uint64_t)i * 0xD1B54A32D192ED03ull));
    uint8_t kind = 0;
    const uint32_t L = a.lens[i];
    uint8_t* f = a.frames + a.offsets[i];
    const uint32_t ihl4 = L >= 1 ? 4u * (f[0] & 0xFu) : 0u;
    const bool usable = L >= 44 && L <= 65535 && (L & 3u) == 0 && (f[0] >> 4) == 4 &&
                        ihl4 >= 20 && ihl4 + 24 <= L;
    if (usable && (uint32_t)(h % 1000000ull) < a.rate_ppm) {
      // the k-th enabled kind, k drawn from the hash
      const uint32_t kinds = a.kinds & (RICRC_FAULT_ICRC | RICRC_FAULT_PAYLOAD | RICRC_FAULT_MASKED);
      const uint32_t cnt = __builtin_popcount(kinds);
      if (cnt) {
        uint32_t k = (uint32_t)((h >> 20) % cnt), m = kinds;
        for (; k; --k) m &= m - 1;
        kind = (uint8_t)(m & (0u - m));
      }
      const uint32_t r = (uint32_t)(h >> 32);
      if (kind == RICRC_FAULT_ICRC) {
        const uint32_t bit = r & 31u;
        f[L - 4 + (bit >> 3)] ^= (uint8_t)(1u << (bit & 7u));
      } else if (kind == RICRC_FAULT_PAYLOAD) {
        uint32_t pos = r % (L - 4);
        if (masked_byte(pos, ihl4)) pos = ihl4 + 8;  // the BTH opcode byte instead
        f[pos] ^= (uint8_t)(1u << ((h >> 56) & 7u));
      } else if (kind == RICRC_FAULT_MASKED) {
        const uint64_t v = splitmix64(h);
        f[1] = (uint8_t)v;                // IP tos
        f[8] = (uint8_t)(v >> 8);         // IP ttl
        f[10] = (uint8_t)(v >> 16);       // IP header checksum
        f[11] = (uint8_t)(v >> 24);
        f[ihl4 + 6] = (uint8_t)(v >> 32);  // UDP checksum
        f[ihl4 + 7] = (uint8_t)(v >> 40);
        f[ihl4 + 12] = (uint8_t)(v >> 48);  // BTH fecn | becn | resv6
      }
    }
    if (a.fault_out) a.fault_out[i] = kind;
  }
}

}  // namespace

hipError_t launch_faults(const FaultArgs& a, int num_cus, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  uint64_t blocks = (a.n + 255u) / 256u;
  const uint64_t cap = (uint64_t)num_cus * 16u;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(fault_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace ricrc
