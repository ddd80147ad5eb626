// RoCEv2 ICRC kernels for MI355X (gfx950, CDNA4).
//
// Computes, per wire frame, the Invariant CRC of datenlord/roce-sim's
// BTH.compute_icrc (src/roce.py:192-223): zlib CRC-32 of
// FF x 8 || frame[0 : len-4] with IP tos/ttl/chksum, UDP chksum and the BTH
// fecn|becn|resv6 byte forced to ones (src/roce.py:204-211).
//
// Work decomposition ("end-aligned dword grid").  A group of G lanes
// (G = 1 .. 64, a power of two) owns one packet.  The packet's n covered
// dwords are laid on a grid of J iterations x 4G dwords whose LAST dword is
// the packet's last covered dword (pad = 4GJ - n zero dwords at the front,
// which do not change a zero-initialised CRC register).  In iteration j, lane
// i of the group reads the 16 contiguous bytes at grid dwords 4Gj + 4i .. +3
// with one dwordx4 load, so a group reads 16G contiguous bytes per
// instruction and a wave reads 64/G such runs.  Each lane keeps four CRC
// registers a_t (t = grid column inside the lane) and folds
//
//      a_t <- Mul(128 G)(a_t ^ w_t)          (= "w_t followed by 16G-4 zero bytes")
//
// where Mul(m) is multiplication by x^m mod P on the reflected register,
// evaluated as four byte-indexed table lookups from LDS.  At the end the
// register of grid column s = 4i + t is off by exactly x^(32 s), so the
// packet CRC is  R = sum_s Mul(-32 s)(a_s): three in-lane Horner steps with
// Mul(-32) and log2 G cross-lane butterfly levels with Mul(-128 * 2^l)
// (__shfl_xor inside the group).  No MFMA: this is a byte scan, bound by HBM.
//
// LDS (per workgroup, one 1024-thread workgroup per CU):
//   [0, 128 KiB)  Mul(128 G) tables replicated 32x so every lane of a
//                 ds_read_b32 half-wave hits its own bank:
//                 addr(tab, e, lane) = (tab >> 1) * 64 KiB + e * 256
//                                      + (tab & 1) * 128 + (lane & 31) * 4
//                 (bank = lane & 31, conflict-free); the address is ONE
//                 v_perm_b32 of the register and a per-lane constant.
//   [128 KiB, +4 KiB * (1 + log2 G))  combine tables, unreplicated.
//
// Masks, seed: the masked dwords are packet dwords 0 (TOS), 2 (TTL, IP csum),
// IHL+1 (UDP csum) and IHL+3 (BTH byte 4); the FF x 8 prefix is folded in as
// the CRC register 0xDEBB20E3 XORed into dword 0.  They are applied in the
// peeled "head" iterations; the body loop is plain loads.
#include "icrc_internal.hpp"
#include "gf2.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ricrc {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

constexpr uint32_t kLdsMain = 131072;
constexpr int kUnroll = 4;  // iterations per body block (dwordx4 loads in flight per lane)

__device__ __forceinline__ uint32_t lds_rd(uint32_t byte_addr) {
  return *(const lds_u32*)(uintptr_t)byte_addr;
}
__device__ __forceinline__ void lds_wr(uint32_t byte_addr, uint32_t v) {
  *(lds_u32*)(uintptr_t)byte_addr = v;
}
__device__ __forceinline__ void lds_wr4(uint32_t byte_addr, uint32_t v) {
  *(lds_u32x4*)(uintptr_t)byte_addr = u32x4{v, v, v, v};
}

__device__ __forceinline__ uint32_t ldg32(const uint8_t* p) {
  return *(const uint32_t*)p;
}
// 16-byte load from a 4-byte-aligned address (frames are only dword aligned;
// gfx950 runs global loads in unaligned mode).
__device__ __forceinline__ u32x4 ldg128(const uint8_t* p) {
  return *(const u32x4*)p;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Mul(128 G)(x) from the replicated LDS tables.
__device__ __forceinline__ uint32_t mul_main(uint32_t x, uint32_t kc0, uint32_t kc1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, kc0, 0x0C0C0400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, kc0, 0x0C0C0500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, kc1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, kc1, 0x0C020700u);
  const uint32_t t0 = lds_rd(a0);
  const uint32_t t1 = lds_rd(a1 + 128);
  const uint32_t t2 = lds_rd(a2);
  const uint32_t t3 = lds_rd(a3 + 128);
  return xor3(t0, t1, t2) ^ t3;
}

// Mul(m)(x) from an unreplicated combine set at LDS byte address `base`.
__device__ __forceinline__ uint32_t mul_comb(uint32_t x, uint32_t base) {
  const uint32_t t0 = lds_rd(base + ((x << 2) & 0x3FCu));
  const uint32_t t1 = lds_rd(base + 1024 + ((x >> 6) & 0x3FCu));
  const uint32_t t2 = lds_rd(base + 2048 + ((x >> 14) & 0x3FCu));
  const uint32_t t3 = lds_rd(base + 3072 + ((x >> 22) & 0x3FCu));
  return xor3(t0, t1, t2) ^ t3;
}

constexpr uint32_t kPktBadLen = 0x01, kPktNotIpv4 = 0x02, kPktNotUdp = 0x04,
                   kPktLenMismatch = 0x08, kPktIcrcMismatch = 0x10,
                   kPktFatal = kPktBadLen | kPktNotIpv4 | kPktNotUdp;

template <int LOG2G, bool RAGGED, bool VERIFY>
__global__ void __launch_bounds__(1024, 1) icrc_kernel(IcrcArgs a) {
  constexpr int G = 1 << LOG2G;
  constexpr int PPW = 64 / G;  // packets per wave step
  constexpr int DPI = 4 * G;   // grid dwords per iteration
  constexpr int NCOMB = 1 + LOG2G;
  constexpr int U = kUnroll;
  const int tid = threadIdx.x;

  // ---- stage the folding tables in LDS ------------------------------------
  {
    const uint32_t* gm = a.tables + LOG2G * 1024;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int i = tid + r * 1024;  // 8192 16-byte quads
      const int tab = i >> 11, e = (i >> 3) & 255, q = i & 7;
      lds_wr4((uint32_t)((tab >> 1) * 65536 + e * 256 + (tab & 1) * 128 + q * 16),
              gm[tab * 256 + e]);
    }
    const uint32_t* gc = a.tables + kNumMainSets * 1024;
    for (int i = tid; i < NCOMB * 1024; i += 1024) lds_wr(kLdsMain + 4u * i, gc[i]);
  }
  __syncthreads();

  const int lane = tid & 63;
  const int gl = lane & (G - 1);
  const int grp = lane >> LOG2G;
  const uint32_t kc0 = (uint32_t)(lane & 31) << 2;
  const uint32_t kc1 = kc0 | 0x10000u;
  const uint32_t nsets = (a.n + PPW - 1) / PPW;
  const uint32_t wave = blockIdx.x * 16u + (uint32_t)(tid >> 6);
  const uint32_t nwaves = gridDim.x * 16u;

  for (uint32_t set = wave; set < nsets; set += nwaves) {
    const uint32_t pkt = set * PPW + grp;
    const bool live = pkt < a.n;
    uint64_t off = 0;
    uint32_t L = 0;
    if (live) {
      if constexpr (RAGGED) {
        off = a.offsets[pkt];
        L = a.lens[pkt];
      } else {
        off = (uint64_t)pkt * a.stride;
        L = a.len;
      }
    }
    const uint8_t* fp = a.frames + off;

    // ---- frame checks (reference warning path -> ICRC 0) --------------------
    uint32_t st = (!live || L < 44 || (L & 3u) || L > 65535u) ? kPktBadLen : 0u;
    uint32_t d0 = 0, d2 = 0;
    if (st == 0) {
      d0 = ldg32(fp);
      d2 = ldg32(fp + 8);
    }
    const int ihl = (int)(d0 & 0xFu);
    if (st == 0) {
      if (((d0 >> 4) & 0xFu) != 4u || ihl < 5)
        st |= kPktNotIpv4;
      else if (((d2 >> 8) & 0xFFu) != 17u)
        st |= kPktNotUdp;
      else if (L < (uint32_t)(4 * ihl + 24))
        st |= kPktBadLen;
      const uint32_t tot = ((d0 >> 8) & 0xFF00u) | (d0 >> 24);
      if (tot != L) st |= kPktLenMismatch;
    }
    const bool good = (st & kPktFatal) == 0;
    const int ndw = good ? (int)((L - 4) >> 2) : 0;
    const int J = (ndw + DPI - 1) / DPI;
    const int pad = J * DPI - ndw;
    const int kub = ihl + 1;  // UDP checksum dword
    const int kbb = ihl + 3;  // BTH fecn|becn|resv6 dword
    int JH = min(J, (kbb + pad) / DPI + 1);
    JH = J - ((J - JH) / U) * U;  // body = whole blocks of U iterations

    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;

    // ---- head: front padding, masks and seed --------------------------------
    for (int j = 0; j < JH; ++j) {
      const int kb = DPI * j + 4 * gl - pad;
      uint32_t w[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = kb + t;
        uint32_t v = 0;
        if (k >= 0) v = ldg32(fp + 4 * k);
        v |= (k == 0 ? 0x0000FF00u : 0u) | (k == 2 ? 0xFFFF00FFu : 0u) |
             (k == kub ? 0xFFFF0000u : 0u) | (k == kbb ? 0x000000FFu : 0u);
        v ^= (k == 0) ? kSeedRegister : 0u;
        w[t] = v;
      }
      a0 = mul_main(a0 ^ w[0], kc0, kc1);
      a1 = mul_main(a1 ^ w[1], kc0, kc1);
      a2 = mul_main(a2 ^ w[2], kc0, kc1);
      a3 = mul_main(a3 ^ w[3], kc0, kc1);
    }

    // ---- body: blocks of U iterations, next block's loads in flight ---------
    const int nb = (J - JH) / U;
    const uint8_t* bp = fp + 4 * (int64_t)(DPI * JH + 4 * gl - pad);
    u32x4 cur[U];
    if (nb > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = ldg128(bp + 16 * G * u);
    }
    for (int b = 0; b < nb; ++b) {
      u32x4 nxt[U];
      if (b + 1 < nb) {
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = ldg128(bp + 16 * G * (U * (b + 1) + u));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a0 = mul_main(a0 ^ cur[u].x, kc0, kc1);
        a1 = mul_main(a1 ^ cur[u].y, kc0, kc1);
        a2 = mul_main(a2 ^ cur[u].z, kc0, kc1);
        a3 = mul_main(a3 ^ cur[u].w, kc0, kc1);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }

    // ---- combine: in-lane Horner, then butterfly across the group -----------
    uint32_t B = mul_comb(a3, kLdsMain) ^ a2;
    B = mul_comb(B, kLdsMain) ^ a1;
    B = mul_comb(B, kLdsMain) ^ a0;
#pragma unroll
    for (int l = 0; l < LOG2G; ++l) {
      const uint32_t m = mul_comb(B, kLdsMain + 4096u * (1 + l));
      const uint32_t t = ((gl >> l) & 1) ? m : B;
      B = t ^ (uint32_t)__shfl_xor((int)t, 1 << l, 64);
    }
    const uint32_t icrc = good ? ~B : 0u;

    if (live && gl == 0) {
      if constexpr (VERIFY) {
        const uint32_t trailer = good ? ldg32(fp + L - 4) : 0u;
        const bool ok = good && trailer == icrc;
        if (good && !ok) st |= kPktIcrcMismatch;
        a.ok_out[pkt] = ok ? 1 : 0;
      }
      if (a.icrc_out) a.icrc_out[pkt] = icrc;
      if (a.status_out) a.status_out[pkt] = (uint8_t)st;
    }
  }
}

__global__ void __launch_bounds__(256) stream_read_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                          uint32_t* sink) {
  constexpr int R = 8;
  const uint64_t gsz = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i + (R - 1) * gsz < n16; i += R * gsz) {
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = p[i + r * gsz];
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= v[r];
  }
  for (; i < n16; i += gsz) acc ^= p[i];
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9E3779B9u) sink[0] = x;  // keeps the loads live; practically never stores
}

typedef void (*kernel_fn)(IcrcArgs);

template <int LOG2G>
kernel_fn pick(bool ragged, bool verify) {
  if (ragged)
    return verify ? icrc_kernel<LOG2G, true, true> : icrc_kernel<LOG2G, true, false>;
  return verify ? icrc_kernel<LOG2G, false, true> : icrc_kernel<LOG2G, false, false>;
}

kernel_fn select_kernel(int log2g, bool ragged, bool verify) {
  switch (log2g) {
    case 0: return pick<0>(ragged, verify);
    case 1: return pick<1>(ragged, verify);
    case 2: return pick<2>(ragged, verify);
    case 3: return pick<3>(ragged, verify);
    case 4: return pick<4>(ragged, verify);
    case 5: return pick<5>(ragged, verify);
    case 6: return pick<6>(ragged, verify);
    default: return nullptr;
  }
}

size_t lds_bytes(int log2g) { return kLdsMain + 4096u * (1 + log2g); }

}  // namespace

void build_table_image(uint32_t* out) {
  for (int l = 0; l < kNumMainSets; ++l) table_set(128ll << l, out + l * 1024);
  uint32_t* comb = out + kNumMainSets * 1024;
  table_set(-32, comb);
  for (int l = 0; l < kMaxLog2G; ++l) table_set(-(128ll << l), comb + (1 + l) * 1024);
}

hipError_t prepare_kernels() {
  for (int l = 0; l <= kMaxLog2G; ++l)
    for (int r = 0; r < 2; ++r)
      for (int v = 0; v < 2; ++v) {
        hipError_t e = hipFuncSetAttribute((const void*)select_kernel(l, r, v),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds_bytes(l));
        if (e != hipSuccess) return e;
      }
  return hipSuccess;
}

hipError_t launch_icrc(const IcrcArgs& a, int log2g, bool ragged, bool verify, int num_cus,
                       hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  kernel_fn k = select_kernel(log2g, ragged, verify);
  if (!k) return hipErrorInvalidValue;
  const uint32_t ppw = 64u >> log2g;
  const uint64_t nsets = (a.n + ppw - 1) / ppw;
  uint64_t blocks = (nsets + 15) / 16;
  if (blocks > (uint64_t)num_cus) blocks = (uint64_t)num_cus;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(1024), lds_bytes(log2g), stream, a);
  return hipGetLastError();
}

hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, uint32_t* sink, int num_cus,
                              hipStream_t stream) {
  const uint64_t n16 = bytes / 16;
  if (n16 == 0) return hipSuccess;
  hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)(num_cus * 8)), dim3(256), 0, stream,
                     (const u32x4*)buf, n16, sink);
  return hipGetLastError();
}

}  // namespace ricrc
