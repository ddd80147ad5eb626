// MR -> packet segmentation fused with the ICRC, for MI355X (gfx950).
//
// Builds, on the GPU and straight from the memory region, every wire frame
// roce-sim's requester and responder emit for a batch of work requests:
// TXLogic.process_send_req (src/roce_sq.py:1243-1321), process_write_req
// (src/roce_sq.py:1323-1411) and ReadReqCtx.commit (src/roce_rq.py:388-438),
// and the header-only packets: process_read_req / process_atomic_req
// (src/roce_sq.py:1413-1466), process_ack / process_nak_* (src/roce_rq.py:
// 767-854) and the atomic acknowledge of AtomicReqCtx.commit
// (src/roce_rq.py:490-525); each packet wrapped in IPv4/UDP as send_ip_pkt / send_pkt do
// (src/roce_sq.py:1186-1197, src/roce_rq.py:705-731), padded as
// Util.add_padding_if_needed (src/roce_util.py:187-199), with its IPv4 header
// checksum, its ICRC (BTH.compute_icrc, src/roce.py:192-223) and its UDP
// checksum (scapy UDP.post_build, which runs after the ICRC is in place).
//
// One pass: a group of G lanes owns one packet; the packet's frame is laid on
// the same dword grid as the ICRC kernel (icrc_kernels.hip) with the frame
// starting at grid column 0 (slots are whole 128-byte lines), so in iteration j
// lane i produces the 16 frame bytes of dwords 4Gj + 4i .. +3: header dwords
// from the WR descriptor, payload dwords with one (unaligned) 16-byte MR load,
// stores them with one aligned 16-byte store and folds them into its four CRC
// columns and its UDP one's-complement sum in registers.  The frame is read
// from the MR once and written once; nothing is read back.  The frame's first
// and last iterations (one 128-byte line each at G = 8) are held back until
// the group has combined its CRC and checksum, then stored whole with the UDP
// checksum (dword 6) and the ICRC in place.
//
// Packet -> WR: a first small kernel writes each packet's WR index into the
// `lens` output array (one workgroup per WR); the segmentation kernel reads
// that entry and overwrites it with the frame length.
#include "icrc_device.hpp"
#include "roce_icrc.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ricrc {

namespace {

typedef u32x4 u32x4_u __attribute__((aligned(1)));

// 16-byte MR read (any alignment).
// (Default policy: non-temporal MR loads measured 12 % slower, seg kernel
// 1.925 vs 1.693 ms over 3 A/B rounds, profiles/r05b.)
__device__ __forceinline__ u32x4 ldmr(const uint8_t* p) {
  return *(const u32x4_u*)p;
}

constexpr int kSegUnroll = 4;  // body iterations (16-byte MR loads per lane) in flight
// last 1/kSegTailDiv of a range claimed dynamically: seg kernel ms (3 A/B
// rounds, profiles/r03q_seg_tail_ab.txt) static 1.692-1.723, 1/4
// 1.660-1.691 (+1.8 %), 1/8 1.661-1.701, 1/16 1.692-1.693
constexpr uint32_t kSegTailDiv = 4;
constexpr uint32_t kSegMaxVictims = 4;
// one workgroup per CU (the tables fill the LDS); 8 waves x ~200 VGPRs: no
// spills (16 waves spill ~20 VGPRs)
constexpr int kSegThreads = 512;
constexpr int kSegWaves = kSegThreads / 64;
// Cache policy of the frame stores (stg128 in icrc_device.hpp; 2 = nt).
constexpr int kSegStorePol = 2;
constexpr uint32_t kRocePort = 4791;   // src/roce_enum.py ROCE_PORT
constexpr uint32_t kAckValue = 31;     // CREDIT_CNT_INVALID, src/roce_enum.py:8
// AETH.code (src/roce.py:267): ACK 0, RNR 1, NAK 3
constexpr uint32_t kAethAck = 0, kAethRnr = 1, kAethNak = 3;
constexpr uint32_t kPktSegBad = 0x20;  // RICRC_PKT_SEG_BAD

__device__ __forceinline__ uint32_t wr_pkt_num(uint32_t len, uint32_t pmtu) {
  // Util.compute_wr_pkt_num, src/roce_util.py:183-185
  return len ? (uint32_t)(((uint64_t)len + pmtu - 1) / pmtu) : 1u;
}

// Everything a lane needs to produce its packet's frame dwords.
struct Seg {
  const uint8_t* src;  // payload start in the MR
  uint8_t* dst;        // slot start
  uint32_t plen;       // payload bytes
  const uint8_t* hi;   // highest start of a 16-byte payload read (see describe_seg)
  int hd;              // header dwords: IPv4 5 + UDP 2 + BTH 3 + extension headers
  int T;               // frame dwords incl. the ICRC slot
  int F;               // dwords fully defined without masking: hd + plen / 4
  // header dwords (big-endian values) except the checksums
  uint32_t h0, h3, h4, h5, h6, h7, h8, h9;
  uint32_t e[7];       // extension header dwords (AtomicETH is the longest, 7)
  uint32_t ipcs;       // IPv4 header checksum
  bool live;
};

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  s = (s & 0xFFFFu) + (s >> 16);
  s = (s & 0xFFFFu) + (s >> 16);
  return s;
}

// The packet of index `pkt`: its WR, opcode, extension headers and geometry
// (the rules of src/roce_sq.py:1243-1411 and src/roce_rq.py:388-438).
__device__ __forceinline__ Seg describe_seg(const SegArgs& a, uint32_t pkt, bool inrange,
                                            uint32_t& status, const uint8_t* mr_hi) {
  Seg s;
  status = 0;
  s.live = false;
  s.dst = a.frames + (uint64_t)pkt * a.slot;
  // A packet without payload reads no MR byte: its (unconditional, masked)
  // payload loads are clamped to the first 16 bytes of its own slot (of the
  // frame buffer's first slot for a lane past the batch).
  s.src = inrange ? s.dst : a.frames;
  s.hi = s.src;
  s.plen = 0;
  s.hd = 10;
  s.T = 0;
  s.F = 0;
  s.h0 = s.h3 = s.h4 = s.h5 = s.h6 = s.h7 = s.h8 = s.h9 = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) s.e[i] = 0;
  s.ipcs = 0;
  if (!inrange) return s;
  const uint32_t w = a.lens[pkt];
  status = kPktSegBad;
  if (w >= a.nwr) return s;
  const ricrc_seg_wr& wr = a.wrs[w];
  const uint64_t mo = wr.mr_offset;
  const uint32_t len = wr.length, op = wr.op;
  const bool data = op <= RICRC_SEG_READ_RESPONSE;  // packets carrying MR bytes
  const uint32_t n = data ? wr_pkt_num(len, a.pmtu) : 1u;
  const uint32_t k = pkt - wr.first_pkt;
  if (pkt < wr.first_pkt || k >= n || op >= RICRC_SEG_NUM_OPS ||
      (data && (mo > a.mr_bytes || len > a.mr_bytes - mo)))
    return s;
  status = 0;
  s.live = true;
  const bool last = k == n - 1, first = k == 0;
  const bool sig = (wr.flags & RICRC_SEG_SIGNALED) != 0;
  const bool sol = (wr.flags & RICRC_SEG_SOLICITED) != 0;
  // payload: full PMTU slices, the remainder on the last packet (none if len == 0)
  const uint32_t off = k * a.pmtu;
  if (data) {
    s.plen = last ? len - off : a.pmtu;
    if (s.plen) {
      s.src = a.mr + mo + off;
      s.hi = mr_hi;
    }
  }

  // ext: 0 none, 1 one dword (ImmDt/IETH/AETH), 3 AETH + AtomicAckETH,
  // 4 RETH, 5 RETHImmDt, 7 AtomicETH
  uint32_t opc, ext = 0;
  uint32_t e0 = 0;
  bool ack = false, se = false;
  const uint32_t va_hi = (uint32_t)(wr.remote_va >> 32), va_lo = (uint32_t)wr.remote_va;
  if (!data) {
    const uint32_t msn = wr.msn & 0xFFFFFFu;
    if (op == RICRC_SEG_READ_REQUEST) {  // src/roce_sq.py:1421-1428
      opc = 0x0Cu;
      ext = 4;  // RETH(va, rkey, dlen = length) below
      ack = true;
    } else if (op <= RICRC_SEG_FETCH_ADD) {  // src/roce_sq.py:1444-1463
      opc = op == RICRC_SEG_COMPARE_SWAP ? 0x13u : 0x14u;
      ext = 7;
      ack = true;
      s.e[0] = va_hi;
      s.e[1] = va_lo;
      s.e[2] = wr.rkey;
      s.e[3] = (uint32_t)(wr.swap >> 32);
      s.e[4] = (uint32_t)wr.swap;
      s.e[5] = (uint32_t)(wr.comp >> 32);
      s.e[6] = (uint32_t)wr.comp;
    } else if (op == RICRC_SEG_ATOMIC_ACK) {  // src/roce_rq.py:517-524
      opc = 0x12u;
      ext = 3;
      s.e[0] = (kAckValue << 24) | msn;
      s.e[1] = (uint32_t)(wr.swap >> 32);  // AtomicAckETH.orig
      s.e[2] = (uint32_t)wr.swap;
    } else {  // ACKNOWLEDGE: ACK / RNR NAK / NAK, src/roce_rq.py:767-853
      opc = 0x11u;
      ext = 1;
      const uint32_t code = op == RICRC_SEG_ACK ? kAethAck : op == RICRC_SEG_RNR_NAK ? kAethRnr
                                                                                     : kAethNak;
      const uint32_t value = op == RICRC_SEG_ACK ? kAckValue : (wr.imm & 31u);
      e0 = (((code << 5) | value) << 24) | msn;
    }
  } else if (op <= RICRC_SEG_SEND_WITH_INV) {
    if (!last) {
      opc = first ? 0x00u : 0x01u;  // SEND_FIRST / SEND_MIDDLE
    } else {
      const bool only = n == 1;
      opc = op == RICRC_SEG_SEND ? (only ? 0x04u : 0x02u)
            : op == RICRC_SEG_SEND_WITH_IMM ? (only ? 0x05u : 0x03u)
                                            : (only ? 0x17u : 0x16u);
      if (op != RICRC_SEG_SEND) {
        ext = 1;
        e0 = wr.imm;  // ImmDt.data / IETH.rkey
      }
      ack = sig;
      se = sol;
    }
  } else if (op <= RICRC_SEG_RDMA_WRITE_WITH_IMM) {
    const bool imm = op == RICRC_SEG_RDMA_WRITE_WITH_IMM;
    if (!last) {
      opc = first ? 0x06u : 0x07u;  // RDMA_WRITE_FIRST (+RETH) / MIDDLE
      ext = first ? 4 : 0;
    } else if (n == 1) {
      opc = imm ? 0x0Bu : 0x0Au;  // RDMA_WRITE_ONLY[_WITH_IMMEDIATE]: RETH[ImmDt]
      ext = imm ? 5 : 4;
    } else {
      opc = imm ? 0x09u : 0x08u;  // RDMA_WRITE_LAST[_WITH_IMMEDIATE]: [ImmDt]
      ext = imm ? 1 : 0;
      e0 = wr.imm;
    }
    if (last) {
      ack = sig;
      se = imm && sol;
    }
  } else {  // RDMA READ response: AETH on FIRST / LAST / ONLY
    opc = n == 1 ? 0x10u : first ? 0x0Du : last ? 0x0Fu : 0x0Eu;
    if (first || last) {
      ext = 1;
      e0 = (kAckValue << 24) | (wr.msn & 0xFFFFFFu);  // rsvd 0, code ACK 0, value 31, msn
    }
  }
  if (ext == 4 || ext == 5) {
    s.e[0] = va_hi;
    s.e[1] = va_lo;
    s.e[2] = wr.rkey;
    s.e[3] = len;  // RETH.dlen = message length (READ_REQUEST: the read size)
    s.e[4] = wr.imm;
  } else if (ext == 1) {
    s.e[0] = e0;
  }
  s.hd = 10 + (int)ext;
  const uint32_t pad = (4u - (s.plen & 3u)) & 3u;
  const int pdw = (int)((s.plen + 3u) >> 2);
  s.T = s.hd + pdw + 1;
  s.F = s.hd + (int)(s.plen >> 2);
  const uint32_t tl = 4u * (uint32_t)s.T;
  s.h0 = 0x45000000u | tl;
  s.h3 = wr.src_ip;
  s.h4 = wr.dst_ip;
  s.h5 = ((uint32_t)wr.sport << 16) | kRocePort;
  s.h6 = (tl - 20u) << 16;  // UDP length, checksum filled in at the end
  s.h7 = (opc << 24) | ((se ? 0x80u : 0u) << 16) | (pad << 20) | 0xFFFFu;  // SE|M|PadCnt|TVer, P_Key
  s.h8 = wr.dqpn & 0xFFFFFFu;                                              // FECN|BECN|resv6 = 0
  s.h9 = (ack ? 0x80000000u : 0u) | ((wr.psn + k) & 0xFFFFFFu);
  // IPv4 header checksum over 0x4500, tl, id 1, frag 0, ttl 64 | proto 17, src, dst
  const uint32_t sum = 0x4500u + tl + 1u + 0x4011u + (s.h3 >> 16) + (s.h3 & 0xFFFFu) +
                       (s.h4 >> 16) + (s.h4 & 0xFFFFu);
  s.ipcs = (~fold16(sum)) & 0xFFFFu;
  return s;
}

// Header dword 4c + t (< hd) in memory (little-endian) order; t is a
// compile-time constant and c the lane's chunk (0..3), so this is three
// selects (a switch on the dword index becomes a private-memory table).
template <int t>
__device__ __forceinline__ uint32_t header_dword(const Seg& s, int c) {
  constexpr uint32_t kId = 0x00010000u;  // id 1, flags/frag 0
  uint32_t v0, v1, v2, v3, v4;
  if constexpr (t == 0) {
    v0 = s.h0; v1 = s.h4; v2 = s.h8; v3 = s.e[2]; v4 = s.e[6];
  } else if constexpr (t == 1) {
    v0 = kId; v1 = s.h5; v2 = s.h9; v3 = s.e[3]; v4 = 0u;
  } else if constexpr (t == 2) {
    v0 = 0x40110000u | s.ipcs; v1 = s.h6; v2 = s.e[0]; v3 = s.e[4]; v4 = 0u;  // ttl 64, proto 17
  } else {
    v0 = s.h3; v1 = s.h7; v2 = s.e[1]; v3 = s.e[5]; v4 = 0u;
  }
  const uint32_t v = c == 0 ? v0 : c == 1 ? v1 : c == 2 ? v2 : c == 3 ? v3 : v4;
  return __builtin_bswap32(v);
}

// 16 payload bytes from `p` without reading past `hi + 16` (hi = the MR end
// minus 16): one unconditional load at min(p, hi), then a byte shift in
// registers.  Bytes that would lie past the MR end come out as garbage; they
// are past the message, so the caller masks them.  Only waves that can reach
// the MR end use this form (see segment_kernel).
__device__ __forceinline__ u32x4 load_payload_clamped(const uint8_t* p, const uint8_t* hi) {
  const uint8_t* q = p < hi ? p : hi;
  const u32x4 v = ldmr(q);
  const uint32_t d = (uint32_t)(p - q);
  const int k = (int)(d >> 2);
  const uint32_t sh = d & 3u;
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(pick4(v, k + 1, 0u), pick4(v, k, 0u), sh);
  o.y = __builtin_amdgcn_alignbyte(pick4(v, k + 2, 0u), pick4(v, k + 1, 0u), sh);
  o.z = __builtin_amdgcn_alignbyte(pick4(v, k + 3, 0u), pick4(v, k + 2, 0u), sh);
  o.w = __builtin_amdgcn_alignbyte(pick4(v, k + 4, 0u), pick4(v, k + 3, 0u), sh);
  return o;
}

// Keep the low `valid` bytes of a payload dword (valid <= 0: none).
__device__ __forceinline__ uint32_t keep_bytes(uint32_t v, int valid) {
  return valid >= 4 ? v : valid <= 0 ? 0u : (v & ((1u << (8 * valid)) - 1u));
}

// A chunk outside the full-payload body: header dwords (HEAD only: all of
// them lie in the first block), payload with its zero pad, the (zero) ICRC
// slot and zeros past the frame end.  `v` holds the 16 MR bytes at payload
// dword max(idx0 - hd, 0) (see seg_load).
template <bool HEAD>
__device__ __forceinline__ u32x4 edge_chunk(const Seg& s, int idx0, const u32x4& v) {
  const int mbase = idx0 > s.hd ? idx0 - s.hd : 0;
  u32x4 w;
#define RICRC_EDGE(c, t)                                                                  \
  {                                                                                       \
    const int idx = idx0 + (t);                                                           \
    const int m = idx - s.hd;                                                             \
    const uint32_t pay = keep_bytes(pick4(v, m - mbase, 0u), (int)s.plen - 4 * m);       \
    if constexpr (HEAD)                                                                   \
      w.c = idx < s.hd ? header_dword<(t)>(s, idx0 >> 2) : pay;                           \
    else                                                                                  \
      w.c = pay;                                                                          \
  }
  RICRC_EDGE(x, 0)
  RICRC_EDGE(y, 1)
  RICRC_EDGE(z, 2)
  RICRC_EDGE(w, 3)
#undef RICRC_EDGE
  return w;
}

// One's-complement accumulation of UDP bytes (dwords >= 5) in memory order.
__device__ __forceinline__ void csum_add(uint64_t& acc, const u32x4& w) {
  acc += (uint64_t)w.x + w.y + w.z + w.w;
}

template <int LOG2G>
__global__ void __launch_bounds__(kSegThreads, 1) segment_kernel(SegArgs a) {
  constexpr int G = 1 << LOG2G;
  constexpr int DPI = 4 * G;
  constexpr int PPW = 64 / G;
  constexpr int U = kSegUnroll;
  const int tid = threadIdx.x;
  announce_batch(a.busy);
  stage_tables<LOG2G, kSegThreads, MainKeys>(a.tables, tid);
  __syncthreads();

  const int lane = tid & 63;
  const int gl = lane & (G - 1);
  const int grp = lane >> LOG2G;
  const int base = grp * G;
  const MainKeys kk = MainKeys::make(lane);
  const uint8_t* mr_end = a.mr + a.mr_bytes;
  // lowest start of a 16-byte read that stays inside the MR (an MR shorter
  // than 16 bytes must be readable for 16, include/roce_icrc.h)
  const uint8_t* mr_hi = a.mr_bytes >= 16 ? mr_end - 16 : a.mr;
  const uint32_t nsets = (a.npkts + PPW - 1) / PPW;
  const uint32_t per_block = (nsets + gridDim.x - 1) / gridDim.x;
  // A workgroup's range [begin, end) of sets; its last 1/kSegTailDiv is
  // claimed set by set through the workgroup's counter, from which the
  // workgroups that finish first also claim (the strided ICRC kernel's tail
  // stealing, icrc_kernels.hip; a packet's frame slot and outputs do not
  // depend on who builds it).
  auto range = [&](uint32_t blk, uint32_t& b, uint32_t& e, uint32_t& split) {
    b = blk * per_block;
    e = min(nsets, b + per_block);
    const uint32_t len = b < e ? e - b : 0u;
    split = e - (a.claims ? len / kSegTailDiv : 0u);
  };
  uint32_t set_begin, set_end, set_split;
  range(blockIdx.x, set_begin, set_end, set_split);
  unsigned long long* claims =
      a.claims ? a.claims + (size_t)(a.epoch % kClaimSlots) * kMaxClaimBlocks : nullptr;
  if (claims && tid == 0) atomicExch(&claims[blockIdx.x], (unsigned long long)a.epoch << 32);

  auto do_set = [&](uint32_t set) {
    const uint32_t pkt = set * PPW + grp;
    uint32_t status;
    const Seg s = describe_seg(a, pkt, pkt < a.npkts, status, mr_hi);
    // CRC geometry (frame at grid column 0): n covered dwords, J iterations,
    // r valid columns in the last one
    const int n = s.live ? s.T - 1 : 1;
    const int J = (n + DPI - 1) / DPI;
    const int r = n - DPI * (J - 1);
    const int Jw = s.live ? (s.T + DPI - 1) / DPI : 0;  // iterations that write
    const int nblk = (Jw + U - 1) / U;                  // blocks of U iterations
    const int t_last = s.T - 1;                          // ICRC slot dword

    // Every MR load is unconditional, so the compiler can count the loads in
    // flight (a predicated load forces a full vmcnt(0) drain).  Iteration j
    // of a block >= 1 reads the 16 payload bytes at dword DPI j + 4 gl - hd
    // from one base pointer (immediate offsets); block 0 clamps header lanes
    // to dword 0.  Reads run up to one block past the frame (into the next
    // packet's bytes); a wave that could read past the MR end, or holds a
    // packet without payload (whose loads stay in its own slot), takes the
    // clamped-and-shifted form of every load instead.
    const int far = max(DPI * (max(nblk, 2) * U - 1) + 4 * gl - s.hd, 0);
    const bool guard = s.hi != mr_hi || s.src + 4 * far + 16 > mr_end;

    Col A = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    uint64_t acc = 0;

    // The frame's first and last iterations (one 128-byte line each at G = 8:
    // the slot is 256-byte aligned) are kept in registers and stored once the
    // group has combined, with the UDP checksum (dword 6) and the ICRC (dword
    // T-1) in place: every line of a frame is written whole, by one wave
    // instruction per iteration.  (Rewriting the 2 + 4 bytes into lines already
    // streamed out measured 4-6 % slower than not writing them at all; holding
    // only the two 16-byte chunks, so those lines went out in two parts, was
    // slower still.)
    u32x4 hold0 = {0, 0, 0, 0}, holdL = {0, 0, 0, 0};
    auto edge = [&](int j, const u32x4& v, auto head) {
      const int idx0 = DPI * j + 4 * gl;
      if (idx0 >= s.T) return;
      u32x4 w = edge_chunk<decltype(head)::value>(s, idx0, v);
      // UDP one's-complement sum: dwords 5 .. T-2 (the ICRC slot is still zero)
      u32x4 cs = w;
      if (idx0 + 0 < 5) cs.x = 0;
      if (idx0 + 1 < 5) cs.y = 0;
      if (idx0 + 2 < 5) cs.z = 0;
      if (idx0 + 3 < 5) cs.w = 0;
      csum_add(acc, cs);
      if (j == 0)
        hold0 = w;
      else if (j == Jw - 1)
        holdL = w;
      else
        stg128<kSegStorePol>(s.dst + 4 * idx0, w);
      if (j < J) {  // CRC: masked header dwords, seed, columns past the end skipped
        w.x = fix_dword(w.x, idx0 + 0, 6, 8);
        w.y = fix_dword(w.y, idx0 + 1, 6, 8);
        w.z = fix_dword(w.z, idx0 + 2, 6, 8);
        w.w = fix_dword(w.w, idx0 + 3, 6, 8);
        if (j == J - 1)
          fold_last(A, w, idx0, n, kk);
        else
          fold(A, w, kk);
      }
    };
    // block b >= 1: the full-payload fast path when all its iterations lie in
    // [hd, F) (no header, no mask, no ICRC slot), else the generic path
    auto block = [&](int b, const u32x4* v) {
      const int j0 = b * U;
      if (DPI * (j0 + U) <= s.F) {
        uint8_t* d = s.dst + 4 * (DPI * j0 + 4 * gl);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          stg128<kSegStorePol>(d + 4 * DPI * u, v[u]);
          csum_add(acc, v[u]);
          fold(A, v[u], kk);
        }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) edge(j0 + u, v[u], std::false_type{});
      }
    };
    // The block loop runs the wave's largest block count (a uniform trip
    // count, so the two buffers ping-pong without waits on fresh loads); a
    // group past its own last block re-reads that block (cache hits) and its
    // chunks fall past the frame end.
    int nbmax = nblk;
#pragma unroll
    for (int l = 1; l < 64; l <<= 1) nbmax = max(nbmax, __shfl_xor(nbmax, l, 64));
    nbmax = __builtin_amdgcn_readfirstlane(nbmax);  // scalar: a uniform loop
    auto run = [&](auto guarded) {
      constexpr bool GUARD = decltype(guarded)::value;
      // block b's loads, b clamped to [1, nblk - 1]
      auto ld_block = [&](int b, u32x4* v) {
        const int bc = max(min(b, nblk - 1), 1);
        if constexpr (GUARD) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int m = max(DPI * min(bc * U + u, max(Jw - 1, 0)) + 4 * gl - s.hd, 0);
            v[u] = load_payload_clamped(s.src + 4 * m, s.hi);
          }
        } else {
          // iterations past the packet's last one re-read that one (no HBM
          // over-read into the next packet)
          const uint8_t* p = s.src + 4 * (DPI * U * bc + 4 * gl - s.hd);
          const int last = max(Jw - 1 - U * bc, 0);
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = ldmr(p + 4 * DPI * min(u, last));
        }
      };
      u32x4 X[U], Y[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int m = max(DPI * u + 4 * gl - s.hd, 0);
        if constexpr (GUARD)
          Y[u] = load_payload_clamped(s.src + 4 * m, s.hi);
        else
          Y[u] = ldmr(s.src + 4 * m);
      }
      ld_block(1, X);
      // block 0 carries the header (hd <= 15 < DPI * U).  A whole buffer is
      // refilled before the other one is used; refilling each chunk right
      // after its use (loads in flight near 2U throughout) measured 3 %
      // slower, also at U = 3 and 5 (3 A/B rounds, round 3).
#pragma unroll
      for (int u = 0; u < U; ++u) edge(u, Y[u], std::true_type{});
      for (int b = 1; b < nbmax; b += 2) {
        ld_block(b + 1, Y);
        block(b, X);
        if (b + 1 >= nbmax) break;
        ld_block(b + 2, X);
        block(b + 1, Y);
      }
    };
    if (__any(guard))
      run(std::true_type{});
    else
      run(std::false_type{});

    // ---- group combine: ICRC, then the UDP checksum over the final bytes -----
    const uint32_t B = combine<LOG2G, MainKeys>(A.P[0] ^ A.T[0], A.P[1] ^ A.T[1], A.P[2] ^ A.T[2],
                                                A.P[3] ^ A.T[3], r, gl, base);
    const uint32_t icrc = ~B;
    uint32_t f = (uint32_t)acc;
    f = (f & 0xFFFFu) + (f >> 16) + (uint32_t)(acc >> 32);
#pragma unroll
    for (int l = 0; l < LOG2G; ++l) f += (uint32_t)__shfl_xor((int)f, 1 << l, 64);
    if (s.live) {
      // pseudo header (src, dst, proto 17, UDP length) in memory byte order,
      // plus the ICRC; the UDP header and payload are in f
      const uint32_t ulen = 4u * (uint32_t)s.T - 20u;
      uint32_t t = f + __builtin_bswap16((uint16_t)(s.h3 >> 16)) + __builtin_bswap16((uint16_t)s.h3) +
                   __builtin_bswap16((uint16_t)(s.h4 >> 16)) + __builtin_bswap16((uint16_t)s.h4) +
                   0x1100u + __builtin_bswap16((uint16_t)ulen) + (icrc & 0xFFFFu) + (icrc >> 16);
      t = fold16(fold16(t));
      uint32_t c = (~t) & 0xFFFFu;
      if (c == 0) c = 0xFFFFu;  // UDP: a computed 0 goes out as 0xFFFF
      if (gl == (4 >> 2)) hold0.z = (hold0.z & 0xFFFFu) | (c << 16);  // dword 6 (G >= 2)
      const int jl = Jw - 1, idxL = DPI * jl + 4 * gl;
      if (idxL <= t_last && t_last < idxL + 4) {  // the lane holding the ICRC slot
        u32x4& h = jl == 0 ? hold0 : holdL;
        const int t = t_last - idxL;
        h.x = t == 0 ? icrc : h.x;
        h.y = t == 1 ? icrc : h.y;
        h.z = t == 2 ? icrc : h.z;
        h.w = t == 3 ? icrc : h.w;
      }
      // the first and last iterations are stored whole (zeros past the frame
      // end, never past the slot): the frame's last line goes out as one full
      // line (+0.5 % over stopping at the 16-byte chunk holding the ICRC,
      // 3 A/B rounds on 128-byte slots, round 3)
      if (16 * gl < (int)a.slot) stg128<kSegStorePol>(s.dst + 16 * gl, hold0);
      if (jl > 0 && 4 * idxL < (int)a.slot) stg128<kSegStorePol>(s.dst + 4 * idxL, holdL);
    }
    if (pkt < a.npkts && gl == 0) {
      a.lens[pkt] = s.live ? 4u * (uint32_t)s.T : 0u;
      if (a.icrc_out) a.icrc_out[pkt] = s.live ? icrc : 0u;
      if (a.status_out) a.status_out[pkt] = (uint8_t)status;
    }
  };
  for (uint32_t set = set_begin + (uint32_t)(tid >> 6); set < set_split; set += (uint32_t)kSegWaves)
    do_set(set);
  if (claims) {  // own tail, then up to kMaxVictims other workgroups' tails
    uint32_t victim = blockIdx.x, tries = 0;
    auto claim = [&](uint32_t v) -> uint32_t {  // set index, or ~0u if v's tail is empty
      unsigned long long old = 0;
      if (lane == 0) old = atomicAdd(&claims[v], 1ull);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)old);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(old >> 32));
      uint32_t vb, ve, vs;
      range(v, vb, ve, vs);
      return (hi == a.epoch && lo < ve - vs) ? vs + lo : ~0u;
    };
    for (;;) {
      const uint32_t cur = claim(victim);
      if (cur == ~0u) {
        if (++tries > kSegMaxVictims) break;
        victim = (blockIdx.x + 2 * tries - 1) % gridDim.x;
        continue;
      }
      do_set(cur);
    }
  }
}

// Packet -> WR map: lens[first_pkt + k] = WR index, one workgroup per WR.
__global__ void __launch_bounds__(256) seg_map_kernel(SegArgs a) {
  for (uint32_t w = blockIdx.x; w < a.nwr; w += gridDim.x) {
    const uint32_t fp = a.wrs[w].first_pkt;
    // (header-only ops are one packet whatever their length field)
    const uint32_t cnt =
        a.wrs[w].op <= RICRC_SEG_READ_RESPONSE ? wr_pkt_num(a.wrs[w].length, a.pmtu) : 1u;
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) {
      const uint64_t p = (uint64_t)fp + k;
      if (p < a.npkts) a.lens[p] = w;
    }
  }
}

// STREAM-style copy with the segmentation kernel's geometry: one 1024-thread
// workgroup per CU over a contiguous chunk, 16-byte nt loads and stores.
__global__ void __launch_bounds__(1024) stream_copy_kernel(const u32x4* __restrict__ src,
                                                           u32x4* __restrict__ dst, uint64_t n16) {
  constexpr int R = 4;
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per;
  const uint64_t b1 = b0 + per < n16 ? b0 + per : n16;
  uint64_t i = b0 + threadIdx.x;
  for (; i + (R - 1) * 1024 < b1; i += R * 1024) {
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = __builtin_nontemporal_load(src + i + r * 1024);
#pragma unroll
    for (int r = 0; r < R; ++r) __builtin_nontemporal_store(v[r], dst + i + r * 1024);
  }
  for (; i < b1; i += 1024) dst[i] = src[i];
}

typedef void (*seg_fn)(SegArgs);

seg_fn select_segment(int log2g) {
  switch (log2g) {
    case 1: return segment_kernel<1>;
    case 2: return segment_kernel<2>;
    case 3: return segment_kernel<3>;
    case 4: return segment_kernel<4>;
    default: return nullptr;
  }
}

size_t seg_lds_bytes(int log2g) { return MainKeys::kComb + 4096u * (1 + log2g) + 256u; }

}  // namespace

hipError_t prepare_segment_kernels() {
  for (int l = 1; l <= 4; ++l) {
    hipError_t e = set_dynamic_lds((const void*)select_segment(l), (int)seg_lds_bytes(l));
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_segment(const SegArgs& a, int log2g, int num_cus, hipStream_t stream) {
  if (a.npkts == 0) return hipSuccess;
  seg_fn k = select_segment(log2g);
  if (!k) return hipErrorInvalidValue;
  if (a.nwr) {
    const uint32_t mb = a.nwr < 8192u ? a.nwr : 8192u;
    hipLaunchKernelGGL(seg_map_kernel, dim3(mb), dim3(256), 0, stream, a);
  }
  const uint32_t ppw = 64u >> log2g;
  const uint64_t nsets = (a.npkts + ppw - 1) / ppw;
  uint64_t blocks = (nsets + kSegWaves - 1) / kSegWaves;
  if (blocks > (uint64_t)num_cus) blocks = (uint64_t)num_cus;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(kSegThreads), seg_lds_bytes(log2g), stream, a);
  return hipGetLastError();
}

hipError_t launch_stream_copy(const uint8_t* src, uint8_t* dst, uint64_t bytes, int num_cus,
                              hipStream_t stream) {
  const uint64_t n16 = bytes / 16;
  if (n16 == 0) return hipSuccess;
  hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)num_cus), dim3(1024), 0, stream,
                     (const u32x4*)src, (u32x4*)dst, n16);
  return hipGetLastError();
}

}  // namespace ricrc
