// RoCEv2 ICRC kernels for MI355X (gfx950, CDNA4).
//
// Computes, per wire frame, the Invariant CRC of datenlord/roce-sim's
// BTH.compute_icrc (src/roce.py:192-223): zlib CRC-32 of
// FF x 8 || frame[0 : len-4] with IP tos/ttl/chksum, UDP chksum and the BTH
// fecn|becn|resv6 byte forced to ones (src/roce.py:204-211).
//
// Work decomposition ("absolute-aligned dword grid").  A group of G lanes
// (G = 1 .. 64, a power of two) owns one packet.  Its n covered dwords are
// laid on a grid of J iterations x 4G dwords aligned to ABSOLUTE memory:
// iteration j covers the dwords [ab/4 + 4G j, ab/4 + 4G (j + 1)), ab = the
// frame start rounded down to 16G bytes, so in iteration j lane i of the
// group reads ONE aligned 16-byte chunk and the group an aligned 16G-byte
// run.  Columns before the frame start hold zero (a zero register stays
// zero); columns past its end skip the last iteration.  Each lane keeps four
// CRC registers a_t (t = grid column inside the lane) and folds
//
//      a_t <- Mul(128 G)(a_t ^ w_t)          (= "w_t followed by 16G-4 zero bytes")
//
// where Mul(m) is multiplication by x^m mod P on the reflected register,
// evaluated as four byte-indexed table lookups from LDS.  The packet ends at
// column r of its last iteration, so column c is off by x^(32 ((c - r) mod
// 4G)): combine() rotates the columns by r and folds R = sum Mul(-32 c')(a_c')
// with three in-lane Horner steps (Mul(-32)) and log2 G cross-lane butterfly
// levels (Mul(-128 * 2^l), __shfl_xor inside the group).  No MFMA: this is a
// byte scan, bound by HBM.
//
// LDS (per workgroup, one 1024-thread workgroup per CU):
//   [0, 128 KiB)  Mul(128 G) tables replicated 32x so every lane of a
//                 ds_read_b32 half-wave hits its own bank:
//                 addr(tab, e, lane) = (tab >> 1) * 64 KiB + e * 256
//                                      + (tab & 1) * 128 + (lane & 31) * 4
//                 (bank = lane & 31, conflict-free); the address is ONE
//                 v_perm_b32 of the register and a per-lane constant.
//   [128 KiB, +4 KiB * (1 + log2 G))  combine tables, unreplicated.
//   (icrc_device.hpp: Keys32; the 16-copy Keys16 layout is an option there
//   and the layout of the small-frame kernel.)
//
// Masks, seed: the masked dwords are packet dwords 0 (TOS), 2 (TTL, IP csum),
// IHL+1 (UDP csum) and IHL+3 (BTH byte 4); the FF x 8 prefix is folded in as
// the CRC register 0xDEBB20E3 XORed into dword 0.  They are applied in the
// peeled "head" iterations; the body loop is plain loads.
#include "icrc_device.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ricrc {

namespace {


// Lane-group kernels: one workgroup per CU (the replicated tables fill the LDS).
// Ragged: 16 waves (its short sorted sets are instruction-bound: 12 waves
// measured 5 % slower on cfg3).  Strided: 12 waves.  With 16 waves x 8
// 16-byte loads per lane in flight a CU holds 128 KiB of reads in flight,
// past what HBM serves best: a pure read stream runs at 7.13 TB/s with
// 64 KiB in flight per CU and 6.70 with 128 KiB (scratch/read_ceiling.hip);
// cfg2 at 12 waves +2 % (6050 -> 6179 GiB/s, 3 A/B rounds; 10 waves +1.7 %,
// 8 waves -1 %).
constexpr int kIcrcThreads = 1024;  // ragged kernel
constexpr int kIcrcWaves = kIcrcThreads / 64;
constexpr int kStridedThreads = 768;
constexpr int kStridedWaves = kStridedThreads / 64;

constexpr uint32_t kPktBadLen = 0x01, kPktNotIpv4 = 0x02, kPktNotUdp = 0x04,
                   kPktLenMismatch = 0x08, kPktIcrcMismatch = 0x10,
                   kPktFatal = kPktBadLen | kPktNotIpv4 | kPktNotUdp;

// One packet as seen by its lane group, on the ALIGNED grid: iteration j
// covers the absolute dwords [ab/4 + DPI j, ab/4 + DPI (j + 1)), so every lane
// load is a 16-byte aligned chunk and every group run is 16G-byte aligned.
struct Pkt {
  const uint8_t* fp;  // frame start
  const uint8_t* ab;  // frame start rounded down to a 4 DPI-byte boundary
  uint32_t L;         // frame length incl. the ICRC slot
  uint32_t pkt;       // index in the batch
  int n;              // covered dwords (IP header .. last pad byte)
  int S;              // grid column of the frame's first dword
  int J;              // iterations
  int r;              // valid columns in the last iteration (1 .. DPI)
  int jh;             // iterations that may hold dwords k <= 8 (masks, seed, k < 0)
  bool live;          // pkt < n: an output slot exists
  bool dead;          // the main path reads nothing: outside the batch, unusable
                      // length, or (unless described for the slow path) unaligned
  bool unal;          // usable frame whose start is not 4-byte aligned: slow path
};

// `unal_ok`: describe a frame at a non-dword-aligned start for the byte-load
// slow path (its grid is then anchored at the frame start itself).
template <int DPI>
__device__ __forceinline__ Pkt describe(const uint8_t* frames, uint32_t pkt, bool live, uint64_t off,
                                        uint32_t L, bool unal_ok = false) {
  Pkt p;
  p.fp = frames + off;
  p.L = L;
  p.pkt = pkt;
  p.live = live;
  const bool lenbad = L < 44 || L > 65535u;
  // a frame at an unaligned start, or whose length is not a multiple of 4
  // (the reference CRCs any length; none of its own emit paths builds one),
  // takes the byte-load slow path
  p.unal = live && !lenbad && (((uintptr_t)p.fp & 3u) != 0 || (L & 3u) != 0);
  p.dead = !live || lenbad || (p.unal && !unal_ok);
  p.S = p.unal ? 0 : (int)(((uintptr_t)p.fp >> 2) & (DPI - 1));
  p.ab = p.fp - 4 * p.S;
  p.n = p.dead ? 1 : (int)((L - 4 + 3) >> 2);  // covered dwords, the last maybe partial
  const int E = p.S + p.n;
  p.J = (E + DPI - 1) / DPI;
  p.r = E - DPI * (p.J - 1);
  p.jh = (8 + p.S) / DPI + 1;
  return p;
}

// The lane's 16-byte chunk of iteration j; chunks with no covered dword are
// not loaded.  An aligned 4 DPI-byte block never crosses a page, so the bytes
// around the frame that share its blocks are always mapped.  These are the
// head and last chunks, whose 128-B lines the neighbouring frames share:
// cached loads, not the body's non-temporal ones, so the neighbour's read of
// the same line hits L2 instead of going to HBM again: cfg2 +2.7 % (6148 ->
// 6317 GiB/s), cfg3 +2.5 % (5670 -> 5806), 3 of 3 A/B rounds.
// SHARED: a cached load (the head and last iterations, whose lines the
// neighbouring frames share); else non-temporal.  Cached loads of the first
// body block as well measured cfg2 -3 %, cfg3 -2 %; the second head
// iteration non-temporal cfg2 -0.3 %, cfg3 -0.2 % (2 rounds), so it stays
// cached.
template <int G, bool SHARED = true>
__device__ __forceinline__ u32x4 load_chunk(const Pkt& p, int j, int gl) {
  constexpr int DPI = 4 * G;
  const int kb = DPI * j + 4 * gl - p.S;
  u32x4 v = {0, 0, 0, 0};
  if (!p.dead && kb + 3 >= 0 && kb < p.n) {
    if constexpr (SHARED)
      v = *(const u32x4*)(p.ab + 16 * (G * j + gl));
    else
      v = ldg128(p.ab + 16 * (G * j + gl));
  }
  return v;
}

// The slow path's chunk of a frame at an unaligned start or of a length that
// is not a multiple of 4: byte loads of the covered dwords only (nothing
// outside the frame is touched).  The last covered dword of such a length
// holds 1-3 covered bytes; its other bytes (the ICRC slot's) enter as zeros,
// i.e. the frame is CRC'd as if followed by 4 - L % 4 zero bytes, which
// slow_packet takes back out of the register (unshift_zero_bytes).
__device__ __forceinline__ uint32_t ldg32_bytes(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
template <int G>
__device__ __forceinline__ u32x4 load_chunk_bytes(const Pkt& p, int j, int gl) {
  const int kb = 4 * G * j + 4 * gl - p.S;
  const uint32_t m = p.L & 3u;
  const uint32_t keep = m ? (1u << (8u * m)) - 1u : 0xFFFFFFFFu;  // of the last dword
  u32x4 v = {0, 0, 0, 0};
#define RICRC_BYTES(c, t)                                                            \
  if (kb + (t) >= 0 && kb + (t) < p.n) {                                             \
    v.c = ldg32_bytes(p.fp + 4 * (kb + (t)));                                        \
    if (kb + (t) == p.n - 1) v.c &= keep;                                            \
  }
  RICRC_BYTES(x, 0)
  RICRC_BYTES(y, 1)
  RICRC_BYTES(z, 2)
  RICRC_BYTES(w, 3)
#undef RICRC_BYTES
  return v;
}

// The reflected CRC register with `z` zero bytes taken back off its end:
// multiplication by x^(-8 z) mod P, one inverse register step per bit (the
// forward step is r -> (r >> 1) ^ (r & 1 ? P : 0), and P has bit 31 set).
__device__ __forceinline__ uint32_t unshift_zero_bytes(uint32_t r, uint32_t z) {
  for (uint32_t b = 0; b < 8u * z; ++b)
    r = (r & 0x80000000u) ? (((r ^ kPoly) << 1) | 1u) : (r << 1);
  return r;
}

// Body iterations (jh <= j < J-1) lie wholly inside the frame: no predicate.
// A block's U loads go out from one 64-bit address per block (the lane's
// chunk of iteration j) with the iteration steps as immediate offsets
// (16 G u < 4 KiB), instead of a 64-bit address build per load.
template <int G>
__device__ __forceinline__ const uint8_t* body_addr(const Pkt& p, int j, int gl) {
  return p.ab + (uint32_t)(16 * (G * j + gl));  // (frame-relative offsets stay below 2^17)
}
template <int G, int U>
__device__ __forceinline__ void load_block(u32x4 (&w)[U], const uint8_t* q) {
#pragma unroll
  for (int u = 0; u < U; ++u) w[u] = ldg128(q + 16 * G * u);
}


// Head fix-up of one chunk (iterations j < jh) for IHL-5 frames: zero dwords
// before the frame, apply masks and seed, and keep the raw header dwords 0
// and 2.  The per-dword (AND, OR, XOR) triple comes from a 13-entry table in
// LDS indexed by clamp(k + 3, 0, 12) (entries 0-2: k < 0, 3-11: k = 0..8,
// 12: k > 8), one ds_read_b128 and two VALU per dword.
__device__ __forceinline__ void fix_chunk5(u32x4& w, int kb, uint32_t lut, uint32_t& h0,
                                           uint32_t& h2) {
  h0 = pick4(w, -kb, h0);
  h2 = pick4(w, 2 - kb, h2);
  u32x4 e;
#define RICRC_FIX(c, t)                                                            \
  e = *(const lds_u32x4*)(uintptr_t)(lut + 16u * (uint32_t)min(max(kb + (t) + 3, 0), 12)); \
  w.c = ((w.c & e.x) | e.y) ^ e.z;
  RICRC_FIX(x, 0)
  RICRC_FIX(y, 1)
  RICRC_FIX(z, 2)
  RICRC_FIX(w, 3)
#undef RICRC_FIX
}

// General-IHL fix-up (slow path for frames with IPv4 options).
__device__ __forceinline__ void fix_chunk(u32x4& w, int kb, int kub, int kbb, uint32_t& h0,
                                          uint32_t& h2) {
  h0 = pick4(w, -kb, h0);
  h2 = pick4(w, 2 - kb, h2);
  w.x = (kb + 0 < 0) ? 0u : fix_dword(w.x, kb + 0, kub, kbb);
  w.y = (kb + 1 < 0) ? 0u : fix_dword(w.y, kb + 1, kub, kbb);
  w.z = (kb + 2 < 0) ? 0u : fix_dword(w.z, kb + 2, kub, kbb);
  w.w = (kb + 3 < 0) ? 0u : fix_dword(w.w, kb + 3, kub, kbb);
}


// Recomputation of one packet by its group with the masks of a general IHL
// (IPv4 options), or of a frame at an unaligned start (byte loads).  Rare
// path: the main loop applies the IHL-5 masks to dword-aligned frames.
template <int LOG2G, class K>
__device__ __noinline__ uint32_t slow_packet(Pkt p, int ihl, int gl, int base) {
  constexpr int G = 1 << LOG2G;
  const K kk = K::make(__lane_id());  // (rebuilt here: no key registers passed on the stack)
  constexpr int DPI = 4 * G;
  const int kub = ihl + 1, kbb = ihl + 3;
  Col A = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  uint32_t h0 = 0, h2 = 0;
  for (int j = 0; j < p.J; ++j) {
    const int kb = DPI * j + 4 * gl - p.S;
    u32x4 w = p.unal ? load_chunk_bytes<G>(p, j, gl) : load_chunk<G>(p, j, gl);
    fix_chunk(w, kb, kub, kbb, h0, h2);
    if (j == p.J - 1)
      fold_last(A, w, kb, p.n, kk);
    else
      fold(A, w, kk);
  }
  const uint32_t B = combine<LOG2G, K>(A.P[0] ^ A.T[0], A.P[1] ^ A.T[1], A.P[2] ^ A.T[2],
                                       A.P[3] ^ A.T[3], p.r, gl, base);
  return (p.L & 3u) ? unshift_zero_bytes(B, 4u - (p.L & 3u)) : B;
}


// A packet's first batch of loads: head chunks, the first body block and the
// last chunk (plus the trailer in verify mode).  Issued one packet set ahead
// so small packets do not wait a full HBM round trip per set.
template <int U>
struct Batch {
  u32x4 wh0, wh1, wl;
  u32x4 cur[U];
  uint32_t trailer;
};

template <int LOG2G, bool VERIFY>
__device__ __forceinline__ Batch<kUnroll> issue_packet(const Pkt& p, int gl) {
  constexpr int G = 1 << LOG2G;
  constexpr int U = kUnroll;
  Batch<U> b;
  const int JL = p.J - 1;
  const int jhh = min(p.jh, JL);
  const int nbody = JL - jhh;
  const int first = nbody == 0 ? 0 : ((nbody - 1) % U) + 1;
  b.trailer = 0;
  if (VERIFY && !p.dead && gl == 0) b.trailer = ldg32(p.fp + p.L - 4);
  b.wh0 = jhh > 0 ? load_chunk<G>(p, 0, gl) : u32x4{0, 0, 0, 0};
  b.wh1 = jhh > 1 ? load_chunk<G>(p, 1, gl) : u32x4{0, 0, 0, 0};
  {
    const uint8_t* q = body_addr<G>(p, jhh, gl);
#pragma unroll
    for (int u = 0; u < U; ++u)
      b.cur[u] = u < first ? ldg128(q + 16 * G * u) : u32x4{0, 0, 0, 0};
  }
  b.wl = load_chunk<G>(p, JL, gl);
  return b;
}

// Where a block's ICRC words go: packets [p0, p0 + cap) into an LDS buffer
// at kOutLds<LOG2G> (written out whole when the block is done), the rest
// straight to icrc_out.  cap = 0: no buffer.  Likewise the verify verdicts
// of packets [ok_p0, ok_p0 + ok_cap) into LDS bytes at ok_lds (the ragged
// kernel's window, written out at the window's end).
struct OutBuf {
  uint32_t p0, cap;
  uint32_t ok_p0 = 0, ok_cap = 0, ok_lds = 0;
};
__device__ __forceinline__ void lds_wr8(uint32_t byte_addr, uint32_t v) {
  *(__attribute__((address_space(3))) uint8_t*)(uintptr_t)byte_addr = (uint8_t)v;
}
__device__ __forceinline__ uint32_t lds_rd8(uint32_t byte_addr) {
  return *(const __attribute__((address_space(3))) uint8_t*)(uintptr_t)byte_addr;
}
template <int LOG2G>
constexpr uint32_t kOutLds = kFixLut<LOG2G, MainKeys> + 256u;  // after the fix-up LUT

// K: the table layout (MainKeys, or Keys8T in the mixed-width ragged
// kernel); LUT: LDS address of the IHL-5 fix-up table.
template <int LOG2G, bool VERIFY, class K, uint32_t LUT>
__device__ __forceinline__ void emit_packet(const IcrcArgs& a, const Pkt& p, const Col& A,
                                            uint32_t h0, uint32_t h2, uint32_t trailer, int gl,
                                            int base, const K& kk, OutBuf ob);

// A wave issues its next body block's loads (lane-group kernels) or its next
// batch's prefetch (small-frame kernel) at raised priority, so the sequencer
// sends loads out ahead of other waves' folds and the HBM queue stays full:
// cfg2 +0.5 % (6012 -> 6042 GiB/s, 3 A/B rounds on each of two boxes;
// priority 2 the same, cfg3 and the segmentation kernel neutral, also raising
// it for a packet's first batch measured worse), cfg5 +2.5-12 %.
__device__ __forceinline__ void body_prio_hi() { __builtin_amdgcn_s_setprio(3); }
__device__ __forceinline__ void body_prio_lo() { __builtin_amdgcn_s_setprio(0); }

// Fold, combine, check and emit one packet whose first batch is in `b`.
template <int LOG2G, bool VERIFY, class K = MainKeys, uint32_t LUT = kFixLut<LOG2G, MainKeys>>
__device__ __forceinline__ void finish_packet(const IcrcArgs& a, const Pkt& p, Batch<kUnroll>& b,
                                              int gl, int base, const K& kk,
                                              OutBuf ob = {0, 0}) {
  constexpr int G = 1 << LOG2G;
  constexpr int DPI = 4 * G;
  constexpr int U = kUnroll;
  constexpr uint32_t kLut = LUT;
  // Iterations: head [0, jhh) with the fix-ups, body [jhh, J-1) in blocks of
  // U (the first block holds the remainder), then the last one (J-1), which
  // skips columns past the end and may also need the fix-ups.
  const int JL = p.J - 1;
  const int jhh = min(p.jh, JL);
  const int nbody = JL - jhh;
  const int first = nbody == 0 ? 0 : ((nbody - 1) % U) + 1;
  const int nblk = (nbody + U - 1) / U;

  Col A = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  uint32_t h0 = 0, h2 = 0;
  for (int j = 0; j < jhh; ++j) {
    u32x4 w = (j == 0) ? b.wh0 : (j == 1) ? b.wh1 : load_chunk<G, false>(p, j, gl);
    fix_chunk5(w, DPI * j + 4 * gl - p.S, kLut, h0, h2);
    fold(A, w, kk);
  }
  // body blocks, ping-pong between b.cur and nxt (no register copies)
  int j0 = jhh, bs = first;
  u32x4 nxt[U];
  for (int bk = 0; bk < nblk; bk += 2) {
    int jn = j0 + bs;
    if (bk + 1 < nblk) {
      body_prio_hi();
      load_block<G, U>(nxt, body_addr<G>(p, jn, gl));
      body_prio_lo();
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < bs) fold(A, b.cur[u], kk);
    if (bk + 1 >= nblk) break;
    j0 = jn;
    jn = j0 + U;
    if (bk + 2 < nblk) {
      body_prio_hi();
      load_block<G, U>(b.cur, body_addr<G>(p, jn, gl));
      body_prio_lo();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) fold(A, nxt[u], kk);
    j0 = jn;
    bs = U;
  }
  {
    u32x4 w = b.wl;
    const int kb = DPI * JL + 4 * gl - p.S;
    if (JL < p.jh) fix_chunk5(w, kb, kLut, h0, h2);
    fold_last(A, w, kb, p.n, kk);
  }
  emit_packet<LOG2G, VERIFY, K, LUT>(a, p, A, h0, h2, b.trailer, gl, base, kk, ob);
}

// Packet done: fold the group's columns, check the header, emit.
template <int LOG2G, bool VERIFY, class K, uint32_t LUT>
__device__ __forceinline__ void emit_packet(const IcrcArgs& a, const Pkt& p, const Col& A,
                                            uint32_t h0, uint32_t h2, uint32_t trailer, int gl,
                                            int base, const K& kk, OutBuf ob) {
  constexpr int G = 1 << LOG2G;
  constexpr int DPI = 4 * G;
  uint32_t B = combine<LOG2G, K>(A.P[0] ^ A.T[0], A.P[1] ^ A.T[1], A.P[2] ^ A.T[2],
                                 A.P[3] ^ A.T[3], p.r, gl, base);
  uint32_t d0 = (uint32_t)__shfl((int)h0, base + (p.S >> 2), 64);
  uint32_t d2 = (uint32_t)__shfl((int)h2, base + (((p.S + 2) & (DPI - 1)) >> 2), 64);
  if (p.unal) {  // (per group) frame at an unaligned start: header bytes read directly
    d0 = ldg32_bytes(p.fp);
    d2 = ldg32_bytes(p.fp + 8);
    if (VERIFY) trailer = ldg32_bytes(p.fp + p.L - 4);
  }
  uint32_t st = (p.dead && !p.unal) ? kPktBadLen : 0u;
  const int ihl = (int)(d0 & 0xFu);
  if (st == 0) {
    if (((d0 >> 4) & 0xFu) != 4u || ihl < 5)
      st |= kPktNotIpv4;
    else if (((d2 >> 8) & 0xFFu) != 17u)
      st |= kPktNotUdp;
    else if (p.L < (uint32_t)(4 * ihl + 24))
      st |= kPktBadLen;
    const uint32_t tot = ((d0 >> 8) & 0xFF00u) | (d0 >> 24);
    if (tot != p.L) st |= kPktLenMismatch;
  }
  const bool good = (st & kPktFatal) == 0;
  if (good && (ihl != 5 || p.unal))
    B = slow_packet<LOG2G, K>(p.unal ? describe<DPI>(p.fp, p.pkt, true, 0, p.L, true) : p, ihl, gl,
                              base);
  const uint32_t icrc = good ? ~B : 0u;
  if (p.live && gl == 0) {
    if constexpr (VERIFY) {
      const bool ok = good && trailer == icrc;
      if (good && !ok) st |= kPktIcrcMismatch;
      const uint32_t ko = p.pkt - ob.ok_p0;
      if (ko < ob.ok_cap)
        lds_wr8(ob.ok_lds + ko, ok ? 1u : 0u);
      else
        stg8<kPktStorePol>(a.ok_out + p.pkt, ok ? 1u : 0u);
    }
    if (a.icrc_out) {
      const uint32_t k = p.pkt - ob.p0;
      if (k < ob.cap)
        lds_wr(kOutLds<LOG2G> + 4u * k, icrc);
      else
        stg32<kPktStorePol>(a.icrc_out + p.pkt, icrc);
    }
    if (a.status_out) stg8<kPktStorePol>(a.status_out + p.pkt, st);
  }
}

// Tail stealing (strided kernel): the last 1/kTailDiv of a workgroup's sets
// are claimed dynamically; a finished wave tries up to kMaxVictims other
// workgroups' tails.  Round 3, cfg2 kernel ms (3 A/B rounds each, two
// sessions, profiles/r03q_tail_ab*.txt): 1/2 0.6417, 1/4 0.6309, 1/8
// 0.6246 (+1.0 %), 1/16 0.6353, 1/32 0.6364; 2 victims at 1/8 0.6274, 8
// victims at 1/4 0.6324.
constexpr uint32_t kTailDiv = 8;
constexpr uint32_t kMaxVictims = 4;

// Cache policy of the block's output run (out_store128): default.  The run
// goes out at the end of the block, when the rest of the chip still streams;
// sc1 measured 0.5 % slower on cfg2 (3 A/B rounds).
constexpr int kStridedOutPol = 0;

// Fixed-size frames at frames + i * stride.
template <int LOG2G, bool VERIFY>
__global__ void __launch_bounds__(kStridedThreads, 1) icrc_strided_kernel(IcrcArgs a) {
  constexpr int G = 1 << LOG2G;
  constexpr int PPW = 64 / G;  // packets per wave step
  const int tid = threadIdx.x;
  announce_batch(a.busy);
  stage_tables<LOG2G, kStridedThreads, MainKeys>(a.tables, tid);
  __syncthreads();

  const int lane = tid & 63;
  const int gl = lane & (G - 1);
  const int grp = lane >> LOG2G;
  const MainKeys kk = MainKeys::make(lane);
  // Each workgroup owns a contiguous range of packet sets, so every CU sweeps
  // one contiguous region of HBM (measured: 6.8 vs 5.6 TB/s for
  // grid-interleaved sets); its 16 waves take consecutive sets of that range.
  const uint32_t nsets = (a.n + PPW - 1) / PPW;
  const uint32_t per_block = (nsets + gridDim.x - 1) / gridDim.x;
  // A workgroup's range [begin, end) of sets; its last 1/kTailDiv ("tail")
  // is claimed set by set through a counter that other workgroups may also
  // claim from once their own range is done (see below).
  auto range = [&](uint32_t blk, uint32_t& b, uint32_t& e, uint32_t& split) {
    b = blk * per_block;
    e = min(nsets, b + per_block);
    const uint32_t len = b < e ? e - b : 0u;
    split = e - (a.claims ? len / kTailDiv : 0u);
  };
  uint32_t set_begin, set_end, set_split;
  range(blockIdx.x, set_begin, set_end, set_split);
  unsigned long long* claims =
      a.claims ? a.claims + (size_t)(a.epoch % kClaimSlots) * kMaxClaimBlocks : nullptr;
  if (claims && tid == 0) atomicExch(&claims[blockIdx.x], (unsigned long long)a.epoch << 32);
  constexpr int DPI = 4 * G;
  auto make = [&](uint32_t set) {
    const uint32_t pkt = set * PPW + grp;
    const bool live = set < nsets && pkt < a.n;
    return describe<DPI>(a.frames, pkt, live, live ? (uint64_t)pkt * a.stride : 0,
                         live ? a.len : 0);
  };
  // The block's ICRC words collect in LDS and go out as one contiguous,
  // coalesced run at the end: 4-byte words written while the frames stream in
  // cost 2.5 % at cfg2 (measured with the stores ablated), HBM writes mixed
  // into the read stream being expensive (small-frame kernel).
  // Only the statically owned sets use the buffer (tail sets may be claimed
  // by another workgroup, which writes their words straight to icrc_out).
  const uint32_t p0 = set_begin * PPW;
  const uint32_t p1 = set_begin < set_split ? min(a.n, set_split * PPW) : p0;
  const OutBuf ob = {p0, min(p1 - p0, (163840u - kOutLds<LOG2G>) / 4u)};
  // (issuing the next set's first batch before finishing this one was
  // measured: no gain at 4 KiB or 108-B frames, and register spills)
  for (uint32_t set = set_begin + (uint32_t)(tid >> 6); set < set_split;
       set += (uint32_t)kStridedWaves) {
    const Pkt p = make(set);
    Batch<kUnroll> b = issue_packet<LOG2G, VERIFY>(p, gl);
    finish_packet<LOG2G, VERIFY>(a, p, b, gl, grp * G, kk, ob);
  }
  // Tail: the workgroups on some XCDs stream measurably slower than others
  // (cfg2: odd XCDs end ~3 % later), so with static ranges the launch waits
  // for the slowest.  A wave that is done claims single sets from its own
  // tail (one returning atomic per set on its workgroup's counter, issued
  // one set ahead so its latency hides behind the current set), then from
  // the tails of workgroups blk + 1, blk + 3, ... (the other XCD parity
  // first), up to kMaxVictims of them.  A counter still holding an older
  // epoch (its owner has not started yet) counts as empty.
  if (claims) {
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
    uint32_t cur = claim(victim);
    for (;;) {
      if (cur == ~0u) {
        if (++tries > kMaxVictims) break;
        victim = (blockIdx.x + 2 * tries - 1) % gridDim.x;
        cur = claim(victim);
        continue;
      }
      const Pkt p = make(cur);
      Batch<kUnroll> b = issue_packet<LOG2G, VERIFY>(p, gl);
      cur = claim(victim);  // the next set, while this one streams in
      finish_packet<LOG2G, VERIFY>(a, p, b, gl, grp * G, kk, OutBuf{0, 0});
    }
  }
  if (a.icrc_out) {  // (uniform)
    __syncthreads();
    const auto dst = out_rsrc(a.icrc_out + p0, 4u * ob.cap);
    for (uint32_t i = (uint32_t)tid; i < ob.cap / 4u; i += kStridedThreads)
      out_store128<kStridedOutPol>(*(const lds_u32x4*)(uintptr_t)(kOutLds<LOG2G> + 16u * i), dst,
                                   16u * i);
    for (uint32_t i = (ob.cap & ~3u) + (uint32_t)tid; i < ob.cap; i += kStridedThreads)
      out_store32<kStridedOutPol>(lds_rd(kOutLds<LOG2G> + 4u * i), dst, 4u * i);
  }
}

// Ragged frames (offsets[i], lens[i]).  The lanes of a wave fold their
// packets in lockstep, so a wave waits for the longest packet of its set.
// Each workgroup therefore takes a contiguous window of packets (locality
// kept) and counting-sorts it in LDS by iteration count; waves then claim
// size-homogeneous sets of the sorted window from both ends.
template <uint32_t BASE, int CAP = 8192>
struct WindowLds {
  static constexpr uint32_t kBase = BASE;  // after the tables and the fix-up LUT
  static constexpr int kBuckets = 128;
  static constexpr uint32_t kHist = kBase;               // kBuckets x u32 counts / cursors
  static constexpr uint32_t kPerm = kBase + 4 * kBuckets;  // window x u16 local indices
  static constexpr int kAvail = (int)(163840u - kPerm);
  // sorted descriptors: u16 local index, u32 offset / 4, u16 length (8 B),
  // then the window's verify verdicts (1 B, in packet order)
  static constexpr int kWindow = (kAvail / 9 >= CAP) ? CAP : (kAvail / 9) / 64 * 64;
  static constexpr uint32_t kRoff = kPerm + 2 * kWindow;
  static constexpr uint32_t kRlen = kRoff + 4 * kWindow;
  static constexpr uint32_t kOk = kRlen + 2 * kWindow;
  static constexpr uint32_t kBytes = kOk + kWindow;
};
template <int LOG2G>
using RaggedLds = WindowLds<kFixLut<LOG2G, MainKeys> + 256u>;

template <int LOG2G, bool VERIFY>
__global__ void __launch_bounds__(kIcrcThreads, 1) icrc_ragged_kernel(IcrcArgs a) {
  constexpr int G = 1 << LOG2G;
  constexpr int PPW = 64 / G;
  constexpr int DPI = 4 * G;
  using LD = RaggedLds<LOG2G>;
  constexpr int W = LD::kWindow;
  constexpr int NB = LD::kBuckets;
  static_assert(W + kIcrcWaves < 65536, "set claims are 16-bit counters");
  const int tid = threadIdx.x;
  announce_batch(a.busy);
  stage_tables<LOG2G, kIcrcThreads, MainKeys>(a.tables, tid);

  const int lane = tid & 63;
  const int gl = lane & (G - 1);
  const int grp = lane >> LOG2G;
  const MainKeys kk = MainKeys::make(lane);
  const uint32_t per_block = (a.n + gridDim.x - 1) / gridDim.x;
  const uint32_t p0 = blockIdx.x * per_block;
  const uint32_t p1 = min(a.n, p0 + per_block);
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  lds_u32* hist = (lds_u32*)(uintptr_t)LD::kHist;
  lds_u16* perm = (lds_u16*)(uintptr_t)LD::kPerm;
  lds_u32* roff = (lds_u32*)(uintptr_t)LD::kRoff;
  lds_u16* rlen = (lds_u16*)(uintptr_t)LD::kRlen;
  constexpr uint32_t kNoOff = 0xFFFFFFFFu;  // offset not representable: read it from HBM
  lds_u32* claim = (lds_u32*)(uintptr_t)(LD::kBase - 4u);  // (free word at the end of the LUT)
  const bool from_back = ((tid >> 6) & 1) != 0;

  // windows of equal size (<= W): no short last window with few sets per wave
  const uint32_t nwin = p1 > p0 ? (p1 - p0 + W - 1) / W : 1;
  const uint32_t wsz = p1 > p0 ? (p1 - p0 + nwin - 1) / nwin : 1;
  for (uint32_t w0 = p0; w0 < p1; w0 += wsz) {
    const int cnt = (int)min(wsz, p1 - w0);
    if (tid < NB) hist[tid] = 0;
    if (tid == NB) *claim = 0;
    __syncthreads();
    // iteration count of every packet of the window -> bucket
    constexpr int KR = (W + kIcrcThreads - 1) / kIcrcThreads;
    int keys[KR];
    uint32_t offw[KR], lw[KR];
    // every descriptor load of the thread first (clamped, unconditional: a
    // guarded load makes the compiler wait for each in turn), then the keys
    uint32_t Lr[KR];
    uint64_t Or[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const int ic = min(tid + r * kIcrcThreads, cnt - 1);
      Lr[r] = a.lens[w0 + ic];
      Or[r] = a.offsets[w0 + ic];
    }
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const int i = tid + r * kIcrcThreads;
      int key = 0;
      offw[r] = kNoOff;
      lw[r] = 0;
      if (i < cnt) {
        const uint32_t L = Lr[r];
        const uint64_t off = Or[r];
        if (off < (1ull << 34) && (off & 3u) == 0) offw[r] = (uint32_t)(off >> 2);
        lw[r] = L > 65535u ? 0u : L;  // (0: unusable, as L > 65535 is)
        if (!(L < 44 || (L & 3u) || L > 65535u || ((uintptr_t)(a.frames + off) & 3u))) {
          const int S = (int)(((uintptr_t)(a.frames + off) >> 2) & (DPI - 1));
          key = min(NB - 1, (S + (int)((L - 4) >> 2) + DPI - 1) / DPI);
        }
        atomicAdd((uint32_t*)&hist[key], 1u);
      }
      keys[r] = key;
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of NB = 128 counts by one wave (2 per lane)
      const uint32_t c0 = hist[2 * tid], c1 = hist[2 * tid + 1];
      uint32_t s = c0 + c1;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)s, d, 64);
        if (tid >= d) s += t;
      }
      const uint32_t excl = s - c0 - c1;
      hist[2 * tid] = excl;
      hist[2 * tid + 1] = excl + c0;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const int i = tid + r * kIcrcThreads;
      if (i < cnt) {
        const uint32_t pos = atomicAdd((uint32_t*)&hist[keys[r]], 1u);
        perm[pos] = (uint16_t)i;
        roff[pos] = offw[r];
        rlen[pos] = (uint16_t)lw[r];
      }
    }
    __syncthreads();
    const int nsets = (cnt + PPW - 1) / PPW;
    auto make = [&](int set) {
      const int idx = set * PPW + grp;
      const bool live = set < nsets && idx < cnt;
      const int ix = live ? idx : 0;
      const uint32_t pkt = w0 + perm[ix], ow = roff[ix];
      const uint64_t off = ow != kNoOff ? (uint64_t)ow << 2 : a.offsets[pkt];
      return describe<DPI>(a.frames, pkt, live, live ? off : 0, live ? (uint32_t)rlen[ix] : 0);
    };
    // Dynamic claims from both ends of the sorted window (one LDS atomic per
    // set on a packed front | back << 16 counter): even waves take the short
    // sets, odd waves the long ones, so a CU mixes instruction-bound and
    // load-bound sets, and no wave idles at the window barrier while sets
    // remain.  Measured against round robin: cfg3 +3-6 %, 2 KiB frames +3 %,
    // 256 B +5 %; a quarter or three quarters of the waves taking the long
    // sets, or claiming the next set before finishing the current one, were
    // no better.
    // verify verdicts collect in LDS and leave as one run per window
    // (written one by one into the read stream they cost 1.3 %, ablated)
    OutBuf ob = {0, 0};
    if constexpr (VERIFY) {
      ob.ok_p0 = w0;
      ob.ok_cap = (uint32_t)cnt;
      ob.ok_lds = LD::kOk;
    }
    for (;;) {
      uint32_t old = 0;
      if (lane == 0) old = atomicAdd((uint32_t*)claim, from_back ? 0x10000u : 1u);
      old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
      const int f = (int)(old & 0xFFFFu), bk = (int)(old >> 16);
      if (f + bk >= nsets) break;
      const int set = from_back ? nsets - 1 - bk : f;
      const Pkt p = make(set);
      Batch<kUnroll> b = issue_packet<LOG2G, VERIFY>(p, gl);
      finish_packet<LOG2G, VERIFY>(a, p, b, gl, grp * G, kk, ob);
    }
    __syncthreads();
    if constexpr (VERIFY) {  // the window's verdicts, one contiguous run
      for (int i = tid; i < cnt; i += kIcrcThreads) a.ok_out[w0 + i] = (uint8_t)lds_rd8(LD::kOk + i);
    }
  }
}

// ---------------------------------------------------------------------------
// Mixed-width ragged kernel (the G = 8 choice for ragged batches).
//
// Short frames are instruction-bound in a lane group: at 256-B MTU a G = 8
// set spends ~90 % of its instructions on per-packet work (describe, head
// fix-ups, rotation, combine) that every lane of the group pays.  Halving the
// group halves that cost per packet, while long frames need G = 8 for whole
// 128-B lines per group load.  This kernel holds both table sets -- Mul(1024)
// for G = 8 and Mul(512) for G = 4, in the two halves of the Keys8 rows (64
// KiB together, icrc_device.hpp) -- and picks the width per set of the sorted
// window: the front waves claim 16 packets from the short end and run them as
// ONE G = 4 set when the claim's longest frame is short, else as two G = 8
// sets; the back waves claim 8 from the long end at G = 8.  The combine sets
// Mul(-32), Mul(-128 * 2^l) (l < 3) serve both widths.  The tables take 80 KiB
// instead of 144, so a window holds up to 8192 packets (one window per
// workgroup at cfg3).
//
// Claims are packets on the packed front | back << 16 counter.  A front claim
// at (f, bk) owns [f, min(f + 16, cnt - bk)); a back claim owns
// [max(cnt - bk - 8, f), cnt - bk): each side sees the other's position at
// its own atomic, so the ranges are disjoint.
//
// Tiny frames (ACK / NAK / atomic-ack sized, <= kTinyLen bytes) are
// instruction-bound even at G = 4: a G = 1 set (one lane per packet, 64
// packets per wave) does a quarter of the per-packet work.  The sort gives
// them a bucket of their own at the front of the window; when a window holds
// at least kTinyMin of them, they run first as G = 1 sets ("phase A") with
// Mul(128) staged into the G = 4 half of the Keys8 rows, and the G = 4 table
// is restaged for the rest of the window (barriers around both restages; a
// window of tiny frames only keeps Mul(128) for the next window).
// Frames of at most this many bytes (the claim's last, i.e. longest, sorted
// frame) run as G = 4 sets.
constexpr uint32_t kMixedShortLen = 600;
constexpr uint32_t kTinyLen = 128;  // frames run as G = 1 sets (0: never)
constexpr int kTinyMin = 256;       // tiny frames a window needs for phase A
using MixedKeysL = Keys8T<0>;  // Mul(1024), G = 8
using MixedKeysS = Keys8T<1>;  // Mul(512), G = 4
constexpr uint32_t kMixedLut = kFixLut<3, MixedKeysL>;  // after the 4 combine sets
constexpr int kMixedWindow = 8192;  // packets per window (the sort's LDS arrays)
using MixedLds = WindowLds<kMixedLut + 256u, kMixedWindow>;

// The four-chain fold of the small kernel (and the ragged kernel's compact
// tiny batches) over dwords [0, n) of one frame,
// each dword through the per-dword masks of an IHL of `ihl` (IPv4 options,
// malformed frames, the last batch read straight from global memory: frame at
// `f`; else the frame staged in LDS at `pb`).  Out of line: its per-dword
// mask constants are uniform values the hot loop would otherwise keep live
// (they were ~200 SGPRs spilled to VGPR lanes in round 2, all in this path).
// Mul(-32) for the four-chain folds: from the unreplicated combine set at LDS
// address COMB, or (COMB == kComb8) from the 8-copy Keys8 layout in the high
// halves of the table rows (conflict-free, one v_perm per address; the
// selectors are those of the low-half keys).
constexpr uint32_t kComb8 = 0xFFFFFFFFu;
template <uint32_t COMB, class K>
__device__ __forceinline__ uint32_t comb4(uint32_t x, const K& kk) {
  if constexpr (COMB == kComb8) {
    Keys8T<1> kc;
    kc.k = kk.k | 0x80808080u;
    kc.s0 = kk.s0;
    kc.s1 = kk.s1;
    kc.s2 = kk.s2;
    kc.s3 = kk.s3;
    uint32_t P = 0, T = 0;
    kc.absorb(P, T, x);
    return P ^ T;
  } else {
    return mul_comb(x, COMB);
  }
}

template <bool GLOBAL, class K, uint32_t COMB, int CH = 4>
__device__ __forceinline__ uint32_t fold_masked4(const uint8_t* f, uint32_t pb, int ihl, int n) {
  // CH chains (K's table is Mul(32 CH)): chain c takes dwords k = CH j + c - pad
  const K kk = K::make(__lane_id());
  const int ns = (n + CH - 1) / CH, pad = CH * ns - n;
  uint32_t P[CH], T[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) P[c] = T[c] = 0;
  for (int j = 0; j < ns; ++j) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int k = CH * j + c - pad;
      uint32_t w = 0;
      if (k >= 0) w = fix_dword(GLOBAL ? ldg32(f + 4 * k) : lds_rd(pb + 4u * (uint32_t)k), k,
                                ihl + 1, ihl + 3);
      kk.absorb(P[c], T[c], w);
    }
  }
  uint32_t R = P[CH - 1] ^ T[CH - 1];
#pragma unroll
  for (int c = CH - 2; c >= 0; --c) R = comb4<COMB>(R, kk) ^ P[c] ^ T[c];
  return R;
}
template <bool GLOBAL, class K, uint32_t COMB, int CH = 4>
__device__ __noinline__ uint32_t small_fold_masked(const uint8_t* f, uint32_t pb, int ihl, int n) {
  return fold_masked4<GLOBAL, K, COMB, CH>(f, pb, ihl, n);
}
// The same fold of a frame in global memory (n <= kSmallMaxStride / 4 - 1
// covered dwords, any IHL): every dword is loaded first, so the frame costs
// one memory round trip instead of one per step: the small-frame kernel's
// last batch, at the very end of the launch (inline there: its registers are
// free; the in-loop fallback for IPv4 options keeps the call above).
template <class K, uint32_t COMB, int CH>
__device__ __forceinline__ uint32_t small_fold_masked_global(const uint8_t* f, int ihl, int n) {
  constexpr int KP = (int)(kSmallMaxStride / 4u);  // padded dwords kp = k + pad < KP
  const K kk = K::make(__lane_id());
  const int ns = (n + CH - 1) / CH, pad = CH * ns - n;
  uint32_t D[KP];
#pragma unroll
  for (int kp = 0; kp < KP; ++kp) D[kp] = ldg32(f + 4 * max(min(kp - pad, n - 1), 0));
  uint32_t P[CH], T[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) P[c] = T[c] = 0;
#pragma unroll
  for (int j = 0; j < KP / CH; ++j) {
    if (j < ns) {  // uniform
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int kp = CH * j + c, k = kp - pad;
        kk.absorb(P[c], T[c], k >= 0 ? fix_dword(D[kp], k, ihl + 1, ihl + 3) : 0u);
      }
    }
  }
  uint32_t R = P[CH - 1] ^ T[CH - 1];
#pragma unroll
  for (int c = CH - 2; c >= 0; --c) R = comb4<COMB>(R, kk) ^ P[c] ^ T[c];
  return R;
}

// Compact groups (the ragged COMPACT variant, icrc_compact_kernel below): 64
// consecutive packets whose frames (44-128 B, dword-aligned) lie in order,
// without overlap, inside one 4 KiB span from the first frame's 16-byte line.
constexpr uint32_t kCompactSpan = 4096;                        // bytes one wave stages per group
constexpr int kCompactLoads = (int)(kCompactSpan / 16u / 64u);  // 16-byte loads per lane
constexpr uint32_t kCompactMaxLen = 128;                        // longest frame a group may hold
// a group's words (one coalesced 256-B store per wave) are written
// non-temporally: ACK bench +1.6-3 % over 3 A/B rounds against the default
// policy (whole-library nt builds: cfg3 neutral; sc1 -1.5 %; profiles/r04x)
constexpr int kCompactStorePol = 2;
constexpr uint32_t kMixedLdsBytes = MixedLds::kBytes;
static_assert(kMixedLdsBytes <= 163840u, "LDS");

template <int LOG2G, bool VERIFY, class K>
__device__ __forceinline__ void mixed_set(const IcrcArgs& a, int s, int e, uint32_t w0, int lane,
                                          const OutBuf& ob) {
  constexpr int G = 1 << LOG2G;
  constexpr int DPI = 4 * G;
  using LD = MixedLds;
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  const lds_u16* perm = (const lds_u16*)(uintptr_t)LD::kPerm;
  const lds_u32* roff = (const lds_u32*)(uintptr_t)LD::kRoff;
  const lds_u16* rlen = (const lds_u16*)(uintptr_t)LD::kRlen;
  // the lane's per-width constants are rebuilt per set (an opaque copy of the
  // lane id), not hoisted out of the claim loop: registers held for one width
  // would be taken from the other's loads in flight
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const int gl = ln & (G - 1), grp = ln >> LOG2G;
  const K kk = K::make(ln);
  const int idx = s + grp;
  const bool live = idx < e;
  const int ix = live ? idx : s;
  const uint32_t pkt = w0 + perm[ix], ow = roff[ix];
  const uint64_t off = ow != 0xFFFFFFFFu ? (uint64_t)ow << 2 : a.offsets[pkt];
  const Pkt p = describe<DPI>(a.frames, pkt, live, live ? off : 0, live ? (uint32_t)rlen[ix] : 0);
  Batch<kUnroll> b = issue_packet<LOG2G, VERIFY>(p, gl);
  finish_packet<LOG2G, VERIFY, K, kMixedLut>(a, p, b, gl, grp * G, kk, ob);
}

// The workgroup's windows.  (Round 4's compact tiny batches inside the
// windows -- "phase 0" -- became a kernel of their own in round 5,
// icrc_compact_kernel below.)
// Prologue: the first window's descriptors go out first, then the table
// words (issue_tables), then the tables are written to LDS (write_tables):
// one round trip for both instead of two in a row at the start of every
// launch.  (Writing the tables only after the first window's keys are
// counted kept their words live across the window loop: spilled.)
template <bool VERIFY, class IssueTables, class WriteTables>
__device__ __forceinline__ void mixed_windows(const IcrcArgs& a, int tid, IssueTables issue_tables,
                                              WriteTables write_tables) {
  constexpr int DPI = 32;  // sort key: G = 8 iterations
  using LD = MixedLds;
  constexpr int W = LD::kWindow;
  constexpr int NB = LD::kBuckets;
  static_assert(W + 16 < 65536, "claims are 16-bit counters");
  const int lane = tid & 63;
  const uint32_t per_block = (a.n + gridDim.x - 1) / gridDim.x;
  const uint32_t p0 = blockIdx.x * per_block;
  const uint32_t p1 = min(a.n, p0 + per_block);
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  lds_u32* hist = (lds_u32*)(uintptr_t)LD::kHist;
  lds_u16* perm = (lds_u16*)(uintptr_t)LD::kPerm;
  lds_u32* roff = (lds_u32*)(uintptr_t)LD::kRoff;
  lds_u16* rlen = (lds_u16*)(uintptr_t)LD::kRlen;
  constexpr uint32_t kNoOff = 0xFFFFFFFFu;
  lds_u32* claim = (lds_u32*)(uintptr_t)(LD::kBase - 4u);  // (free words at the end of the LUT)
  lds_u32* tclaim = (lds_u32*)(uintptr_t)(LD::kBase - 8u);  // phase A's claim counter
  const bool from_back = ((tid >> 6) & 1) != 0;
  bool s_tiny = false;  // (uniform) the G = 4 half holds Mul(128) instead of Mul(512)

  const uint32_t nwin = p1 > p0 ? (p1 - p0 + W - 1) / W : 1;
  const uint32_t wsz = p1 > p0 ? (p1 - p0 + nwin - 1) / nwin : 1;
  constexpr int KR = (W + kIcrcThreads - 1) / kIcrcThreads;
  uint32_t Lr[KR];
  uint64_t Or[KR];
  // every descriptor load of the thread first (clamped, unconditional: a
  // guarded load makes the compiler wait for each in turn)
  auto load_descriptors = [&](uint32_t w, int n) __attribute__((always_inline)) {
    // (an opaque window start, which the round-4 phase 0 needed against
    // spills; kept: the sorted kernel's code is unchanged by it)
    asm volatile("" : "+s"(w));
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const int ic = min(tid + r * kIcrcThreads, n - 1);
      Lr[r] = a.lens[w + ic];
      Or[r] = a.offsets[w + ic];
    }
  };
  // Lr / Or are dead once the keys are computed: their registers hold no
  // value (freeze(poison)) from there to the next window's load, so the
  // window loop's back edge does not keep them live across the phases
  auto kill_descriptors = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      Lr[r] = __builtin_nondeterministic_value(Lr[r]);
      Or[r] = __builtin_nondeterministic_value(Or[r]);
    }
  };
  if (p0 < p1) load_descriptors(p0, (int)min(wsz, p1 - p0));  // (uniform) the first window's
  issue_tables();
  write_tables();
  bool first = true;  // (uniform)
  for (uint32_t w0 = p0; w0 < p1; w0 += wsz) {
    const int cnt = (int)min(wsz, p1 - w0);
    if (tid < NB) hist[tid] = 0;
    if (tid == NB) *claim = 0;
    if (tid == NB + 1) *tclaim = 0;
    __syncthreads();
    int keys[KR];
    uint32_t offw[KR], lw[KR];  // (the sort runs outside the set loop: registers are free)
    if (!first) load_descriptors(w0, cnt);
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const bool compact = false;  // (round 4: the packet of a compact batch)
      // sort key, offset / 4 and length of window packet i
      const int i = tid + r * kIcrcThreads;
      int key = 0;
      offw[r] = kNoOff;
      lw[r] = 0;
      if (i < cnt && !compact) {
        const uint32_t L = Lr[r];
        const uint64_t off = Or[r];
        if (off < (1ull << 34) && (off & 3u) == 0) offw[r] = (uint32_t)(off >> 2);
        lw[r] = L > 65535u ? 0u : L;  // (0: unusable, as L > 65535 is)
        if (!(L < 44 || (L & 3u) || L > 65535u || ((uintptr_t)(a.frames + off) & 3u))) {
          const int S = (int)(((uintptr_t)(a.frames + off) >> 2) & (DPI - 1));
          // bucket 0: tiny frames (and unusable ones, which cost nothing)
          key = L <= kTinyLen ? 0 : min(NB - 1, 1 + (S + (int)((L - 4) >> 2) + DPI - 1) / DPI);
        }
      }
      keys[r] = compact ? -1 : key;
      // (one LDS atomic per packet: wave-aggregated adds, one per distinct
      // key, measured no faster)
      const bool counted = i < cnt && !compact;
      if (counted) atomicAdd((uint32_t*)&hist[keys[r]], 1u);
    }
    kill_descriptors();
    first = false;
    __syncthreads();
    OutBuf ob = {0, 0};
    if constexpr (VERIFY) {
      ob.ok_p0 = w0;
      ob.ok_cap = (uint32_t)cnt;
      ob.ok_lds = LD::kOk;
    }
    const int cs = cnt;  // (uniform) the packets the sort phases take
    // (uniform) the window's tiny frames, sorted to its front
    const int ntiny_all = (int)__builtin_amdgcn_readfirstlane((int)hist[0]);
    const int ntiny = ntiny_all >= kTinyMin ? ntiny_all : 0;
    __syncthreads();  // every wave has read hist[0] before the scan rewrites it
    if (tid < 64) {  // exclusive scan of NB = 128 counts by one wave (2 per lane)
      const uint32_t c0 = hist[2 * tid], c1 = hist[2 * tid + 1];
      uint32_t s = c0 + c1;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)s, d, 64);
        if (tid >= d) s += t;
      }
      const uint32_t excl = s - c0 - c1;
      hist[2 * tid] = excl;
      hist[2 * tid + 1] = excl + c0;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const int i = tid + r * kIcrcThreads;
      const bool placed = i < cnt && keys[r] >= 0;
      uint32_t pos = 0;
      if (placed) pos = atomicAdd((uint32_t*)&hist[keys[r]], 1u);
      if (placed) {
        perm[pos] = (uint16_t)i;
        roff[pos] = offw[r];
        rlen[pos] = (uint16_t)lw[r];
      }
    }
    __syncthreads();
    // ---- phase A: the tiny prefix [0, ntiny) as G = 1 sets of 64 packets,
    // claimed from both ends, with Mul(128) in the Keys8 rows' G = 4 half
    if (ntiny > 0) {
      if (!s_tiny) {
        MixedKeysS::template stage<kIcrcThreads>(a.tables + 0 * 1024, tid);  // main set 0: Mul(128)
        s_tiny = true;
        __syncthreads();
      }
      for (;;) {
        uint32_t old = 0;
        if (lane == 0) old = atomicAdd((uint32_t*)tclaim, from_back ? (64u << 16) : 64u);
        old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
        const int f = (int)(old & 0xFFFFu), bk = (int)(old >> 16);
        if (f + bk >= ntiny) break;
        const int e = from_back ? ntiny - bk : min(f + 64, ntiny - bk);
        const int s = from_back ? max(e - 64, f) : f;
        mixed_set<0, VERIFY, MixedKeysS>(a, s, e, w0, lane, ob);
      }
      __syncthreads();  // phase A done before its table is replaced
    }
    if (ntiny < cs && s_tiny) {  // (uniform) phase B needs Mul(512) back
      MixedKeysS::template stage<kIcrcThreads>(a.tables + 2 * 1024, tid);
      s_tiny = false;
      __syncthreads();
    }
    // ---- phase B: [ntiny, cs) as G = 4 / G = 8 sets (below), claims
    // counted from ntiny
    const int nb = cs - ntiny;
    // Claim size: 16 packets while the frames at this wave's end of the window
    // are short, else 8.  Decided from the window's first 16 / last frame, then
    // from the wave's own previous claim (the front end only grows longer, the
    // back end only shorter), so a claim costs one LDS atomic.
    uint32_t size = nb <= 0 ? 8u
                    : (uint32_t)__builtin_amdgcn_readfirstlane(
                          (int)rlen[from_back ? cs - 1 : ntiny + min(15, nb - 1)]) <= kMixedShortLen
                        ? 16u : 8u;
    for (;;) {
      uint32_t old = 0;
      if (lane == 0) old = atomicAdd((uint32_t*)claim, from_back ? (size << 16) : size);
      old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
      const int f = (int)(old & 0xFFFFu), bk = (int)(old >> 16);
      if (f + bk >= nb) break;
      // the claim [s, e) (window indices, from ntiny): 16 packets run as one
      // G = 4 set if the longest (sorted last) is short, else as G = 8 sets of 8
      int s, e;
      if (from_back) {
        e = cs - bk;
        s = max(e - (int)size, ntiny + f);
      } else {
        s = ntiny + f;
        e = min(ntiny + f + (int)size, cs - bk);
      }
      if (size == 16u) {
        const uint32_t longest = (uint32_t)__builtin_amdgcn_readfirstlane((int)rlen[e - 1]);
        if (longest <= kMixedShortLen) {
          mixed_set<2, VERIFY, MixedKeysS>(a, s, e, w0, lane, ob);
          continue;
        }
        if (!from_back) size = 8u;  // the front has reached long frames
        if (e - s > 8) {
          mixed_set<3, VERIFY, MixedKeysL>(a, s, e - 8, w0, lane, ob);
          s = e - 8;
        }
        mixed_set<3, VERIFY, MixedKeysL>(a, s, e, w0, lane, ob);
      } else {
        const uint32_t shortest = from_back ? rlen[s] : 0xFFFFu;  // (used after the set)
        mixed_set<3, VERIFY, MixedKeysL>(a, s, e, w0, lane, ob);
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int)shortest) <= kMixedShortLen) size = 16u;
      }
    }
    __syncthreads();
    if constexpr (VERIFY) {  // the window's verdicts, one contiguous run
      for (int i = tid; i < cnt; i += kIcrcThreads) a.ok_out[w0 + i] = (uint8_t)lds_rd8(LD::kOk + i);
    }
  }
}

// The AUTO hint of the ragged launches (icrc_capi.cpp hint_word): the
// launch's first workgroup looks at the batch's first kHintGroups 64-packet
// groups, one per wave (`probe`: the thread's packet length, packet tid of the
// batch, clamped to its last), and stores into the context's host-mapped word
// whether at least half of them hold only frames of at most kCompactMaxLen
// bytes -- the compact kernel's candidates.  Both ragged kernels probe the
// same groups, so the hint depends on the batch, not on which variant ran
// last.  One store over PCIe per launch (a store per wave made the kernel
// 2.9x slower, round 4); `scratch`: one LDS word per wave, free at this point.
constexpr int kHintGroups = 12;
template <int WAVES>
__device__ __forceinline__ void store_tiny_hint(uint32_t* hint, uint32_t scratch, int tid, uint32_t probe) {
  static_assert(WAVES >= kHintGroups, "one probing wave per group");
  if ((tid & 63) == 0) lds_wr(scratch + 4u * (uint32_t)(tid >> 6), __all(probe <= kCompactMaxLen) ? 1u : 0u);
  __syncthreads();
  if (tid == 0) {
    uint32_t tiny = 0;
#pragma unroll
    for (int w = 0; w < kHintGroups; ++w) tiny += lds_rd(scratch + 4u * (uint32_t)w);
    __hip_atomic_store(hint, 2u * tiny >= (uint32_t)kHintGroups ? 1u : 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The SORTED variant: the window loop above (the compact variant is
// icrc_compact_kernel below).
template <bool VERIFY>
__global__ void __launch_bounds__(kIcrcThreads, 1) icrc_ragged_mixed_kernel(IcrcArgs a) {
  const int tid = threadIdx.x;
  const uint32_t probe = blockIdx.x == 0 && a.n > 0 ? a.lens[min((uint32_t)tid, a.n - 1u)] : 0xFFFFFFFFu;
  announce_batch(a.busy);
  // (uniform) the hint; scratch: the window's sort arrays, not yet in use
  if (a.tiny_hint && blockIdx.x == 0) store_tiny_hint<kIcrcWaves>(a.tiny_hint, MixedLds::kPerm, tid, probe);
  TablesStaged<3, kIcrcThreads, MixedKeysL> tl;
  MixedKeysS::Staged<kIcrcThreads> ts;
  mixed_windows<VERIFY>(
      a, tid,
      [&]() __attribute__((always_inline)) {
        tl.load(a.tables, tid);
        ts.load(a.tables + 2 * 1024, tid);
      },
      [&]() __attribute__((always_inline)) {
        tl.store(tid);
        ts.store(tid);
      });
}

// ---------------------------------------------------------------------------
// The ragged COMPACT variant as a kernel of its own (round 5): packed runs of
// small frames -- the responder's ACK / NAK / atomic-ack stream
// (src/roce_rq.py:767-853) -- streamed group by group, with no windows, no
// window barriers and no sort.
//
// A wave takes 64-packet groups of its workgroup's contiguous range
// (round-robin over the workgroup's waves: one group per turn, or with the
// output ring below kCompactTurn consecutive groups per turn).  Per group: the lanes' 12-byte
// descriptors, then the compact test of phase 0 (every live frame 44-128 B,
// dword-aligned, in order without overlap, inside 4 KiB from the first
// frame's 16-byte line); a compact group's span arrives with four coalesced
// 16-byte loads per lane, goes to the wave's LDS slot, and each lane patches
// and folds its frame there (two Mul(64) chains and a Mul(-32) step,
// kCompactChains).  The pipeline per wave, two register sets
// ping-ponging: while group i folds, the spans of groups i+1 and i+2 and the
// descriptors of group i+3 are in flight -- eight KiB per wave, against the
// round-4 phase 0's one span per wave and a descriptor round trip plus three
// barriers per 8192-packet window.  A group that fails the test (frames out
// of order, overlapping, larger, unaligned) is listed in LDS and folded after
// the pipeline has drained, by G = 8 lane groups, eight packets at a time
// (compact_fallback_group): the pipeline's registers and the fallback's do
// not overlap.  A workgroup's range goes in chunks of kCompactChunk groups
// (the list's capacity).
// Twelve waves (A/B, round 5: 16 waves, or three span buffers per wave, ran
// 2-4 % slower; at 16 waves the pipeline and the fallback's registers spill).
// Output words of compute launches (icrc_out, no verify): each wave holds 16
// rounds of words in registers and writes them back to back, and takes its
// groups 8 consecutive ones per turn, so a flush covers two contiguous 2-KiB
// runs.  The 4-byte words written into the saturating read stream cost far
// more than their bytes: the ACK kernel without its stores ran 0.1545-0.1573
// ms against 0.1817-0.1836 (words to an L2-resident window: the same 0.155,
// so the cost is HBM writes, not the store instructions; round 6,
// profiles/r06/ab_r06b.txt, ab_r06c.txt).  2^24 ACK frames, 3 A/B rounds
// (ab_r06c, ab_r06d): one store per group (nt) 0.1817-0.1836 ms; ring 16
// 0.1741-0.1749; ring 16 + 16-group turns 0.1679-0.1685, with sc1 stores
// 0.1665-0.1682, nt sc1 0.1667-0.1673, default policy 0.1743-0.1749; ring 16
// + 8-group turns + sc1 0.1659-0.1671 (kept); ring 8 + 8-group turns + sc1
// 0.1706-0.1721; ring 32 + 32-group turns 0.1797-0.1839 (168 VGPRs); 16-group
// turns without the ring 0.1904-0.1910 (hence one-group turns when there is
// no ring: verify launches and compute launches without icrc_out).
constexpr int kCompactRing = 16;    // rounds held (a power of two)
constexpr int kCompactTurn = 8;     // consecutive groups per wave per turn (with the ring)
constexpr int kCompactRingPol = 16;  // sc1
typedef uint32_t compact_ring_t __attribute__((ext_vector_type(kCompactRing)));
constexpr int kCompactWaves = 12;
// Chains per frame: two over Mul(64) (the small-frame kernel's set), one
// Mul(-32) combine step: ACK kernel 0.1930 -> 0.1865 ms over 4 A/B rounds
// against four over Mul(128) and three steps (52 vs 60 lookups per 48-B
// frame, profiles/r05/ab_r05h.txt).
constexpr int kCompactChains = 2;
constexpr int kCompactFoldSet = kCompactChains == 4 ? 0 : kMul64Set;
constexpr int kCompactThreads = 64 * kCompactWaves;
constexpr uint32_t kCompactSlots = kMixedLut + 256u;  // a kCompactSpan slot per wave
constexpr uint32_t kCompactChunk = 1024;               // groups per chunk: the deferred list's capacity
constexpr uint32_t kCompactDefer = kCompactSlots + kCompactWaves * kCompactSpan;  // u32 x kCompactChunk
constexpr uint32_t kCompactDeferN = kCompactDefer + 4u * kCompactChunk;           // two u32 counters
constexpr size_t kCompactLdsBytes = kCompactDeferN + 8u;
static_assert(kCompactLdsBytes <= 163840u, "compact kernel LDS");

// One group of a wave after its test.  Per lane: descriptor, offset in the
// span; uniform: the span's start (from the 16-byte line below frames) and
// length, 0 when the group is not compact.
struct CGroup {
  uint32_t L;
  uint64_t off;
  uint32_t rel;
  uint64_t b16;
  uint32_t span;
};

__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

// The test of group g (packets 64 g ..), from the lane's descriptor.
__device__ __forceinline__ CGroup compact_test(const IcrcArgs& a, uint32_t g, uint32_t L, uint64_t off,
                                               int lane) {
  CGroup c;
  c.L = L;
  c.off = off;
  c.rel = 0;
  c.b16 = 0;
  c.span = 0;
  const uint32_t p0 = g * 64u;
  if (p0 >= a.n) return c;  // (uniform) past the batch
  const int nlive = (int)min(64u, a.n - p0);
  const bool live = lane < nlive;
  const uint64_t addr = a.frames_lo4 + off;  // (from the line below frames)
  const uint64_t b16 = readfirstlane64(addr) & ~15ull;
  const uint64_t rel64 = addr - b16;
  const uint32_t rel = rel64 < kCompactSpan ? (uint32_t)rel64 : 0xFFFF0000u;
  const uint32_t end = rel + L;
  // the left neighbour's end: one DPP wave shift (lane 0 gets 0)
  const uint32_t prev_end = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)end, 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
  const bool ok = !live || (L >= 44 && L <= kCompactMaxLen && (L & 3u) == 0 && (rel & 3u) == 0 &&
                            end <= kCompactSpan && rel >= prev_end);
  if (__all(ok)) {
    c.rel = rel;
    c.b16 = b16;
    // in order without overlap: the last live frame ends the span
    c.span = (uint32_t)__builtin_amdgcn_readlane((int)end, nlive - 1);
  }
  return c;
}

// A group that is not compact: eight sets of eight packets, G = 8 lanes per
// packet (the window kernel's long-frame path, unsorted), Mul(1024) from the
// table rows' low halves.  L, off: the lane's descriptor (packet 64 g + lane).
template <bool VERIFY>
__device__ __forceinline__ void compact_fallback_group(const IcrcArgs& a, uint32_t g, uint32_t L, uint64_t off) {
  const uint8_t* frames = a.frames;
  const uint32_t n = a.n;
  const int lane = __lane_id();
  const int gl = lane & 7, grp = lane >> 3;
  const MixedKeysL kk = MixedKeysL::make(lane);
#pragma unroll 1
  for (int k = 0; k < 8; ++k) {
    const int src = 8 * k + grp;
    const uint32_t pkt = g * 64u + (uint32_t)src;
    const bool live = pkt < n;
    const uint32_t Ls = (uint32_t)__shfl((int)L, src, 64);
    const uint64_t os = (uint64_t)(uint32_t)__shfl((int)(uint32_t)off, src, 64) |
                        ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), src, 64) << 32);
    const Pkt p = describe<32>(frames, pkt, live, live ? os : 0, live ? Ls : 0);
    Batch<kUnroll> b = issue_packet<3, VERIFY>(p, gl);
    finish_packet<3, VERIFY, MixedKeysL, kMixedLut>(a, p, b, gl, grp * 8, kk, OutBuf{0, 0});
  }
}

template <bool VERIFY, int OUTS>  // OUTS: 1 = icrc_out, 2 = status_out present
__global__ void __launch_bounds__(kCompactThreads, 1) icrc_compact_kernel(IcrcArgs a) {
  constexpr bool RING = (OUTS & 1) != 0 && !VERIFY;  // icrc_out words through the register ring
  const int tid = threadIdx.x;
  announce_batch(a.busy);
  // Mul(1024) in the rows' low halves with the combine sets and fix-up LUT
  // (fallback groups, as the window kernel), the compact fold's Mul(64) in
  // the high halves
  const uint32_t probe = blockIdx.x == 0 ? a.lens[min((uint32_t)tid, a.n - 1u)] : 0xFFFFFFFFu;
  {  // both table sets' words first: one round trip
    TablesStaged<3, kCompactThreads, MixedKeysL> tl;
    MixedKeysS::Staged<kCompactThreads> ts;
    tl.load(a.tables, tid);
    ts.load(a.tables + kCompactFoldSet * 1024, tid);
    tl.store(tid);
    ts.store(tid);
  }
  // (uniform) the AUTO hint; scratch: the staging slots, not yet in use
  if (a.tiny_hint && blockIdx.x == 0) store_tiny_hint<kCompactWaves>(a.tiny_hint, kCompactSlots, tid, probe);
  lds_u32* const ndef = (lds_u32*)(uintptr_t)kCompactDeferN;  // deferred groups of chunk k: ndef[k & 1]
  lds_u32* const defer = (lds_u32*)(uintptr_t)kCompactDefer;
  if (tid < 2) ndef[tid] = 0;
  __syncthreads();
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const MixedKeysS kk = MixedKeysS::make(lane);
  constexpr uint32_t kComb = MixedKeysS::kComb;  // Mul(-32)
  const uint32_t slot = kCompactSlots + (uint32_t)wave * kCompactSpan;
  const uint32_t ngroups = (a.n + 63u) / 64u;
  const uint32_t per_block = (ngroups + gridDim.x - 1) / gridDim.x;
  const uint32_t g0 = blockIdx.x * per_block;
  const uint32_t g1 = min(ngroups, g0 + per_block);
  uint32_t chunk = 0;
  for (uint32_t c0 = g0; c0 < g1; c0 += kCompactChunk, ++chunk) {
    const uint32_t c1 = min(g1, c0 + kCompactChunk);
    lds_u32* const nd = ndef + (chunk & 1u);
    // this wave's groups of the chunk: turns of kCompactWaves * K groups, the
    // wave's K consecutive ones in each, i < cnt
    constexpr uint32_t K = RING ? (uint32_t)kCompactTurn : 1u, TURN = kCompactWaves * K;
    const uint32_t ng = c1 - c0, nturn = ng / TURN, rem = ng - nturn * TURN;
    const uint32_t mine = rem > (uint32_t)wave * K ? min(K, rem - (uint32_t)wave * K) : 0u;
    const int cnt = (int)(nturn * K + mine);
    auto group = [&](int i) {
      return c0 + (uint32_t)i / K * TURN + (uint32_t)wave * K + (uint32_t)i % K;
    };
    if (cnt > 0) {  // (uniform)
      compact_ring_t wr = {};
      uint32_t held = 0;  // (uniform) ring slots holding a compact group's words
      // the ring's rounds [base, base + count) to icrc_out, back to back
      auto flush = [&](int base, int count) __attribute__((always_inline)) {
        if constexpr (RING) {
#pragma unroll
          for (int r = 0; r < kCompactRing; ++r) {
            if (r < count && ((held >> r) & 1u)) {  // (uniform)
              const uint32_t pk = group(base + r) * 64u + (uint32_t)lane;
              if (pk < a.n) stg32<kCompactRingPol>(a.icrc_out + pk, wr[r]);
            }
          }
          held = 0;
        }
      };
      // descriptors of the wave's group i (clamped: unconditional loads)
      auto load_desc = [&](int i, uint32_t& L, uint64_t& off) __attribute__((always_inline)) {
        const uint32_t gi = group(min(i, cnt - 1));
        const uint32_t p = min(gi * 64u + (uint32_t)lane, a.n - 1u);
        L = a.lens[p];
        off = a.offsets[p];
      };
      // a compact group's span chunks (unconditional, clamped); a group that is
      // not compact loads 16 bytes of the table image (always mapped, L2-hot)
      auto issue = [&](const CGroup& c, u32x4 (&X)[kCompactLoads]) __attribute__((always_inline)) {
        const bool cp = c.span != 0;
        const uint8_t* base = cp ? a.frames + (c.b16 - a.frames_lo4) : (const uint8_t*)a.tables;
        const uint32_t last = cp ? (c.span + 15u) / 16u - 1u : 0u;
#pragma unroll
        for (int t = 0; t < kCompactLoads; ++t) X[t] = ldg128(base + 16u * min((uint32_t)(lane + 64 * t), last));
      };
      // group i: patch, fold and emit from the slot (compact), or list it for
      // the fallback after the chunk's pipeline
      auto run = [&](int i, const CGroup& c) __attribute__((always_inline)) {
        const uint32_t gi = group(i);
        if (c.span == 0) {  // (uniform)
          if (lane == 0) defer[atomicAdd((uint32_t*)nd, 1u)] = gi;
          return;
        }
        // (an opaque lane id: the compiler otherwise hoists the output addresses
        // of both unrolled groups)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t pkt = gi * 64u + (uint32_t)ln;
        const bool live = pkt < a.n;
        const uint32_t L = c.L;  // (dead lanes repeat the last live frame)
        const uint32_t pb = slot + c.rel;
        const int n = (int)((L - 4u) >> 2);  // (10 .. 31: the test checked every lane)
        // frames of 48 or 64 B on 16-byte slot boundaries, one length (packed
        // ACK runs): read as 16-byte quads (conflict-free at a 48-B stride,
        // where dword reads are 4-way)
        u32x4 q[4];
        uint32_t d0, d2, trailer;
        const uint32_t L0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)L);
        const bool quads = __all((pb & 15u) == 0 && L == L0 && (L0 == 48u || L0 == 64u));
        if (quads) {  // (uniform)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < 3 || L0 == 64u) q[t] = *(const lds_u32x4*)(uintptr_t)(pb + 16u * (uint32_t)t);
          d0 = q[0].x;
          d2 = q[0].z;
          trailer = VERIFY ? (L0 == 64u ? q[3].w : q[2].w) : 0u;
        } else {
          d0 = lds_rd(pb);
          d2 = lds_rd(pb + 8);
          trailer = VERIFY ? lds_rd(pb + 4u * (uint32_t)n) : 0u;
        }
        uint32_t st = 0;
        const int ihl = (int)(d0 & 0xFu);
        if (((d0 >> 4) & 0xFu) != 4u || ihl < 5)
          st |= kPktNotIpv4;
        else if (((d2 >> 8) & 0xFFu) != 17u)
          st |= kPktNotUdp;
        else if (L < (uint32_t)(4 * ihl + 24))
          st |= kPktBadLen;
        if ((((d0 >> 8) & 0xFF00u) | (d0 >> 24)) != L) st |= kPktLenMismatch;
        const bool good = (st & kPktFatal) == 0;
        uint32_t R;
        constexpr int CH = kCompactChains;
        // the chains' fold from the slot with the lane's zero pad in front
        // (absorbing zeros into a zero register keeps it zero, so shorter
        // frames just start later); PAD < 0: per-lane pads, frames patched in
        // place; else every frame of the group has the same length, its masks
        // and seed applied in registers (dwords 0 and 2 are d0 and d2)
        auto fold = [&](auto padc, int ns, uint32_t pz, int pad, auto qc) __attribute__((always_inline)) {
          constexpr int PAD = decltype(padc)::value;
          constexpr bool Q = decltype(qc)::value;  // dwords from q[] (one length, PAD 1)
          uint32_t P[CH], T[CH];
#pragma unroll
          for (int cc = 0; cc < CH; ++cc) P[cc] = T[cc] = 0;
#pragma unroll
          for (int j = 0; j < (int)(kCompactMaxLen / 4u) / CH; ++j) {
            if (j < ns) {  // uniform
#pragma unroll
              for (int cc = 0; cc < CH; ++cc) {
                const int kp = CH * j + cc;
                uint32_t w;
                if constexpr (PAD < 0) {
                  w = lds_rd(pz + 4u * (uint32_t)kp);
                  w = kp >= pad ? w : 0u;
                } else {
                  const int k = kp - PAD;  // (a constant after unrolling)
                  // a zero absorbed into a zero register leaves it zero
                  if (k < 0) continue;
                  if (k == 0)
                    w = (d0 | 0x0000FF00u) ^ kSeedRegister;
                  else if (k == 2)
                    w = d2 | 0xFFFF00FFu;
                  else if constexpr (Q)
                    w = q[(k >> 2) & 3][k & 3];
                  else
                    w = lds_rd(pz + 4u * (uint32_t)kp);
                  if (k == 6) w |= 0xFFFF0000u;
                  if (k == 8) w |= 0x000000FFu;
                }
                kk.absorb(P[cc], T[cc], w);
              }
            }
          }
          uint32_t r = P[CH - 1] ^ T[CH - 1];
#pragma unroll
          for (int cc = CH - 2; cc >= 0; --cc) r = mul_comb(r, kComb) ^ P[cc] ^ T[cc];
          return r;
        };
        const int n0 = __builtin_amdgcn_readfirstlane(n);
        if (__all(good && ihl == 5 && n == n0)) {  // (uniform) one length
          const int ns = (n0 + CH - 1) / CH, pad = CH * ns - n0;
          static_assert(CH == 2, "one instantiation per pad");
          if (quads)  // (48 or 64 B: pad 1)
            R = fold(std::integral_constant<int, 1>{}, ns, pb - 4u, 1, std::true_type{});
          else if (pad == 0)
            R = fold(std::integral_constant<int, 0>{}, ns, pb, 0, std::false_type{});
          else
            R = fold(std::integral_constant<int, 1>{}, ns, pb - 4u, 1, std::false_type{});
        } else if (__all(good && ihl == 5)) {
          // masks and seed patched in place (every lane reads its dwords before
          // any writes them: a dead lane's copy of the last frame writes the same
          // values)
          lds_wr(pb, (d0 | 0x0000FF00u) ^ kSeedRegister);
          lds_wr(pb + 8, d2 | 0xFFFF00FFu);
          lds_wr(pb + 24, lds_rd(pb + 24) | 0xFFFF0000u);
          lds_wr(pb + 32, lds_rd(pb + 32) | 0x000000FFu);
          __asm__ __volatile__("" ::: "memory");
          int nsm = (n + CH - 1) / CH;
          const int ns0 = __builtin_amdgcn_readfirstlane(nsm);
          if (!__all(nsm == ns0)) {  // (uniform) frames of several lengths: the longest
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) nsm = max(nsm, __shfl_xor(nsm, d, 64));
          }
          const int ns = __builtin_amdgcn_readfirstlane(nsm);
          const int pad = CH * ns - n;
          R = fold(std::integral_constant<int, -1>{}, ns, pb - 4u * (uint32_t)pad, pad, std::false_type{});
        } else {
          R = fold_masked4<false, MixedKeysS, kComb, kCompactChains>(nullptr, pb, ihl, n);
        }
        const uint32_t icrc = good ? ~R : 0u;
        if (live) {
          if constexpr (VERIFY) {
            const bool ok = good && trailer == icrc;
            if (good && !ok) st |= kPktIcrcMismatch;
            stg8<kCompactStorePol>(a.ok_out + pkt, ok ? 1u : 0u);
          }
          if constexpr ((OUTS & 1) != 0 && !RING) stg32<kCompactStorePol>(a.icrc_out + pkt, icrc);
          if constexpr ((OUTS & 2) != 0) stg8<kCompactStorePol>(a.status_out + pkt, st);
        }
        if constexpr (RING) {
          wr[i & (kCompactRing - 1)] = icrc;
          held |= 1u << (i & (kCompactRing - 1));
        }
        __asm__ __volatile__("" ::: "memory");
      };
      // write a group's span registers into the slot (the slot's previous group
      // is folded: LDS ops of a wave run in issue order)
      auto stage = [&](const CGroup& c, const u32x4 (&X)[kCompactLoads]) __attribute__((always_inline)) {
        // (unclamped: the slot holds all 256 chunks; the chunks past the span
        // repeat its last one and are never read)
#pragma unroll
        for (int t = 0; t < kCompactLoads; ++t) *(lds_u32x4*)(uintptr_t)(slot + 16u * (uint32_t)(lane + 64 * t)) = X[t];
        __asm__ __volatile__("" ::: "memory");
      };

      // Issue order, so that no wait retires a younger span: step i stages group
      // i (its span issued two steps before), issues group i + 3's descriptors,
      // tests group i + 2 (descriptors issued one step before, ahead of group
      // i + 1's span), issues its span and folds group i.  Descriptors of the
      // groups two and three ahead ping-pong between (La, oa) and (Lb, ob).
      uint32_t L0, L1, La, Lb;
      uint64_t o0, o1, oa, ob;
      load_desc(0, L0, o0);
      load_desc(1, L1, o1);
      load_desc(2, La, oa);
      u32x4 XA[kCompactLoads], XB[kCompactLoads];
      CGroup ca = compact_test(a, group(0), L0, o0, lane);
      issue(ca, XA);
      CGroup cb = compact_test(a, group(min(1, cnt - 1)), L1, o1, lane);
      if (cnt < 2) cb.span = 0;
      issue(cb, XB);
      // group i in (c, X); the next group's descriptors into (Ln, on); group
      // i + 2's in (Lt, ot)
      auto step = [&](int i, CGroup& c, u32x4 (&X)[kCompactLoads], uint32_t& Lt, uint64_t& ot, uint32_t& Ln,
                      uint64_t& on) __attribute__((always_inline)) {
        const CGroup cur = c;
        body_prio_hi();
        if (cur.span != 0) stage(cur, X);  // (uniform)
        load_desc(i + 3, Ln, on);
        c = compact_test(a, group(min(i + 2, cnt - 1)), Lt, ot, lane);
        if (i + 2 >= cnt) c.span = 0;
        issue(c, X);
        body_prio_lo();
        run(i, cur);
        if (RING && (i & (kCompactRing - 1)) == kCompactRing - 1) flush(i - (kCompactRing - 1), kCompactRing);
      };
      int i = 0;
      for (; i + 1 < cnt; i += 2) {
        step(i, ca, XA, La, oa, Lb, ob);
        step(i + 1, cb, XB, Lb, ob, La, oa);
      }
      if (i < cnt) step(i, ca, XA, La, oa, Lb, ob);
      if (RING && (cnt & (kCompactRing - 1)) != 0) flush(cnt & ~(kCompactRing - 1), cnt & (kCompactRing - 1));
    }  // (cnt > 0)
    // the chunk's listed groups, by every wave of the workgroup; the other
    // counter is free until the next chunk
    __syncthreads();
    const uint32_t ndc = (uint32_t)__builtin_amdgcn_readfirstlane((int)*nd);
    if (tid == 0) ndef[(chunk + 1u) & 1u] = 0;
    for (uint32_t k = (uint32_t)wave; k < ndc; k += kCompactWaves) {
      const uint32_t gi = (uint32_t)__builtin_amdgcn_readfirstlane((int)defer[k]);
      const uint32_t p = min(gi * 64u + (uint32_t)lane, a.n - 1u);
      compact_fallback_group<VERIFY>(a, gi, a.lens[p], a.offsets[p]);
    }
    __syncthreads();  // (the list is refilled by the next chunk)
  }  // chunks
}

// ---------------------------------------------------------------------------
// Small frames (strided, stride <= kSmallMaxStride): one LANE per packet.
//
// With a group of lanes per packet, a 108-byte frame gives each lane a dozen
// dwords against a fixed per-packet cost (describe, head fix-ups, rotation,
// combine) of several hundred instructions.  Here a wave takes a batch of 64
// consecutive packets: their 64 x stride bytes arrive with fully coalesced
// 16-byte loads (issued two batches ahead, held in registers), go to the
// wave's LDS staging slot, each lane patches its frame's masked dwords and
// seed in place, and folds the frame as two interleaved chains: chain c takes
// the dwords k = 2 j + c - pad (pad = 2 ns - n zero dwords in front, ns =
// ceil(n / 2) steps), (P, T) <- Mul(64)(P ^ T ^ w_k), and the packet register
// is R = Mul(-32)(chain 1) ^ chain 0 -- one Horner step.  The joins do not
// depend on the frame length.  The batch holding the last packet reads its
// frames straight from global memory (no 16-byte over-read past the buffer).
//
// Nothing between a batch's loads and their use may be predicated or fenced:
// the compiler would then drain every load in flight (vmcnt(0)), including
// the prefetch.  Hence unconditional LDS writes into the slot and the masks
// applied in LDS rather than by uniform selects in the loop.
//
// LDS: [0, 64 KiB) Mul(64) in the Keys8 layout (icrc_device.hpp: 8
// conflict-free copies in the low half of 256 rows of 256 B, one v_perm_b32
// per address), then one staging slot of 64 x stride bytes per wave, the
// output ring's tail, and Mul(-32) in the last 4 KiB.  The output ring
// starts in the free high halves of the table rows (32 KiB) and continues
// after the staging slots.
// 12 waves (cfg5, 108-B frames: 8 waves 4975, 11 4899, 12 5034, 13 4773
// GiB/s, 3 A/B rounds; an odd count leaves one SIMD a wave short, so the
// launch rounds it down to even).  With Keys16 tables (64 KiB) and the ring
// after the slots, 8 waves were best (6-10 waves: -10 % to -2.5 %); Keys8
// (32 KiB of tables, the ring's head in the free row halves) gained +1.8 %
// at 8 waves.
constexpr int kSmallMaxWaves = 12;
// Tail stealing (below): cfg5 kernel ms, 6 A/B rounds over two sessions
// (profiles/r03q_small_tail_ab*.txt): static 0.3132-0.3161, 1/4 0.3139-0.3175,
// 1/8 0.3115-0.3122, 1/16 0.3106-0.3148 (+0.9 % mean), 1/32 0.3122-0.3135.
constexpr uint32_t kSmallTailDiv = 16;
// Staging: LDS-DMA (global_load_lds_dwordx4) into the wave's slot one batch
// ahead.  cfg5 kernel ms, 5 A/B rounds over two sessions (profiles/r04a, r04c
// cfg5_ab): 16-byte loads into registers two batches ahead, written into the
// slot with ds_write_b128, 0.3102-0.3129; LDS-DMA 0.3058-0.3098 (-1.2 %).
constexpr uint32_t kSmallAhead = 1;  // batches a wave's loads run ahead of its fold
using SmallKeys = Keys8;
// Mul(-32) for the combine, unreplicated in the last 4 KiB.  (8 conflict-free
// copies in the high halves of the table rows, the output ring then entirely
// after the staging slots: -5 %, -2 % at 10 waves.)
constexpr uint32_t kSmallComb = 163840u - 4096u;
constexpr uint32_t kSmallEnd = kSmallComb;  // end of the staging + ring tail
constexpr uint32_t kSmallStage = 65536;
constexpr uint32_t kSmallHoleWords = 256u * (256u - Keys8::kHole) / 4u;  // ring words in the row halves
// LDS byte address of ring word k / ring quad i (16 B): the row halves first,
// then the tail after the staging slots
__device__ __forceinline__ uint32_t small_ring_word(uint32_t tail, uint32_t k) {
  return k < kSmallHoleWords ? (k >> 5) * 256u + Keys8::kHole + (k & 31u) * 4u
                             : tail + 4u * (k - kSmallHoleWords);
}
__device__ __forceinline__ uint32_t small_ring_quad(uint32_t tail, uint32_t i) {
  return i < kSmallHoleWords / 4u ? (i >> 3) * 256u + Keys8::kHole + (i & 7u) * 16u
                                  : tail + 16u * (i - kSmallHoleWords / 4u);
}
// Chains of the fold: two over Mul(64).  Against four over Mul(128) they need
// one Mul(-32) combine step instead of three and read one pad dword at most:
// 108 lookups per 108-B frame instead of 124.  cfg5 kernel ms, 6 A/B rounds
// over two sessions (profiles/r04p, r04q): four chains 0.3050-0.3089, two
// 0.2980-0.3006 (-2.5 %), one (Mul(32), no combine, a dependent chain of 26
// lookups) 0.3257-0.3288.
constexpr int kSmallChains = 2;
constexpr int kSmallMaxSteps = (kSmallMaxStride / 4 + kSmallChains - 1) / kSmallChains;
constexpr int kSmallOutRounds = 64;  // output ring depth in rounds (0 = off)
// Cache policy of the ring's flushes (out_store128).  The words written into
// the saturating read stream cost several times their own transfer time;
// scope-sc1 stores cut that: cfg5 4625 -> 4865 GiB/s (3 A/B rounds; nt the
// same, 4870).  Microbenchmark (scratch/rw_mix.hip, read pattern without the
// CRC): read only 0.266 ms, + words flushed every 16 rounds plain 0.325, nt
// 0.314, sc1 0.307; every 30 rounds with sc1 0.293 (larger bursts are
// cheaper, but the ring cannot grow beside 8 staging slots); a 9th "writer"
// wave draining the ring, with or without bursts aligned to a global clock,
// 0.320-0.344.
constexpr int kSmallOutPol = 16;
// Ring rounds held in registers before the LDS ring: each lane keeps its word
// of the first kSmallRegRounds rounds of a ring window in a vector register
// (uniform dynamic index), so a flush writes kSmallRegRounds + the LDS ring's
// rounds at once (larger write bursts into the read stream).  cfg5 kernel ms
// over 4 A/B rounds (profiles/r05/ab_r05k.txt, ab_r05l.txt, ab_r05m.txt):
// 16 rounds -2.3 % against none (8 -1.9 %; 32 slower: spills); with the
// batch's exact chunk count and unmasked DMA / slot reads (below; 88 -> 25
// SGPRs spilled into VGPR lanes, 12 fewer VGPRs) 24 rounds and then 28 fit:
// 0.2962 -> 0.2917 ms (28), 0.2900 with the early first DMA.
constexpr int kSmallRegRounds = 28;
typedef uint32_t small_regring_t __attribute__((ext_vector_type(kSmallRegRounds > 0 ? kSmallRegRounds : 1)));

template <int C, bool VERIFY, int OUTS>  // OUTS: 1 = icrc_out, 2 = status_out present
__global__ void __launch_bounds__(64 * kSmallMaxWaves, 1) icrc_small_kernel(IcrcArgs a) {
  const int tid = threadIdx.x;
  const uint32_t S = (uint32_t)a.stride, L = a.len;
  announce_batch(a.busy);
  const bool dead = L < 44 || (L & 3u) || L > 65535u || L > S;
  constexpr int CH = kSmallChains;
  const int n = dead ? 0 : (int)((L - 4) >> 2);  // covered dwords (uniform, <= 31)
  const int ns = (n + CH - 1) / CH, pad = CH * ns - n;  // steps, zero dwords in front (0 or 1)
  const int lane = tid & 63, wave = tid >> 6;
  const SmallKeys kk = SmallKeys::make(lane);
  const uint32_t nchunk = 4 * S;  // 16-byte chunks per batch (<= 64 C)
  const uint32_t nw = blockDim.x >> 6;
  const uint32_t stage = kSmallStage + (uint32_t)wave * 64u * S;
  const uint32_t nb = (a.n + 63) / 64;
  const uint32_t last = nb - 1;  // the batch holding packet n-1: direct path
  const uint32_t per_block = (nb + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = blockIdx.x * per_block, b1 = min(nb, b0 + per_block);

  // header checks of one frame (dwords 0 and 2)
  auto check = [&](uint32_t d0, uint32_t d2, int& ihl) {
    uint32_t st = dead ? kPktBadLen : 0u;
    ihl = (int)(d0 & 0xFu);
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
    return st;
  };
  // Output ring (compute mode with icrc_out): the ICRC words of kOutRounds
  // rounds of nw batches (one batch per wave) collect in LDS after the
  // staging slots, and the workgroup writes them out together as one
  // contiguous run of 16-byte stores between two barriers, instead of each
  // wave storing 256 B per batch into the read stream.
  constexpr bool kRing = kSmallOutRounds > 0 && (OUTS & 1) != 0 && !VERIFY;
  const uint32_t ring = kSmallStage + nw * 64u * S;  // the ring's tail (small_ring_word)
  const uint32_t rounds_cap =
      kRing ? min((uint32_t)kSmallOutRounds, (kSmallHoleWords + (kSmallEnd - ring) / 4u) / (nw * 64u)) : 0u;
  uint32_t ring_base = 0;  // first packet of the ring's current window
  // the window's rounds in registers (C = 8: 24, as 28 spill a VGPR there)
  constexpr int RR = kRing ? (C >= 8 ? 24 : kSmallRegRounds) : 0;
  small_regring_t W = {};
  uint32_t in_ring = 0;  // the current round's index in the window
  auto emit = [&](uint32_t pkt, bool live, uint32_t st, uint32_t R, uint32_t trailer,
                  bool to_ring = false) {
    const bool good = (st & kPktFatal) == 0;
    const uint32_t icrc = good ? ~R : 0u;
    if (live) {
      if constexpr (VERIFY) {
        const bool ok = good && trailer == icrc;
        if (good && !ok) st |= kPktIcrcMismatch;
        a.ok_out[pkt] = ok ? 1 : 0;
      }
      if constexpr ((OUTS & 1) != 0) {
        if (kRing && to_ring) {
          if (RR > 0 && in_ring < (uint32_t)RR)  // (uniform)
            W[in_ring] = icrc;
          else
            lds_wr(small_ring_word(ring, pkt - ring_base - (uint32_t)RR * nw * 64u), icrc);
        } else
          a.icrc_out[pkt] = icrc;
      }
      if constexpr ((OUTS & 2) != 0) a.status_out[pkt] = (uint8_t)st;
    }
  };
  // the four chains over dwords [0, n); rd(k, kp) returns dword k >= 0
  // (kp = k + pad, a compile-time index into the padded frame) ready to
  // absorb; dwords k < 0 are the zero pad
  auto fold4 = [&](auto rd) {
    uint32_t P[CH], T[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) P[c] = T[c] = 0;
#pragma unroll
    for (int j = 0; j < kSmallMaxSteps; ++j) {
      if (j < ns) {  // uniform
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const int k = CH * j + c - pad;
          const uint32_t w = rd(k < 0 ? 0 : k, CH * j + c);  // (never read before the frame)
          kk.absorb(P[c], T[c], (j == 0 && k < 0) ? 0u : w);
        }
      }
    }
    uint32_t R = P[CH - 1] ^ T[CH - 1];
#pragma unroll
    for (int c = CH - 2; c >= 0; --c) R = comb4<kSmallComb>(R, kk) ^ P[c] ^ T[c];
    return R;
  };
  // per-dword masks (IPv4 options, the direct path, malformed frames)

  // Batches a wave loads are clamped to the workgroup's own staged range:
  // the prefetch two rounds past its end re-reads the range's last batch
  // (still in L2) instead of the next workgroup's first ones, which that
  // workgroup reads again much later (an extra ~2.3 % of HBM reads at cfg5).
  //
  // Tail stealing (as in the strided kernel): the last 1/kSmallTailDiv of a
  // workgroup's staged batches [split, end) are claimed batch by batch
  // through its counter, by its own waves and by workgroups that are done;
  // their words go straight to icrc_out.  The ring covers [b0, split).
  auto range = [&](uint32_t blk, uint32_t& rb, uint32_t& re, uint32_t& rs) {
    rb = blk * per_block;
    re = min(min(nb, rb + per_block), last);
    const uint32_t len = rb < re ? re - rb : 0u;
    rs = re - (a.claims ? len / kSmallTailDiv : 0u);
  };
  uint32_t rb_, re_, bs_end;
  range(blockIdx.x, rb_, re_, bs_end);
  unsigned long long* claims =
      a.claims ? a.claims + (size_t)(a.epoch % kClaimSlots) * kMaxClaimBlocks : nullptr;
  if (claims && tid == 0) atomicExch(&claims[blockIdx.x], (unsigned long long)a.epoch << 32);
  uint32_t lim = bs_end > 0 ? bs_end - 1u : 0u;  // prefetch clamp (no clamp while claiming)
  auto load_at = [&](const uint8_t* base) __attribute__((always_inline)) {
    // LDS-DMA straight into the wave's slot: chunk lane + 64 t of the batch
    // lands at stage + 1024 t + 16 lane; lanes past the batch's last chunk
    // stay idle (the slot holds exactly the batch)
#pragma unroll
    for (int t = 0; t < C; ++t)
      if (t < C - 1 || (uint32_t)(lane + 64 * t) < nchunk)  // (C: exactly ceil(nchunk / 64))
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(base + 16u * (uint32_t)(lane + 64 * t)),
            (__attribute__((address_space(3))) void*)(uintptr_t)(stage + 1024u * (uint32_t)t), 16, 0, 2);
  };
  auto load = [&](uint32_t b) __attribute__((always_inline)) {  // unconditional: clamped batch index
    load_at(a.frames + (uint64_t)min(b, lim) * 64u * S);
  };
  // The tables arrive by LDS-DMA like the batches: no table word passes
  // through a register, so the compiler has no load of its own to wait for
  // (it counts no LDS-DMA load: a load of its own would make it wait
  // vmcnt(0), draining the first batch's DMA too).  Mul(64): the 256 Keys8
  // rows (128 B each, built on the host, kSmallImageOff) into the low halves
  // of the 256-B LDS rows -- 64 instructions of 1 KiB of LDS, the lanes whose
  // 16 bytes fall in a row's high half idle; Mul(-32) unreplicated at
  // kSmallComb, 4 more.  Instruction j goes to wave j mod nw.  Then the wave's
  // first batch, then vmcnt(C): the C younger batch loads may still be in
  // flight, every table load of the wave has landed; then the barrier.
  {
    const uint8_t* rows = (const uint8_t*)(a.tables + kSmallImageOff);
    const uint8_t* cm32 = (const uint8_t*)(a.tables + kNumMainSets * 1024);  // combine set 0: Mul(-32)
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(wave);
#pragma unroll 1
    for (uint32_t j = wv; j < 68u; j += nw) {  // (uniform)
      if (j < 64u) {
        if ((lane & 8) == 0)  // LDS chunk 64 j + lane: row 4 j + lane / 16, its low half
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(rows + 16u * (32u * j + (uint32_t)((lane >> 4) << 3) +
                                                                            (uint32_t)(lane & 7))),
              (__attribute__((address_space(3))) void*)(uintptr_t)(1024u * j), 16, 0, 0);
      } else {
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(cm32 + 16u * (64u * (j - 64u) + (uint32_t)lane)),
            (__attribute__((address_space(3))) void*)(uintptr_t)(kSmallComb + 1024u * (j - 64u)), 16, 0, 0);
      }
    }
    // (no branch around the DMA: a workgroup without staged batches loads a
    // clamped full batch, or with none in the launch (n <= 64) the table
    // image, and never folds it)
    load_at(last > 0 ? a.frames + (uint64_t)min(b0 + (uint32_t)wave, lim) * 64u * S
                     : (const uint8_t*)a.tables);
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0F70 | C);  // vmcnt(C): the table rows are in LDS
    __asm__ __volatile__("" ::: "memory");
  }
  // (the barrier alone: __syncthreads' fence would wait for the DMA, vmcnt(0))
  __builtin_amdgcn_s_barrier();
  __asm__ __volatile__("" ::: "memory");
  // The last batch, straight from global memory (one wave of the owning
  // block): its per-dword loads and dependent fold run first, under the other
  // waves' streams, not at the end of the launch (cfg5 0.2906-0.2925 ->
  // 0.2880-0.2921 ms, 4 A/B rounds, profiles/r06/ab_r06p.txt).
  {
    if (last >= b0 && last < b1 && (uint32_t)wave == (last - b0) % nw) {
      const uint32_t pkt = last * 64u + (uint32_t)lane;
      const bool live = pkt < a.n;
      const uint8_t* f = a.frames + (uint64_t)(live ? pkt : a.n - 1) * S;
      int ihl;
      const uint32_t st = check(ldg32(f), ldg32(f + 8), ihl);
      const uint32_t R = small_fold_masked_global<SmallKeys, kSmallComb, CH>(f, ihl, n);
      emit(pkt, live, st, R, VERIFY ? ldg32(f + 4 * n) : 0u);
    }
  }
  // One batch: the slot's batch has landed; the wave reads its frames into
  // registers and at once refills the slot with the next batch (in flight
  // during the fold, its loads at raised wave priority), then checks the
  // headers, applies the masks and the seed in registers and folds.  (Round
  // 4 patched the masked dwords in LDS first: two LDS round trips before the
  // next batch's loads could go out.)  live: the batch is the wave's (its
  // words are emitted); to_ring: its words go to the output ring (when there
  // is one).
  auto stage_and_fold = [&](uint32_t b, uint32_t bnext, bool live = true,
                            bool to_ring = true) __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the batch is in the slot
    __asm__ __volatile__("" ::: "memory");
    const uint32_t pb = stage + (uint32_t)lane * S;
    const uint32_t pz = pb - 4u * (uint32_t)pad;  // dword k at pz + 4 (k + pad)
    uint32_t D[CH * kSmallMaxSteps];
#pragma unroll
    for (int kp = 0; kp < CH * kSmallMaxSteps; ++kp)
      D[kp] = kp <= 4 * (C - 1) || kp < CH * ns ? lds_rd(pz + 4u * (uint32_t)kp) : 0u;
    const uint32_t trailer = VERIFY ? lds_rd(pb + 4u * n) : 0u;
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot is read
    __asm__ __volatile__("" ::: "memory");
    body_prio_hi();
    load(bnext);
    body_prio_lo();
    // (pad is 0 or 1 and uniform: dword k is D[k] or D[k + 1])
    const bool p1 = pad != 0;
    const uint32_t d0 = p1 ? D[1] : D[0], d2 = p1 ? D[3] : D[2];
    int ihl;
    uint32_t st = check(d0, d2, ihl);
    uint32_t R;
    if (__all((st & kPktFatal) == 0 && ihl == 5)) {
      // IHL 5 everywhere: the masked dwords 0, 2, 6, 8 and the seed
      if (p1) {
        D[1] = (D[1] | 0x0000FF00u) ^ kSeedRegister;
        D[3] |= 0xFFFF00FFu;
        D[7] |= 0xFFFF0000u;
        D[9] |= 0x000000FFu;
      } else {
        D[0] = (D[0] | 0x0000FF00u) ^ kSeedRegister;
        D[2] |= 0xFFFF00FFu;
        D[6] |= 0xFFFF0000u;
        D[8] |= 0x000000FFu;
      }
      R = fold4([&](int, int kp) { return D[kp]; });
    } else {  // per-dword masks (IPv4 options; malformed frames), from HBM
      // (out of line; the slot already holds the next batch)
      const uint8_t* f = a.frames + (uint64_t)(b * 64u + (uint32_t)lane) * S;
      R = small_fold_masked<true, SmallKeys, kSmallComb, CH>(live ? f : a.frames, 0u, ihl, n);
    }
    emit(b * 64u + (uint32_t)lane, live, st, R, trailer, kRing && to_ring);
    __asm__ __volatile__("" ::: "memory");
  };

  // staged batches [b0 + wave, bs_end) step nw, each batch's loads issued one
  // batch ahead (kSmallAhead), two rounds per loop iteration
  if (kRing && rounds_cap > 0 && b0 < bs_end) {  // (uniform)
    // rounds: round r is batch b0 + r nw + wave of every wave (waves past
    // bs_end recompute a clamped batch and emit nothing); every rounds_cap
    // rounds the ring goes out.  LDS-only waits at the barriers: the
    // prefetched loads stay in flight across them.
    const uint32_t nrounds = (bs_end - b0 + nw - 1) / nw;
    ring_base = b0 * 64u;
    in_ring = 0;
    auto flush = [&]() {
      // rounds [0, RR) from the waves' registers, the rest from the LDS ring
      const uint32_t rb0 = ring_base / 64u, lb0 = rb0 + (uint32_t)RR * nw;
      const uint32_t words =
          in_ring > (uint32_t)RR && bs_end > lb0 ? min((in_ring - (uint32_t)RR) * nw, bs_end - lb0) * 64u : 0u;
      // lgkmcnt(0): this wave's ring words are written.  The compiler-level
      // memory clobbers pin the ring's LDS accesses on their side of the
      // barrier (the barrier intrinsic alone is not a memory operation at IR
      // level); they emit no wait, so the prefetched global loads stay in flight.
      __asm__ __volatile__("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      __asm__ __volatile__("" ::: "memory");
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        const uint32_t b = rb0 + (uint32_t)r * nw + (uint32_t)wave;
        if ((uint32_t)r < in_ring && b < bs_end)  // (uniform)
          stg32<kSmallOutPol>(a.icrc_out + b * 64u + (uint32_t)lane, W[r]);
      }
      const auto dst = out_rsrc(a.icrc_out + (size_t)lb0 * 64u, 4u * words);
      for (uint32_t i = (uint32_t)tid; i < words / 4u; i += blockDim.x)
        out_store128<kSmallOutPol>(*(const lds_u32x4*)(uintptr_t)small_ring_quad(ring, i), dst, 16u * i);
      __asm__ __volatile__("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0xC07F);  // the ring is read before anyone writes it again
      __builtin_amdgcn_s_barrier();
      __asm__ __volatile__("" ::: "memory");
      ring_base += in_ring * nw * 64u;
      in_ring = 0;
    };
    const uint32_t window = rounds_cap + (uint32_t)RR;
    for (uint32_t r = 0; r < nrounds; r += 2) {
      uint32_t b = b0 + r * nw + (uint32_t)wave;
      stage_and_fold(b, b + kSmallAhead * nw, b < bs_end);
      if (++in_ring == window) flush();
      if (r + 1 < nrounds) {
        b += nw;
        stage_and_fold(b, b + kSmallAhead * nw, b < bs_end);
        if (++in_ring == window) flush();
      }
    }
    if (in_ring) flush();
  } else if (b0 < bs_end) {  // (uniform) loads stay inside batches [0, last)
    const uint32_t first = b0 + (uint32_t)wave;
    const int cnt = first < bs_end ? (int)((bs_end - first + nw - 1) / nw) : 0;
    uint32_t b = first;
    int i = 0;
    for (; i + 1 < cnt; i += 2, b += 2 * nw) {
      stage_and_fold(b, b + kSmallAhead * nw);
      stage_and_fold(b + nw, b + nw + kSmallAhead * nw);
    }
    if (i < cnt) stage_and_fold(b, b + kSmallAhead * nw);
  }
  if (claims) {  // own tail, then up to kMaxVictims other workgroups' tails
    lim = 0xFFFFFFFFu;
    uint32_t victim = blockIdx.x, tries = 0;
    auto claim = [&]() -> uint32_t {  // a batch, or ~0u when every tail tried is empty
      for (;;) {
        unsigned long long old = 0;
        if (lane == 0) old = atomicAdd(&claims[victim], 1ull);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)old);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(old >> 32));
        uint32_t vb, ve, vs;
        range(victim, vb, ve, vs);
        if (hi == a.epoch && vs < ve && lo < ve - vs) return vs + lo;
        if (++tries > kMaxVictims) return ~0u;
        victim = (blockIdx.x + 2 * tries - 1) % gridDim.x;
      }
    };
    uint32_t cur = claim();
    if (cur != ~0u) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // (an unused first DMA has landed)
      load(cur);
      for (;;) {  // the next claim's loads go out while this batch folds
        const uint32_t nxt = claim();
        stage_and_fold(cur, nxt == ~0u ? cur : nxt, true, false);
        if (nxt == ~0u) break;
        cur = nxt;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // no DMA outlives its slot's use
}

// STREAM-style read ceiling: one workgroup per CU sweeping a contiguous
// chunk with 16-byte nt loads, 8 per lane, 8 waves (64 KiB in flight per CU).
// Sweep over the cfg2 buffer (scratch/read_ceiling.hip): this shape 7.13 TB/s;
// 16 waves x 8 loads (the round-1 ceiling kernel) 6.70; ping-pong buffers
// 7.10 at 64 KiB in flight, 6.8-7.0 at 128 KiB; plain loads 5.95-6.18.
constexpr int kStreamThreads = 512;
__global__ void __launch_bounds__(kStreamThreads) stream_read_kernel(const u32x4* __restrict__ p,
                                                                     uint64_t n16, uint32_t* sink) {
  constexpr int R = 8;
  constexpr uint64_t T = kStreamThreads;
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per;
  const uint64_t b1 = b0 + per < n16 ? b0 + per : n16;
  u32x4 acc = {0, 0, 0, 0};
  uint64_t i = b0 + threadIdx.x;
  for (; i + (R - 1) * T < b1; i += R * T) {
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = __builtin_nontemporal_load(p + i + r * T);
#pragma unroll
    for (int r = 0; r < R; ++r) acc ^= v[r];
  }
  for (; i < b1; i += T) acc ^= p[i];
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9E3779B9u) sink[0] = x;  // keeps the loads live; practically never stores
}

// ---------------------------------------------------------------------------
// Per-packet service: the low-latency form of ricrc_compute_one (the
// drop-in for BTH.compute_icrc, src/roce.py:192-223, one frame per call).
//
// A launched kernel costs more than the CRC of one frame (launch, copies and
// a stream synchronisation put a plain call at ~25 us, where zlib.crc32 needs
// ~4 us for 4 KiB).  Here ONE wave stays resident and polls a request slot in
// pinned fine-grained host memory (ServiceRing, icrc_internal.hpp): the host
// copies the frame into the slot and publishes a sequence number; the wave
// sees it, reads the frame straight from host memory over PCIe (64 lanes,
// one 16-byte load each per KiB, all in flight at once), folds it with the
// batch kernels' 64-lane group code (Mul(8192) tables in LDS, butterfly
// combine) and writes the ICRC, the status and the sequence number back into
// host memory, where the caller spins on it.
//
// Polling uses relaxed system-scope loads (no cache maintenance per poll);
// one acquire fence per request makes the frame bytes the host wrote before
// publishing visible.  The request (sequence number + length) and the answer
// (ICRC + status + sequence number) are single 8-byte words, so each
// direction is one PCIe transaction with no fence between value and flag.  The wave leaves when the host raises `stop` (context
// destroyed, or about to launch batch work, which needs this CU's LDS) or
// after `idle_ticks` of the 100 MHz real-time counter without a request:
// every path through the loop reaches one of the two, so the grid always
// drains; the host relaunches it on the next call.
// Polls of the request slot in flight at once (2 or 4; A/B switch).
constexpr int kSvcPolls = 2;
constexpr int kSvcThreads = 512;  // all stage the tables; wave 0 serves, waves 1-7 help with bursts
constexpr int kSvcWaves = kSvcThreads / 64;
// LDS of the service (round 3): Mul(8192) for single frames (G = 64) and
// Mul(1024) for bursts (G = 8) as the two halves of the Keys8 rows (64 KiB),
// the combine sets Mul(-32), Mul(-128 2^l), l < 6 (both widths use the
// first ones), the fix-up LUT; then the results of a burst (ICRC words,
// verdicts, status bytes, written through generic pointers) and a 64 KiB
// staging area a burst's frames are copied into with LDS-DMA before they are
// folded from LDS.
using SvcKeysL = Keys8T<0>;  // Mul(8192), G = 64
using SvcKeysS = Keys8T<1>;  // Mul(1024), G = 8
constexpr uint32_t kSvcLut = kFixLut<6, SvcKeysL>;
constexpr uint32_t kSvcOut = kSvcLut + 256u - 16u;  // single frame: ICRC + status (the LUT's spare bytes)
constexpr uint32_t kBurstIcrc = kSvcLut + 256u;
constexpr uint32_t kBurstOk = kBurstIcrc + 4u * kSvcMaxBurst;
constexpr uint32_t kBurstSt = kBurstOk + kSvcMaxBurst;
// burst hand-off to the helper waves: generation, (count | verify << 31),
// finished helpers, exit flag; then the burst's descriptors
constexpr uint32_t kSvcCtl = kBurstSt + kSvcMaxBurst;
constexpr uint32_t kSvcDescLds = kSvcCtl + 16u;
constexpr uint32_t kBurstStage = (kSvcDescLds + 8u * kSvcMaxBurst + 1023u) & ~1023u;
constexpr size_t kSvcLds = kBurstStage + kSvcMaxFrame + 1024u;  // (+ the last chunk's reach)
static_assert(kSvcLds <= 163840, "service LDS");

// One burst's share of wave `wave`: frame i at stage + (desc[i] & 0xFFFFFFFF),
// length desc[i] >> 32 (descriptors in LDS), eight frames per round (G = 8
// groups), rounds wave, wave + kSvcWaves, ... folded from LDS.
template <bool VERIFY>
__device__ __forceinline__ void serve_burst(uint32_t cnt, int lane, int wave) {
  constexpr int LOG2G = 3, G = 8, DPI = 4 * G;
  const uint64_t dl = *(const __attribute__((address_space(3))) uint64_t*)(uintptr_t)(kSvcDescLds + 8u * (uint32_t)lane);
  const uint32_t dlo = (uint32_t)dl, dhi = (uint32_t)(dl >> 32);
  const uint8_t* stage = (const uint8_t*)(__attribute__((address_space(3))) uint8_t*)(uintptr_t)kBurstStage;
  IcrcArgs a{};
  a.frames = stage;
  a.n = cnt;
  a.icrc_out = (uint32_t*)(lds_u32*)(uintptr_t)kBurstIcrc;  // flat stores into LDS
  a.ok_out = (uint8_t*)(lds_u32*)(uintptr_t)kBurstOk;
  a.status_out = (uint8_t*)(lds_u32*)(uintptr_t)kBurstSt;
  const int gl = lane & (G - 1), grp = lane >> LOG2G;
  const SvcKeysS kk = SvcKeysS::make(lane);
  for (uint32_t s0 = (uint32_t)wave * (64 / G); s0 < cnt; s0 += kSvcWaves * (64 / G)) {
    const uint32_t i = s0 + (uint32_t)grp;
    const bool live = i < cnt;
    const uint32_t ii = live ? i : 0u;
    // this group's descriptor (lane ii of the wave holds it)
    const uint32_t off = (uint32_t)__shfl((int)dlo, (int)ii, 64);
    uint32_t L = (uint32_t)__shfl((int)dhi, (int)ii, 64);
    if (off > kSvcMaxFrame || L > kSvcMaxFrame - off) L = 0;  // (a bad descriptor: BAD_LEN)
    const Pkt p = describe<DPI>(stage, i, live, off, live ? L : 0u);
    Batch<kUnroll> b = issue_packet<LOG2G, VERIFY>(p, gl);
    finish_packet<LOG2G, VERIFY, SvcKeysS, kSvcLut>(a, p, b, gl, grp * G, kk);
  }
}

__global__ void __launch_bounds__(kSvcThreads, 1) icrc_service_kernel(ServiceArgs s) {
  constexpr int LOG2G = 6;
  constexpr int DPI = 4 << LOG2G;
  const int tid = threadIdx.x;
  stage_tables<LOG2G, kSvcThreads, SvcKeysL>(s.tables, tid);
  SvcKeysS::template stage<kSvcThreads>(s.tables + 3 * 1024, tid);  // main set 3: Mul(1024)
  if (tid < 4) lds_wr(kSvcCtl + 4u * (uint32_t)tid, 0u);
  __syncthreads();
  typedef __attribute__((address_space(3))) uint32_t lds_w;
  auto ctl = [](uint32_t i) {  // (the helpers' spin reads must not be hoisted)
    return __hip_atomic_load((lds_w*)(uintptr_t)(kSvcCtl + 4u * i), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  if (tid >= 64) {
    // helper wave: each burst generation wave 0 posts, fold this wave's
    // rounds, count itself done; leave when wave 0 leaves
    const int wave = tid >> 6, hl = tid & 63;
    uint32_t gen = 0;
    for (;;) {
      const uint32_t g = (uint32_t)__builtin_amdgcn_readfirstlane((int)ctl(0));
      if (g != gen) {
        gen = g;
        const uint32_t prm = (uint32_t)__builtin_amdgcn_readfirstlane((int)ctl(1));
        const uint32_t cnt = min(prm & 0xFFu, kSvcMaxBurst);
        if (prm >> 31)
          serve_burst<true>(cnt, hl, wave);
        else
          serve_burst<false>(cnt, hl, wave);
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0);  // this wave's results have landed
        __asm__ __volatile__("" ::: "memory");
        if (hl == 0)
          __hip_atomic_fetch_add((lds_w*)(uintptr_t)(kSvcCtl + 8u), 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        continue;
      }
      if (ctl(3) != 0u) return;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  const int lane = tid;
  const SvcKeysL kk = SvcKeysL::make(lane);
  ServiceRing* r = s.ring;
  const uint8_t* frame = (const uint8_t*)r + kSvcFrame;
  // the group's result goes to two LDS words past the tables (flat stores
  // through generic pointers), then out as one 8-byte answer
  constexpr uint32_t kOut = kSvcOut;
  IcrcArgs a{};
  a.frames = frame;
  a.n = 1;
  a.icrc_out = (uint32_t*)(lds_u32*)(uintptr_t)kOut;
  a.status_out = (uint8_t*)(lds_u32*)(uintptr_t)(kOut + 4u);
  uint32_t served = s.served;
  const auto ring_rsrc = out_rsrc(r, 64u);
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  uint32_t polls = 0;
  // one poll's value: 0 = nothing to do, 1 = a request served, 2 = leave
  // the device's busy word (announce_batch): a batch workgroup started less
  // than busy_ticks ago -> leave once no request is pending
  const auto busy_rsrc = out_rsrc((void*)s.busy, s.busy ? 16u : 0u);  // (0 bytes: loads give 0)
  auto step = [&](const u32x4 head, const u32x4 bz) -> int {
    const uint64_t req = (uint64_t)head.x | ((uint64_t)head.y << 32);
    const uint32_t seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)req);
    // a batch kernel started on the device less than busy_ticks ago: the
    // wave answers what is pending and leaves (a caller that keeps the wave
    // busy must not keep a batch workgroup off this CU: round 4 measured a
    // batch 1.21x slower beside one thread calling back to back)
    const uint64_t stamp = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)bz.x) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)bz.y) << 32);
    const bool batch_young =
        stamp != 0 && (int64_t)(__builtin_amdgcn_s_memrealtime() - stamp) < (int64_t)s.busy_ticks;
    const int served_rc = batch_young ? 2 : 1;
    if (seq != served) {
      const uint64_t t_seen = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the frame the host wrote before req
      uint32_t L = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(req >> 32));
      bool inl = false;
      uint32_t d12[12];
      if (L & kSvcInline) {  // (uniform) the 48 bytes of lanes 1-3 against the check word
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          d12[4 * q + 0] = (uint32_t)__builtin_amdgcn_readlane((int)head.x, q + 1);
          d12[4 * q + 1] = (uint32_t)__builtin_amdgcn_readlane((int)head.y, q + 1);
          d12[4 * q + 2] = (uint32_t)__builtin_amdgcn_readlane((int)head.z, q + 1);
          d12[4 * q + 3] = (uint32_t)__builtin_amdgcn_readlane((int)head.w, q + 1);
        }
        inl = (uint32_t)__builtin_amdgcn_readfirstlane((int)head.w) == svc_inline_check(seq, d12) &&
              (L & ~kSvcInline) <= kSvcInlineMax;
      }
      if (inl) {
        L &= ~kSvcInline;
        const uint32_t d0 = d12[0], d2 = d12[2];
        if ((L & 3u) == 0 && L >= 44 && ((d0 >> 4) & 0xFu) == 4u && (d0 & 0xFu) == 5u &&
            ((d2 >> 8) & 0xFFu) == 17u) {
          // IHL 5, IPv4/UDP, whole dwords (ACK, NAK, read request, atomic
          // ack): lane p of the first 16 holds frame dword k = p - (16 - n)
          // (zeros in front), masked; each lane multiplies its dword by
          // x^(-32 p) (the bits of p: Mul(-32), Mul(-32)^2, Mul(-128),
          // Mul(-256), the service's combine sets), the 16 lanes XOR, and
          // Mul(-512) then Mul(1024) make it x^(32 (16 - p)) per dword: the
          // register after the frame.  Five dependent table steps and a
          // reduction instead of the group code's head, fold and combine.
          const int n = (int)((L - 4u) >> 2);  // 10 or 11
          const int p = lane & 15, k = p - (16 - n);
          uint32_t v = 0;
#pragma unroll
          for (int j = 0; j < 12; ++j) v = k == j ? d12[j] : v;
          v = fix_dword(v, k, 6, 8);
          if (lane >= 16 || k < 0) v = 0;
          constexpr uint32_t kC = SvcKeysL::kComb;  // Mul(-32), then Mul(-128 2^l)
          uint32_t y = mul_comb(v, kC);
          v = (p & 1) ? y : v;
          y = mul_comb(mul_comb(v, kC), kC);
          v = (p & 2) ? y : v;
          y = mul_comb(v, kC + 4096u);
          v = (p & 4) ? y : v;
          y = mul_comb(v, kC + 2u * 4096u);
          v = (p & 8) ? y : v;
#pragma unroll
          for (int d = 8; d >= 1; d >>= 1) v ^= (uint32_t)__shfl_xor((int)v, d, 16);
          v = mul_comb(v, kC + 3u * 4096u);  // Mul(-512)
          uint32_t P = 0, T = 0;
          SvcKeysS::make(lane).absorb(P, T, v);  // Mul(1024)
          const uint32_t icrc = ~(P ^ T);
          const uint32_t st = ((((d0 >> 8) & 0xFF00u) | (d0 >> 24)) != L) ? kPktLenMismatch : 0u;
          if (lane == 0) {
            const uint64_t ans = (uint64_t)icrc | ((uint64_t)st << 32) | ((uint64_t)(seq & kSvcSeqMask) << 40);
            r->t_seen = t_seen;
            r->t_done = __builtin_amdgcn_s_memrealtime();
            r->polls = polls;
            __hip_atomic_store(&r->resp, ans, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          polls = 0;
          served = seq;
          t_last = __builtin_amdgcn_s_memrealtime();
          return served_rc;
        }
        // other inline frames: into LDS, then folded from there as a
        // one-frame burst on this wave (G = 8)
        if (lane >= 1 && lane <= 3) *(lds_u32x4*)(uintptr_t)(kBurstStage + 16u * (uint32_t)(lane - 1)) = head;
        if (lane == 0)
          *(__attribute__((address_space(3))) uint64_t*)(uintptr_t)kSvcDescLds = (uint64_t)L << 32;
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);  // (lgkmcnt(0): the frame and descriptor are in LDS)
        __asm__ __volatile__("" ::: "memory");
        serve_burst<false>(1u, lane, 0);
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0);  // the result's flat stores have landed
        __asm__ __volatile__("" ::: "memory");
        if (lane == 0) {
          const uint64_t ans = (uint64_t)lds_rd(kBurstIcrc) | ((uint64_t)lds_rd8(kBurstSt) << 32) |
                               ((uint64_t)(seq & kSvcSeqMask) << 40);
          r->t_seen = t_seen;
          r->t_done = __builtin_amdgcn_s_memrealtime();
          r->polls = polls;
          __hip_atomic_store(&r->resp, ans, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        polls = 0;
        served = seq;
        t_last = __builtin_amdgcn_s_memrealtime();
        return served_rc;
      }
      L &= ~kSvcInline;  // (a torn inline read: the frame at kSvcFrame, below)
      if (L & kSvcBurst) {
        const uint32_t cnt = min(L & 0xFFu, kSvcMaxBurst);
        const uint32_t kib = min((L >> 16) & 0x7Fu, kSvcMaxFrame / 1024u);  // packed KiB
        const uint64_t* desc = (const uint64_t*)((const uint8_t*)r + kSvcDesc);
        // the packed frames into LDS: one LDS-DMA wave-instruction per KiB, all
        // in flight at once (one PCIe round trip), and every descriptor with
        // one load
        for (uint32_t k = 0; k < kib; ++k)
          __builtin_amdgcn_global_load_lds(
              (const __attribute__((address_space(1))) void*)(frame + 1024u * k + 16u * (uint32_t)lane),
              (__attribute__((address_space(3))) void*)(uintptr_t)(kBurstStage + 1024u * k), 16, 0, 0);
        const uint64_t dl = (uint32_t)lane < cnt ? desc[lane] : 0ull;
        *(__attribute__((address_space(3))) uint64_t*)(uintptr_t)(kSvcDescLds + 8u * (uint32_t)lane) = dl;
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0);  // frames and descriptors are in LDS
        __asm__ __volatile__("" ::: "memory");
        if (cnt > 0) {
          // post the burst to the helper waves, take this wave's rounds
          if (lane == 0) {
            lds_wr(kSvcCtl + 4u, cnt | ((L & kSvcVerify) ? 0x80000000u : 0u));
            __asm__ __volatile__("" ::: "memory");
            __builtin_amdgcn_s_waitcnt(0xC07F);  // (lgkmcnt(0): the parameters first)
            __asm__ __volatile__("" ::: "memory");
            __hip_atomic_store((lds_w*)(uintptr_t)kSvcCtl, ctl(0) + 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          if (L & kSvcVerify)
            serve_burst<true>(cnt, lane, 0);
          else
            serve_burst<false>(cnt, lane, 0);
          // every helper counts itself done (those with no round at once);
          // bounded: a burst not finished within 100 ms ends the service
          // unanswered (the host then times out and takes the launch path)
          const uint64_t tw = __builtin_amdgcn_s_memrealtime();
          bool helped = true;
          while ((uint32_t)__builtin_amdgcn_readfirstlane((int)ctl(2)) < (uint32_t)(kSvcWaves - 1)) {
            if (__builtin_amdgcn_s_memrealtime() - tw > 10000000ull) {
              helped = false;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (!helped) return 2;
          if (lane == 0) lds_wr(kSvcCtl + 8u, 0u);
        }
        // the results (flat and LDS stores) have landed before the lanes read them
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0);
        __asm__ __volatile__("" ::: "memory");
        if (lane == 0) {  // (diagnostics, before the answers: the host reads them after)
          r->t_seen = t_seen;
          r->t_done = __builtin_amdgcn_s_memrealtime();
          r->polls = polls;
        }
        // each answer carries the request's tag: one 8-byte store per frame,
        // no fence (the host cleared the answers before the request)
        if ((uint32_t)lane < cnt) {
          const uint64_t ans = (uint64_t)lds_rd(kBurstIcrc + 4u * (uint32_t)lane) |
                               ((uint64_t)lds_rd8(kBurstSt + (uint32_t)lane) << 32) |
                               ((uint64_t)lds_rd8(kBurstOk + (uint32_t)lane) << 40) |
                               ((uint64_t)svc_burst_tag(seq) << 48);
          __hip_atomic_store((uint64_t*)((uint8_t*)r + kSvcAns) + lane, ans, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
        polls = 0;
        served = seq;
        t_last = __builtin_amdgcn_s_memrealtime();
        return served_rc;
      }
      const Pkt p = describe<DPI>(frame, 0, true, 0, L <= kSvcMaxFrame ? L : 0u);
      Batch<kUnroll> b = issue_packet<LOG2G, false>(p, lane);
      finish_packet<LOG2G, false, SvcKeysL, kSvcLut>(a, p, b, lane, 0, kk);
      // the flat stores of the result (through generic pointers into LDS)
      // have landed before lane 0 reads the words back with LDS reads
      __asm__ __volatile__("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0);
      __asm__ __volatile__("" ::: "memory");
      if (lane == 0) {
        const uint64_t ans = (uint64_t)lds_rd(kOut) | ((uint64_t)(lds_rd(kOut + 4u) & 0xFFu) << 32) |
                             ((uint64_t)(seq & kSvcSeqMask) << 40);
        // (timing of this request for ricrc_ctx_service_times: diagnostics,
        // not ordered against the answer)
        r->t_seen = t_seen;
        r->t_done = __builtin_amdgcn_s_memrealtime();
        r->polls = polls;
        __hip_atomic_store(&r->resp, ans, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      polls = 0;
      served = seq;
      t_last = __builtin_amdgcn_s_memrealtime();
      return served_rc;
    }
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)head.z) != 0u) return 2;  // stop
    if (batch_young) return 2;  // a batch starts
    if (__builtin_amdgcn_s_memrealtime() - t_last > s.idle_ticks) return 2;
    __builtin_amdgcn_s_sleep(2);
    return 0;
  };
  // ONE PCIe read per poll: the request word and the stop flag share the
  // slot's first 16 bytes (a 16-byte system-coherent load, sc0 sc1; two
  // separate loads made every poll two round trips), and TWO polls in
  // flight: the next one is issued before this one's value is looked at, so
  // a request is seen about half a round trip sooner.  A poll issued before a
  // request was served shows its sequence number again (== served): ignored.
  // The busy word is read beside the slot (both loads in flight together).
  // (lanes 0-3 read the slot's first 64 bytes: request, stop, check and the
  // inline frame; the other lanes repeat lane 3's chunk -- one 64-byte read)
  const uint32_t poll_off = 16u * (uint32_t)min(lane, 3);
  auto poll = [&]() { return __builtin_amdgcn_raw_buffer_load_b128(ring_rsrc, poll_off, 0u, 17); };
  auto poll_busy = [&]() { return __builtin_amdgcn_raw_buffer_load_b128(busy_rsrc, 0u, 0u, 17); };
  if constexpr (kSvcPolls == 4) {  // four polls in flight
    u32x4 hA = poll(), bA = poll_busy(), hB = poll(), bB = poll_busy(), hC = poll(), bC = poll_busy();
    for (;;) {
      const u32x4 hD = poll(), bD = poll_busy();
      ++polls;
      if (step(hA, bA) == 2) break;
      hA = poll();
      bA = poll_busy();
      ++polls;
      if (step(hB, bB) == 2) break;
      hB = poll();
      bB = poll_busy();
      ++polls;
      if (step(hC, bC) == 2) break;
      hC = poll();
      bC = poll_busy();
      ++polls;
      if (step(hD, bD) == 2) break;
    }
  } else {
    u32x4 hA = poll(), bA = poll_busy();
    for (;;) {
      const u32x4 hB = poll(), bB = poll_busy();
      ++polls;
      if (step(hA, bA) == 2) break;
      hA = poll();
      bA = poll_busy();
      ++polls;
      if (step(hB, bB) == 2) break;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // the poll still in flight has returned
  if (lane == 0)  // the helper waves leave too
    __hip_atomic_store((lds_w*)(uintptr_t)(kSvcCtl + 12u), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) __hip_atomic_store(&r->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef void (*kernel_fn)(IcrcArgs);

template <int LOG2G>
kernel_fn pick(bool ragged, bool verify) {
  if (ragged && ragged_has_compact(LOG2G))  // the mixed-width kernel (SORTED)
    return verify ? icrc_ragged_mixed_kernel<true> : icrc_ragged_mixed_kernel<false>;
  if (ragged) return verify ? icrc_ragged_kernel<LOG2G, true> : icrc_ragged_kernel<LOG2G, false>;
  return verify ? icrc_strided_kernel<LOG2G, true> : icrc_strided_kernel<LOG2G, false>;
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

template <bool V>
kernel_fn pick_compact(int outs) {
  switch (outs) {
    case 0: return icrc_compact_kernel<V, 0>;
    case 1: return icrc_compact_kernel<V, 1>;
    case 2: return icrc_compact_kernel<V, 2>;
    default: return icrc_compact_kernel<V, 3>;
  }
}
kernel_fn select_compact(bool verify, int outs) {
  return verify ? pick_compact<true>(outs) : pick_compact<false>(outs);
}

size_t lds_bytes(int log2g, bool ragged) {
  if (!ragged) return 163840u;  // tables, fix-up LUT, then the block's ICRC words
  switch (log2g) {
    case 0: return RaggedLds<0>::kBytes;
    case 1: return RaggedLds<1>::kBytes;
    case 2: return RaggedLds<2>::kBytes;
    case 3: return kMixedLdsBytes;
    case 4: return RaggedLds<4>::kBytes;
    case 5: return RaggedLds<5>::kBytes;
    default: return RaggedLds<6>::kBytes;
  }
}

template <int C, bool V>
kernel_fn pick_small(int outs) {
  switch (outs) {
    case 0: return icrc_small_kernel<C, V, 0>;
    case 1: return icrc_small_kernel<C, V, 1>;
    case 2: return icrc_small_kernel<C, V, 2>;
    default: return icrc_small_kernel<C, V, 3>;
  }
}

kernel_fn select_small(int C, bool verify, int outs) {
  switch (C) {
    case 3: return verify ? pick_small<3, true>(outs) : pick_small<3, false>(outs);
    case 4: return verify ? pick_small<4, true>(outs) : pick_small<4, false>(outs);
    case 5: return verify ? pick_small<5, true>(outs) : pick_small<5, false>(outs);
    case 6: return verify ? pick_small<6, true>(outs) : pick_small<6, false>(outs);
    case 7: return verify ? pick_small<7, true>(outs) : pick_small<7, false>(outs);
    case 8: return verify ? pick_small<8, true>(outs) : pick_small<8, false>(outs);
    default: return nullptr;
  }
}


}  // namespace

void build_table_image(uint32_t* out) {
  for (int l = 0; l < kNumMainSets; ++l) table_set(128ll << l, out + l * 1024);
  uint32_t* comb = out + kNumMainSets * 1024;
  table_set(-32, comb);
  for (int l = 0; l < kMaxLog2G; ++l) table_set(-(128ll << l), comb + (1 + l) * 1024);
  const uint32_t* m64 = out + kMul64Set * 1024;
  table_set(64, out + kMul64Set * 1024);
  uint32_t* rows = out + kSmallImageOff;  // Keys8 rows of Mul(64), the LDS image's low halves
  for (int e = 0; e < 256; ++e)
    for (int t = 0; t < 4; ++t)
      for (int c = 0; c < 8; ++c) rows[e * 32 + t * 8 + c] = m64[t * 256 + e];
}

hipError_t set_dynamic_lds(const void* fn, int bytes) {
  hipFuncAttributes fa;
  hipError_t e = hipFuncGetAttributes(&fa, fn);
  if (e != hipSuccess) return e;
  if (fa.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

hipError_t prepare_kernels() {
  for (int l = 0; l <= kMaxLog2G; ++l)
    for (int r = 0; r < 2; ++r)
      for (int v = 0; v < 2; ++v) {
        hipError_t e = set_dynamic_lds((const void*)select_kernel(l, r, v), (int)lds_bytes(l, r));
        if (e != hipSuccess) return e;
      }
  for (int c = kSmallMinChunks; c <= kSmallMaxChunks; ++c)
    for (int v = 0; v < 2; ++v)
      for (int o = 0; o < 4; ++o) {
        hipError_t e = set_dynamic_lds((const void*)select_small(c, v, o), 163840);
        if (e != hipSuccess) return e;
      }
  for (int v = 0; v < 2; ++v)
    for (int o = 0; o < 4; ++o) {
      hipError_t e = set_dynamic_lds((const void*)select_compact(v, o), (int)kCompactLdsBytes);
      if (e != hipSuccess) return e;
    }
  hipError_t e = set_dynamic_lds((const void*)icrc_service_kernel, (int)kSvcLds);
  if (e != hipSuccess) return e;
  return prepare_segment_kernels();
}

hipError_t launch_service(const ServiceArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(icrc_service_kernel, dim3(1), dim3(kSvcThreads), kSvcLds, stream, a);
  return hipGetLastError();
}

hipError_t launch_icrc(const IcrcArgs& a, int log2g, bool ragged, bool verify, int num_cus,
                       hipStream_t stream, bool compact) {
  if (a.n == 0) return hipSuccess;
  if (ragged && compact) {  // the streaming compact kernel (any lanes setting: its own)
    const int outs = (a.icrc_out ? 1 : 0) | (a.status_out ? 2 : 0);
    const uint64_t groups = (a.n + 63) / 64;
    uint64_t blocks = (groups + kCompactWaves - 1) / kCompactWaves;
    if (blocks > (uint64_t)num_cus) blocks = (uint64_t)num_cus;
    hipLaunchKernelGGL(select_compact(verify, outs), dim3((unsigned)blocks), dim3(kCompactThreads),
                       kCompactLdsBytes, stream, a);
    return hipGetLastError();
  }
  kernel_fn k = select_kernel(log2g, ragged, verify);
  if (!k) return hipErrorInvalidValue;
  const uint32_t ppw = 64u >> log2g;
  const uint64_t nsets = (a.n + ppw - 1) / ppw;
  const int waves = ragged ? kIcrcWaves : kStridedWaves;
  uint64_t blocks = (nsets + waves - 1) / waves;
  const uint64_t cap = (uint64_t)num_cus;  // one workgroup per CU (the LDS holds one)
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(64 * waves), lds_bytes(log2g, ragged), stream, a);
  return hipGetLastError();
}

hipError_t launch_icrc_small(const IcrcArgs& a, bool verify, int num_cus, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  if (a.stride > kSmallMaxStride || (a.stride & 3u) || a.stride < kSmallMinStride) return hipErrorInvalidValue;
  // 16-byte loads per lane per batch: exactly ceil(4 stride / 64), so only
  // the last one is partial (cfg5, 108 B: 432 chunks, C = 7)
  const int C = (int)((a.stride + 15u) / 16u);
  if (C < kSmallMinChunks || C > kSmallMaxChunks) return hipErrorInvalidValue;
  const int outs = (a.icrc_out ? 1 : 0) | (a.status_out ? 2 : 0);
  kernel_fn k = select_small(C, verify, outs);
  if (!k) return hipErrorInvalidValue;
  const uint32_t slot = 64u * (uint32_t)a.stride;
  uint32_t nw = min((uint32_t)kSmallMaxWaves, (kSmallEnd - kSmallStage) / slot);
  if (nw > 2 && (nw & 1u)) --nw;  // even: every SIMD the same number of waves
  if (nw < 8) return hipErrorInvalidValue;  // (the kernel stages its tables with >= 512 threads)
  const size_t lds = 163840;  // staging slots, then the output ring in what is left
  const uint64_t nb = (a.n + 63) / 64;
  uint64_t blocks = (nb + nw - 1) / nw;
  if (blocks > (uint64_t)num_cus) blocks = (uint64_t)num_cus;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(64 * nw), lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, uint32_t* sink, int num_cus,
                              hipStream_t stream) {
  const uint64_t n16 = bytes / 16;
  if (n16 == 0) return hipSuccess;
  hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)num_cus), dim3(kStreamThreads), 0, stream,
                     (const u32x4*)buf, n16, sink);
  return hipGetLastError();
}

}  // namespace ricrc
