/*
 * roce_icrc.h -- C ABI of the MI355X (gfx950) RoCEv2 ICRC engine, libroceicrc.so.
 *
 * Drop-in boundary for datenlord/roce-sim's per-packet Invariant CRC:
 *
 *   reference                                   replaced by
 *   ------------------------------------------  ---------------------------------
 *   BTH.compute_icrc(self, p)  src/roce.py:192   ricrc_icrc / ricrc_compute_one / ricrc_compute_batch
 *     (fires from BTH.post_build src/roce.py:228-233, itself run by scapy
 *      send() at src/roce_sq.py:1197 (requester emit, retry re-emit via
 *      src/roce_sq.py:743) and src/roce_rq.py:731 (responder emit))
 *   zlib.crc32(raw(pshdr)[:-4]) src/roce.py:218  the HIP kernels behind every entry point
 *   BTH.pack_icrc               src/roce.py:187  icrc_out[i] is the uint32 CRC; its wire
 *                                                bytes are its little-endian encoding
 *   (no receive-side check; the reference only  ricrc_verify_batch[_dev]: recompute and
 *    parses BTH.icrc, src/roce.py:184,           compare with the 4 trailing bytes
 *    src/roce_v2.py:350, src/roce_rq.py:901)
 *
 * Frame convention.  Every frame is a WIRE IPv4 frame: IPv4 header (IHL >= 5)
 * | UDP | BTH | extension headers | payload | pad | 4-byte ICRC slot.  `len`
 * includes the ICRC slot.  The engine applies the reference's masks itself
 * (IP tos, ttl, header checksum; UDP checksum; BTH fecn|becn|resv6 byte, all
 * forced to ones, src/roce.py:204-211) and the 8 x 0xFF pseudo-LRH prefix
 * (src/roce.py:204), so callers pass the bytes exactly as they go on the wire.
 *
 * Per-packet status.  A frame that is not IPv4 (version != 4 or IHL < 5), not
 * UDP (protocol != 17), shorter than IP+UDP+BTH+ICRC or longer than 65535
 * bytes gets ICRC 0 and a status bit -- the reference's "warning + ICRC
 * 00000000" path (src/roce.py:195-200, 220-223).  These are not call errors:
 * the batch call still returns RICRC_OK.  Frames of any other length are
 * CRC'd like zlib.crc32 does (those that are not a multiple of 4 bytes long,
 * which roce-sim's emit paths never build, and those at unaligned addresses
 * take a slower byte-load path).
 *
 * Ownership.  The caller owns every buffer.  No pointer is retained after a
 * synchronous call returns; the *_dev variants are asynchronous on `stream`
 * and use their arguments until that stream has executed the work.
 *
 * Threading.  All entry points are re-entrant.  A ricrc_ctx owns one HIP
 * stream plus device scratch and is NOT thread-safe: use one context per host
 * thread (the reference calls from a 10-thread gRPC pool,
 * src/sanity_side.py:383), or the context-free ricrc_icrc, which is
 * thread-safe.  Python's ctypes releases the GIL around calls.
 *
 * Return codes: 0 on success, a negative errno-style code otherwise.
 */
#ifndef ROCE_ICRC_H
#define ROCE_ICRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RICRC_ABI_VERSION 5

/* call-level return codes */
#define RICRC_OK 0
#define RICRC_EINVAL (-22) /* bad argument (null pointer, n too large, ...) */
#define RICRC_ENOMEM (-12) /* host or device allocation failed              */
#define RICRC_ENODEV (-19) /* no usable gfx950 device / device index        */
#define RICRC_EIO (-5)     /* HIP runtime or kernel launch failure          */

/* per-packet status bits (status_out[i]) */
#define RICRC_PKT_BAD_LEN 0x01       /* too short, or > 65535                     */
#define RICRC_PKT_NOT_IPV4 0x02      /* IP version != 4 or IHL < 5 (ICRC = 0)     */
#define RICRC_PKT_NOT_UDP 0x04       /* IP protocol != 17 (ICRC = 0)              */
#define RICRC_PKT_LEN_MISMATCH 0x08  /* IP total length != len (ICRC still computed) */
#define RICRC_PKT_ICRC_MISMATCH 0x10 /* verify: trailer != recomputed ICRC        */
#define RICRC_PKT_FATAL (RICRC_PKT_BAD_LEN | RICRC_PKT_NOT_IPV4 | RICRC_PKT_NOT_UDP)

typedef struct ricrc_ctx ricrc_ctx;

/* ---- library / device -------------------------------------------------- */
int ricrc_abi_version(void);
const char* ricrc_strerror(int code);
/* Number of visible HIP devices (0 when none). */
int ricrc_device_count(int* count);

/* ---- context ------------------------------------------------------------ */
/* Create a context on HIP device `device`: selects the device, creates one
 * non-blocking stream, builds the GF(2) folding tables and uploads them. */
int ricrc_ctx_create(int device, ricrc_ctx** out);
void ricrc_ctx_destroy(ricrc_ctx* ctx);
/* Lanes cooperating on one packet (1,2,4,...,64); 0 = automatic by length
 * (strided frames with a stride of 44-128 bytes, a multiple of 4, then use
 * the lane-per-packet kernel with LDS-staged loads -- shorter strides hold
 * only unusable frames, which the lane-group kernels mark RICRC_PKT_BAD_LEN
 * as that kernel would; any non-zero setting forces
 * the lane-group kernels).  For ragged batches 8 selects the mixed-width
 * kernel, which runs sorted claims of short frames (<= 600 B) with 4 lanes
 * per packet and the rest with 8; it is also the automatic choice of the
 * device-resident ragged calls. */
int ricrc_ctx_set_lanes_per_packet(ricrc_ctx* ctx, int lanes);
/* The hipStream_t the synchronous host-buffer calls run on. */
void* ricrc_ctx_stream(ricrc_ctx* ctx);

/* Ragged-kernel variant (ABI 5).  Ragged batches (automatic lanes, or 8) run
 * one of two kernels.  COMPACT streams 64-frame groups: a group whose frames
 * are 44-128 B, dword-aligned, in order and inside 4 KiB (a responder's ACK /
 * NAK / atomic-ack stream, src/roce_rq.py:767-853) is folded lane-per-frame
 * straight from one coalesced span read; any other group is folded by lane
 * groups, unsorted.  SORTED counting-sorts windows of 8192 frames by length
 * and folds them in size-homogeneous lane groups (mixed-MTU data,
 * src/roce_v2.py:327-372).  Both give the same words; each is the faster one
 * for its composition (2^24 ACK frames: compact 1.25x; mixed MTU: sorted).
 *   RICRC_RAGGED_AUTO     default.  Host-buffer calls decide per call from
 *                         the lengths they hold (compact when at least half
 *                         of the batch's 64-frame groups hold only frames of
 *                         at most 128 B).  Device-resident calls cannot see
 *                         the lengths: they follow the context's learned
 *                         hint, which the previous ragged launch's first
 *                         workgroup sets by the same rule from the batch's
 *                         first 12 groups (both kernels probe the same
 *                         ones) -- so launches enqueued back to back
 *                         follow the last launch FINISHED before them.
 *   RICRC_RAGGED_COMPACT  every ragged launch of the context runs the compact
 *                         kernel.
 *   RICRC_RAGGED_SORTED   ... the sorted kernel.
 * A context is single-threaded, so a caller whose device-resident batches
 * alternate composition sets the variant before each call. */
#define RICRC_RAGGED_AUTO 0
#define RICRC_RAGGED_COMPACT 1
#define RICRC_RAGGED_SORTED 2
int ricrc_ctx_set_ragged_variant(ricrc_ctx* ctx, int variant);
/* The variant the context's last ragged launch ran (RICRC_RAGGED_COMPACT or
 * RICRC_RAGGED_SORTED; RICRC_RAGGED_SORTED also for the single-width ragged
 * kernels that an explicit lanes setting other than 8 selects),
 * RICRC_RAGGED_AUTO before any.  A launch that failed to enqueue does not
 * change it. */
int ricrc_ctx_last_ragged_variant(ricrc_ctx* ctx, int* variant_out);

/* ---- host buffers, synchronous (H2D + kernel + D2H) --------------------- */
/* The per-packet drop-in for BTH.compute_icrc (src/roce.py:192): one wire
 * frame in, its ICRC out.  By default it goes through the context's
 * per-packet service: one resident GPU wave polling a request slot in pinned
 * host memory, which reads the frame over PCIe and answers in host memory --
 * no kernel launch, copy or stream synchronisation per call.  The wave is
 * launched by the first call and leaves after `idle_us` without a call, when
 * the context launches batch work (it holds one CU's LDS while it runs), or
 * when the context is destroyed.  Frames over 64 KiB, or a context whose
 * service is off, take one staged kernel launch per call instead. */
int ricrc_compute_one(ricrc_ctx* ctx, const uint8_t* frame, size_t len, uint32_t* icrc_out,
                      uint8_t* status_out /* nullable */);
/* The same per-packet drop-in without a context, thread-safe: what a
 * `compute_icrc` hook (src/roce.py:192) called from any thread of the
 * reference's gRPC pool (src/sanity_side.py:383) binds to.  Each calling
 * thread borrows one library-owned context on its current HIP device (created
 * on the thread's first call, ~ms); a thread that exits returns it to a pool
 * that later threads reuse, and the pool lives until process exit.  Same
 * answers, status bits and costs as ricrc_compute_one. */
int ricrc_icrc(const uint8_t* frame, size_t len, uint32_t* icrc_out,
               uint8_t* status_out /* nullable */);
/* Idle timeout of the per-packet service in microseconds (default 1000);
 * 0 turns the service off (ricrc_compute_one and small bursts then launch a
 * kernel per call). */
int ricrc_ctx_set_service(ricrc_ctx* ctx, uint32_t idle_us);

/* Ragged batch: frame i is frames[offsets[i] .. offsets[i] + lens[i]).
 * `frames_bytes` is the size of the `frames` buffer (bounds for the copy).
 * A small burst (up to 64 frames, 64 KiB packed; automatic lanes) goes to the
 * same resident wave as ricrc_compute_one, as one request (the wave copies
 * the packed frames into LDS and folds eight at a time); larger batches, a
 * context whose service is off, or an explicit lanes setting launch the
 * kernels (copy in, kernel, copy out). */
int ricrc_compute_batch(ricrc_ctx* ctx, const uint8_t* frames, size_t frames_bytes,
                        const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                        uint32_t* icrc_out, uint8_t* status_out /* nullable */);
int ricrc_verify_batch(ricrc_ctx* ctx, const uint8_t* frames, size_t frames_bytes,
                       const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                       uint8_t* ok_out, uint32_t* icrc_out /* nullable */,
                       uint8_t* status_out /* nullable */);

/* Fixed-size frames at frames + i * stride, each `len` bytes long. */
int ricrc_compute_strided(ricrc_ctx* ctx, const uint8_t* frames, uint64_t stride, uint32_t len,
                          uint32_t n, uint32_t* icrc_out, uint8_t* status_out /* nullable */);

/* Round-robin split over several contexts (one per GPU): packet i goes to
 * ctxs[i % nctx] (per-packet independence, src/roce.py:192-219).  One host
 * thread per distinct context streams its shard in chunks through two pinned
 * staging blocks the context owns (gather of chunk k + 1 overlaps the copies
 * and kernel of chunk k); contexts named more than once run their shards one
 * after another. */
int ricrc_compute_batch_multi(ricrc_ctx** ctxs, int nctx, const uint8_t* frames,
                              size_t frames_bytes, const uint64_t* offsets,
                              const uint32_t* lens, uint32_t n, uint32_t* icrc_out,
                              uint8_t* status_out /* nullable */);
/* The receive side of the same split: what RoCEv2.recv_pkts
 * (src/roce_v2.py:327-372) would call with one received batch on a node of
 * several GPUs.  ok_out[i] = 1 iff frame i's trailer equals its ICRC (the
 * ricrc_verify_batch rule). */
int ricrc_verify_batch_multi(ricrc_ctx** ctxs, int nctx, const uint8_t* frames,
                             size_t frames_bytes, const uint64_t* offsets,
                             const uint32_t* lens, uint32_t n, uint8_t* ok_out,
                             uint32_t* icrc_out /* nullable */,
                             uint8_t* status_out /* nullable */);

/* Page-lock a caller buffer so the H2D/D2H copies above run at DMA speed. */
int ricrc_host_register(void* ptr, size_t bytes);
int ricrc_host_unregister(void* ptr);

/* ---- device-resident, asynchronous on `stream` (a hipStream_t; NULL is the
 *      HIP null stream, as for any HIP API); all pointers are device
 *      pointers ------------------------------------------------------------ */
int ricrc_compute_batch_dev(ricrc_ctx* ctx, const uint8_t* d_frames, const uint64_t* d_offsets,
                            const uint32_t* d_lens, uint32_t n, uint32_t* d_icrc,
                            uint8_t* d_status /* nullable */, void* stream);
int ricrc_verify_batch_dev(ricrc_ctx* ctx, const uint8_t* d_frames, const uint64_t* d_offsets,
                           const uint32_t* d_lens, uint32_t n, uint8_t* d_ok,
                           uint32_t* d_icrc /* nullable */, uint8_t* d_status /* nullable */,
                           void* stream);
int ricrc_compute_strided_dev(ricrc_ctx* ctx, const uint8_t* d_frames, uint64_t stride,
                              uint32_t len, uint32_t n, uint32_t* d_icrc,
                              uint8_t* d_status /* nullable */, void* stream);
int ricrc_verify_strided_dev(ricrc_ctx* ctx, const uint8_t* d_frames, uint64_t stride,
                             uint32_t len, uint32_t n, uint8_t* d_ok,
                             uint32_t* d_icrc /* nullable */, uint8_t* d_status /* nullable */,
                             void* stream);

/* ---- MR -> packet segmentation fused with the ICRC (device-built frames) --
 *
 *   reference                                        replaced by
 *   -----------------------------------------------  -----------------------------
 *   TXLogic.process_send_req    src/roce_sq.py:1243   one ricrc_seg_wr of op SEND*
 *   TXLogic.process_write_req   src/roce_sq.py:1323   one ricrc_seg_wr of op RDMA_WRITE*
 *   ReadReqCtx.commit           src/roce_rq.py:388    one ricrc_seg_wr of op READ_RESPONSE
 *   TXLogic.process_read_req    src/roce_sq.py:1413   op READ_REQUEST (BTH + RETH)
 *   TXLogic.process_atomic_req  src/roce_sq.py:1441   op COMPARE_SWAP / FETCH_ADD (+ AtomicETH)
 *   RXLogic.process_ack         src/roce_rq.py:767    op ACK (AETH ACK, value 31)
 *   RXLogic.process_nak_rnr     src/roce_rq.py:778    op RNR_NAK (AETH RNR, value = imm)
 *   RXLogic.process_nak_seq_err src/roce_rq.py:805    op NAK, imm 0 (AETH NAK, value 0)
 *   RXLogic.process_nak_err     src/roce_rq.py:827    op NAK, imm 1 / 2 / 3 (or 31)
 *   AtomicReqCtx.commit         src/roce_rq.py:490    op ATOMIC_ACK (AETH ACK 31 + AtomicAckETH)
 *   Util.compute_wr_pkt_num     src/roce_util.py:183  ricrc_segment_plan
 *   Util.add_padding_if_needed  src/roce_util.py:187  (in the kernel)
 *   IP()/UDP() wrap of send_ip_pkt / send_pkt         (in the kernel: IPv4 id 1, ttl 64,
 *     src/roce_sq.py:1186-1197, src/roce_rq.py:705-731  header checksum, UDP dport 4791,
 *                                                       UDP checksum over the final bytes)
 *   BTH.compute_icrc            src/roce.py:192       (in the kernel, same register fold)
 *
 * Packet k (0-based) of a WR of n = compute_wr_pkt_num(length, pmtu) packets
 * gets PSN (psn + k) mod 2^24, the FIRST/MIDDLE/LAST/ONLY opcode of its
 * position, the extension headers of that opcode (RETH on WRITE FIRST/ONLY,
 * RETHImmDt on WRITE_ONLY_WITH_IMM, ImmDt on *_WITH_IMM last, IETH on
 * SEND_*_WITH_INV last, AETH(ACK, 31, msn) on READ_RESPONSE FIRST/LAST/ONLY),
 * the MR bytes [mr_offset + k*pmtu, ...) as payload (none when length == 0),
 * zero padding to 4 bytes with BTH.padcount, ackreq = SIGNALED and solicited
 * = SOLICITED on the last packet only (solicited only for SEND* and
 * RDMA_WRITE_WITH_IMM, as the reference), and its ICRC.
 *
 * Header-only ops are one packet each and read no MR bytes (mr_offset and
 * flags unused; `length` is RETH.dlen for READ_REQUEST and ignored otherwise):
 *   READ_REQUEST        0x0C  ackreq 1, RETH(remote_va, rkey, length)
 *   COMPARE_SWAP        0x13  ackreq 1, AtomicETH(remote_va, rkey, swap, comp)
 *   FETCH_ADD           0x14  ackreq 1, AtomicETH(remote_va, rkey, swap, comp)
 *   ACK                 0x11  AETH(code ACK, value 31 = CREDIT_CNT_INVALID, msn)
 *   RNR_NAK             0x11  AETH(code RNR, value imm & 31 (min RNR timer), msn)
 *   NAK                 0x11  AETH(code NAK, value imm & 31: 0 sequence error, 1
 *                             invalid request, 2 remote access, 3 remote op, msn)
 *   ATOMIC_ACK          0x12  AETH(ACK, 31, msn), AtomicAckETH(orig = swap)
 * (PSN = psn, no solicited bit.)  A batch may mix every op: data and
 * header-only packets of one call are built by ONE segmentation launch.
 *
 * Output: packet p (WR order, packet order) is the wire frame at
 * frames + p * slot_bytes, lens[p] bytes long (0 with status
 * RICRC_PKT_SEG_BAD when its WR is invalid).  Slot bytes past the frame end
 * are written as zeros up to the end of the frame's last 16*G-byte run (G =
 * lanes per packet: the next 128-byte boundary at 8 lanes; at least the next
 * 16-byte boundary), never past the slot; later slot bytes are left as they
 * were.
 */
#define RICRC_SEG_SEND 0
#define RICRC_SEG_SEND_WITH_IMM 1
#define RICRC_SEG_SEND_WITH_INV 2
#define RICRC_SEG_RDMA_WRITE 3
#define RICRC_SEG_RDMA_WRITE_WITH_IMM 4
#define RICRC_SEG_READ_RESPONSE 5
#define RICRC_SEG_READ_REQUEST 6
#define RICRC_SEG_COMPARE_SWAP 7
#define RICRC_SEG_FETCH_ADD 8
#define RICRC_SEG_ACK 9
#define RICRC_SEG_RNR_NAK 10
#define RICRC_SEG_NAK 11
#define RICRC_SEG_ATOMIC_ACK 12
#define RICRC_SEG_NUM_OPS 13
#define RICRC_SEG_SIGNALED 0x1  /* SEND_FLAGS.SIGNALED (src/roce_sq.py:1256)  */
#define RICRC_SEG_SOLICITED 0x2 /* SEND_FLAGS.SOLICITED (src/roce_sq.py:1257) */
#define RICRC_PKT_SEG_BAD 0x20  /* WR op unknown, MR range out of bounds, or packet not covered */

typedef struct ricrc_seg_wr {
  uint64_t mr_offset; /* message start: byte offset into the MR buffer (any alignment) */
  uint64_t remote_va; /* RETH.va (RDMA WRITE, READ_REQUEST), AtomicETH.va             */
  uint64_t swap;      /* AtomicETH.swap; AtomicAckETH.orig (ATOMIC_ACK)               */
  uint64_t comp;      /* AtomicETH.comp (compare value / FETCH_ADD addend)            */
  uint32_t length;    /* message bytes; 0 = one packet without payload                */
  uint32_t psn;       /* PSN of the first packet (24 bits)                            */
  uint32_t dqpn;      /* BTH.dqpn (24 bits)                                           */
  uint32_t src_ip;    /* IPv4 source as an integer (10.1.1.48 = 0x0A010130)           */
  uint32_t dst_ip;    /* IPv4 destination                                             */
  uint32_t rkey;      /* RETH.rkey, AtomicETH.rkey                                    */
  uint32_t imm;       /* ImmDt.data (*_WITH_IMM), IETH.rkey (SEND_WITH_INV), AETH
                         value (RNR_NAK, NAK)                                         */
  uint32_t msn;       /* AETH.msn (READ_RESPONSE, ACK, NAKs, ATOMIC_ACK; 24 bits)     */
  uint16_t sport;     /* UDP source port = the sender's QPN (src/roce_sq.py:1191)     */
  uint8_t op;         /* RICRC_SEG_*                                                  */
  uint8_t flags;      /* RICRC_SEG_SIGNALED | RICRC_SEG_SOLICITED                     */
  uint32_t first_pkt; /* index of the WR's first packet; set by ricrc_segment_plan    */
  uint32_t reserved[2];
} ricrc_seg_wr; /* 80 bytes */

/* Host-only planning (no GPU): checks every WR's op, fills wrs[i].first_pkt
 * with the running packet count, returns the total packets and the slot size
 * (the largest frame for `pmtu`, rounded up to 128 bytes).  pmtu: 256, 512,
 * 1024, 2048 or 4096 (IB MTU). */
int ricrc_segment_plan(ricrc_seg_wr* wrs, uint32_t nwr, uint32_t pmtu, uint32_t* npkts_out,
                       uint32_t* slot_bytes_out);
/* Host buffers, synchronous: MR copied to the device, frames built and
 * ICRC'd there, frames/lens/ICRCs copied back.  `wrs` must be planned.
 * frames_bytes >= npkts * slot_bytes. */
int ricrc_segment(ricrc_ctx* ctx, const uint8_t* mr, size_t mr_bytes, const ricrc_seg_wr* wrs,
                  uint32_t nwr, uint32_t pmtu, uint8_t* frames, size_t frames_bytes,
                  uint32_t* lens, uint32_t* icrc_out /* nullable */,
                  uint8_t* status_out /* nullable */);
/* Device-resident, asynchronous on `stream`: d_mr (mr_bytes) and d_wrs
 * (planned on the host, then copied) are device pointers; frames go to
 * d_frames + p * slot_bytes (slot_bytes: multiple of 128, >= the plan's;
 * d_frames 256-byte aligned).  d_lens doubles as the packet -> WR map while
 * the call runs.  WRs are validated on the device (status RICRC_PKT_SEG_BAD,
 * length 0).  No byte outside [d_mr, d_mr + mr_bytes) is read, except that an
 * MR shorter than 16 bytes must be readable for 16 when some packet carries
 * payload (a batch of header-only ops and empty messages may pass d_mr NULL). */
int ricrc_segment_dev(ricrc_ctx* ctx, const uint8_t* d_mr, uint64_t mr_bytes,
                      const ricrc_seg_wr* d_wrs, uint32_t nwr, uint32_t pmtu, uint32_t npkts,
                      uint8_t* d_frames, uint32_t slot_bytes, uint32_t* d_lens,
                      uint32_t* d_icrc /* nullable */, uint8_t* d_status /* nullable */,
                      void* stream);

/* ---- ICRC fault injection -------------------------------------------------
 *
 *   reference                                        replaced by
 *   -----------------------------------------------  -----------------------------
 *   hook functions  src/hooks.py:10-138, registered  ricrc_inject_faults_dev: the
 *     by SideServicer.SetHook src/sanity_side.py:     ICRC error case the reference
 *     345-364 (they edit BTH/RETH/AETH/payload of     lacks, for whole batches;
 *     one packet before it is built)                  roce_icrc.hooks for one packet
 *
 * Corrupts, in place, the frames of a seed-determined subset of a batch:
 * packet i is hit when splitmix64(seed ^ i * 0xD1B54A32D192ED03) mod 10^6 <
 * rate_ppm, with one of the kinds enabled in `kinds` (drawn from the same
 * hash).  d_fault_out[i] = the kind applied, 0 for none (frames that are not
 * well-formed IPv4 are never hit).  Expected verify outcome: ok unless the
 * kind is ICRC or PAYLOAD. */
#define RICRC_FAULT_ICRC 0x1    /* flip one bit of the 4-byte ICRC trailer             */
#define RICRC_FAULT_PAYLOAD 0x2 /* flip one bit of a covered byte the ICRC does not mask */
#define RICRC_FAULT_MASKED 0x4  /* randomise IP tos/ttl/checksum, UDP checksum, BTH
                                   fecn|becn|resv6: the ICRC must not change         */
int ricrc_inject_faults_dev(ricrc_ctx* ctx, uint8_t* d_frames, const uint64_t* d_offsets,
                            const uint32_t* d_lens, uint32_t n, uint64_t seed, uint32_t rate_ppm,
                            uint32_t kinds, uint8_t* d_fault_out /* nullable */, void* stream);

/* ---- measurement -------------------------------------------------------- */
/* STREAM-style copy of `bytes` (multiple of 16) from d_src to d_dst with
 * 16-B loads and stores: the read+write denominator of the segmentation
 * roofline. */
int ricrc_stream_copy_dev(ricrc_ctx* ctx, const uint8_t* d_src, uint8_t* d_dst, uint64_t bytes,
                          void* stream);
/* STREAM-style read of `bytes` (multiple of 16) from d_buf with 16-B coalesced
 * loads, XOR-folded into d_sink[0]: the HBM-read denominator for the roofline. */
int ricrc_stream_read_dev(ricrc_ctx* ctx, const uint8_t* d_buf, uint64_t bytes,
                          uint32_t* d_sink, void* stream);
/* Timing of the last request the per-packet service answered: out3[0] / [1] =
 * the GPU's 100 MHz real-time counter when the wave saw it / when its result
 * was written (so (out3[1] - out3[0]) * 10 ns is the GPU-side time),
 * out3[2] = the wave's polls of the request slot before it saw it. */
int ricrc_ctx_service_times(ricrc_ctx* ctx, uint64_t* out3);
/* Lanes per packet the engine would use for frames of `len` bytes (1 for the
 * lane-per-packet kernel of small strided frames). */
int ricrc_lanes_for_len(ricrc_ctx* ctx, uint32_t len);

#ifdef __cplusplus
}
#endif

#endif /* ROCE_ICRC_H */
