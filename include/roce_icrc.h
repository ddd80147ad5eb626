/*
 * roce_icrc.h -- C ABI of the MI355X (gfx950) RoCEv2 ICRC engine, libroceicrc.so.
 *
 * Drop-in boundary for datenlord/roce-sim's per-packet Invariant CRC:
 *
 *   reference                                   replaced by
 *   ------------------------------------------  ---------------------------------
 *   BTH.compute_icrc(self, p)  src/roce.py:192   ricrc_compute_one / ricrc_compute_batch
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
 * UDP (protocol != 17), shorter than IP+UDP+BTH+ICRC, longer than 65535 bytes
 * or not a multiple of 4 bytes long gets ICRC 0 and a status bit -- the
 * reference's "warning + ICRC 00000000" path (src/roce.py:195-200, 220-223).
 * These are not call errors: the batch call still returns RICRC_OK.
 *
 * Ownership.  The caller owns every buffer.  No pointer is retained after a
 * synchronous call returns; the *_dev variants are asynchronous on `stream`
 * and use their arguments until that stream has executed the work.
 *
 * Threading.  All entry points are re-entrant.  A ricrc_ctx owns one HIP
 * stream plus device scratch and is NOT thread-safe: use one context per host
 * thread (the reference calls from a 10-thread gRPC pool,
 * src/sanity_side.py:383).  Python's ctypes releases the GIL around calls.
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

#define RICRC_ABI_VERSION 1

/* call-level return codes */
#define RICRC_OK 0
#define RICRC_EINVAL (-22) /* bad argument (null pointer, n too large, ...) */
#define RICRC_ENOMEM (-12) /* host or device allocation failed              */
#define RICRC_ENODEV (-19) /* no usable gfx950 device / device index        */
#define RICRC_EIO (-5)     /* HIP runtime or kernel launch failure          */

/* per-packet status bits (status_out[i]) */
#define RICRC_PKT_BAD_LEN 0x01       /* len % 4, too short, or > 65535            */
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
/* Lanes cooperating on one packet (1,2,4,...,64); 0 = automatic by length. */
int ricrc_ctx_set_lanes_per_packet(ricrc_ctx* ctx, int lanes);
/* The hipStream_t the synchronous host-buffer calls run on. */
void* ricrc_ctx_stream(ricrc_ctx* ctx);

/* ---- host buffers, synchronous (H2D + kernel + D2H) --------------------- */
/* The per-packet drop-in for BTH.compute_icrc (src/roce.py:192): one wire
 * frame in, its ICRC out (runs on the GPU through the context's scratch). */
int ricrc_compute_one(ricrc_ctx* ctx, const uint8_t* frame, size_t len, uint32_t* icrc_out,
                      uint8_t* status_out /* nullable */);

/* Ragged batch: frame i is frames[offsets[i] .. offsets[i] + lens[i]).
 * `frames_bytes` is the size of the `frames` buffer (bounds for the copy). */
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
 * ctxs[i % nctx]; host threads gather, copy, launch and scatter per device. */
int ricrc_compute_batch_multi(ricrc_ctx** ctxs, int nctx, const uint8_t* frames,
                              size_t frames_bytes, const uint64_t* offsets,
                              const uint32_t* lens, uint32_t n, uint32_t* icrc_out,
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

/* ---- measurement -------------------------------------------------------- */
/* STREAM-style read of `bytes` (multiple of 16) from d_buf with 16-B coalesced
 * loads, XOR-folded into d_sink[0]: the HBM-read denominator for the roofline. */
int ricrc_stream_read_dev(ricrc_ctx* ctx, const uint8_t* d_buf, uint64_t bytes,
                          uint32_t* d_sink, void* stream);
/* Lanes per packet the engine would use for frames of `len` bytes. */
int ricrc_lanes_for_len(ricrc_ctx* ctx, uint32_t len);

#ifdef __cplusplus
}
#endif

#endif /* ROCE_ICRC_H */
