/*
 * CPU oracle for the RoCEv2 ICRC -- TEST INFRASTRUCTURE ONLY.
 *
 * Linked/loaded only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, as the checker and the CPU baseline.  Never part of the
 * product library (roce-sim_amd/ -> libroceicrc.so).
 *
 * Restates BTH.compute_icrc (datenlord/roce-sim src/roce.py:192-223):
 *   icrc = zlib.crc32(FF x 8 || masked frame[0 : len-4])
 * with the masks of src/roce.py:204-211 (IP tos/ttl/chksum, UDP chksum,
 * BTH byte 4 = fecn|becn|resv6) and the little-endian wire encoding of
 * src/roce.py:187-190.  Two independent evaluations of the same rule:
 *
 *   oracle_icrc_bitwise  -- reflected CRC-32 (poly 0xEDB88320) bit by bit from
 *                           the register 0xDEBB20E3 that the FF x 8 prefix leaves
 *                           (no tables; Linux rxe uses the same seed).
 *   oracle_icrc_batch    -- slice-by-8 tables, init 0xFFFFFFFF over the literal
 *                           FF x 8 prefix (zlib's formulation), pthreads over
 *                           packets.  Used to check full-size GPU batches and as
 *                           the multi-core "port" CPU baseline.
 *
 * Non-IPv4 / non-UDP / too-short frames give ICRC 0 (the reference's warning
 * path, src/roce.py:195-200, 220-223).  See oracle/icrc_oracle.py for the
 * parity-pinning status.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define POLY 0xEDB88320u

static uint32_t T8[8][256];
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t r = b;
    for (int i = 0; i < 8; ++i) r = (r >> 1) ^ ((r & 1) ? POLY : 0);
    T8[0][b] = r;
  }
  for (int k = 1; k < 8; ++k)
    for (uint32_t b = 0; b < 256; ++b)
      T8[k][b] = (T8[k - 1][b] >> 8) ^ T8[0][T8[k - 1][b] & 0xFF];
}

/* Returns the offset of the UDP header, or -1 when the frame is not a
 * CRC-able IPv4/UDP/BTH frame (reference: warning + ICRC 0). */
static int frame_layout(const uint8_t* f, size_t len) {
  if (len < 20 || (f[0] >> 4) != 4) return -1;
  int ihl = f[0] & 0xF;
  if (ihl < 5 || f[9] != 17) return -1;
  if (len < (size_t)(4 * ihl + 8 + 12 + 4)) return -1;
  return 4 * ihl;
}

static inline uint8_t masked_byte(const uint8_t* f, size_t i, int udp) {
  if (i == 1 || i == 8 || i == 10 || i == 11) return 0xFF;
  if (i == (size_t)udp + 6 || i == (size_t)udp + 7) return 0xFF;
  if (i == (size_t)udp + 12) return 0xFF;
  return f[i];
}

uint32_t oracle_icrc_bitwise(const uint8_t* frame, size_t len) {
  int udp = frame_layout(frame, len);
  if (udp < 0) return 0;
  uint32_t r = 0xDEBB20E3u;
  for (size_t i = 0; i < len - 4; ++i) {
    r ^= masked_byte(frame, i, udp);
    for (int b = 0; b < 8; ++b) r = (r >> 1) ^ ((r & 1) ? POLY : 0);
  }
  return r ^ 0xFFFFFFFFu;
}

static uint32_t crc_update_bytes(uint32_t r, const uint8_t* p, size_t n) {
  while (n && ((uintptr_t)p & 7)) {
    r = T8[0][(r ^ *p++) & 0xFF] ^ (r >> 8);
    --n;
  }
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= r;
    r = T8[7][lo & 0xFF] ^ T8[6][(lo >> 8) & 0xFF] ^ T8[5][(lo >> 16) & 0xFF] ^
        T8[4][lo >> 24] ^ T8[3][hi & 0xFF] ^ T8[2][(hi >> 8) & 0xFF] ^
        T8[1][(hi >> 16) & 0xFF] ^ T8[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) r = T8[0][(r ^ *p++) & 0xFF] ^ (r >> 8);
  return r;
}

uint32_t oracle_icrc_sliced(const uint8_t* frame, size_t len) {
  pthread_once(&tables_once, build_tables);
  int udp = frame_layout(frame, len);
  if (udp < 0) return 0;
  /* zlib formulation: init 0xFFFFFFFF, the 8 x 0xFF prefix, the masked header,
   * then the rest of the frame as is, final xor. */
  uint8_t head[96];
  size_t hlen = (size_t)udp + 8 + 12; /* IP + UDP + BTH */
  for (size_t i = 0; i < hlen; ++i) head[i] = masked_byte(frame, i, udp);
  static const uint8_t ff8[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};
  uint32_t r = 0xFFFFFFFFu;
  r = crc_update_bytes(r, ff8, 8);
  r = crc_update_bytes(r, head, hlen);
  r = crc_update_bytes(r, frame + hlen, len - 4 - hlen);
  return r ^ 0xFFFFFFFFu;
}

typedef struct {
  const uint8_t* base;
  const uint64_t* offs;
  const uint32_t* lens;
  uint64_t stride;
  uint32_t len;
  uint64_t begin, end;
  uint32_t* out;
  uint8_t* ok;
} job_t;

static void* run_job(void* arg) {
  job_t* j = (job_t*)arg;
  for (uint64_t i = j->begin; i < j->end; ++i) {
    uint64_t off = j->offs ? j->offs[i] : i * j->stride;
    uint32_t len = j->lens ? j->lens[i] : j->len;
    const uint8_t* f = j->base + off;
    uint32_t c = oracle_icrc_sliced(f, len);
    if (j->out) j->out[i] = c;
    if (j->ok) {
      uint32_t t;
      memcpy(&t, f + len - 4, 4);
      j->ok[i] = (uint8_t)(frame_layout(f, len) >= 0 && t == c);
    }
  }
  return NULL;
}

/* Batch over frames at base+offs[i] (or base+i*stride when offs == NULL) with
 * length lens[i] (or len).  out and/or ok may be NULL. */
int oracle_icrc_batch(const uint8_t* base, const uint64_t* offs, const uint32_t* lens,
                      uint64_t stride, uint32_t len, uint64_t n, uint32_t* out, uint8_t* ok,
                      int nthreads) {
  pthread_once(&tables_once, build_tables);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  pthread_t th[256];
  job_t jobs[256];
  uint64_t per = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (job_t){base, offs, lens, stride, len, t * per, (t + 1) * per, out, ok};
    if (jobs[t].begin > n) jobs[t].begin = n;
    if (jobs[t].end > n) jobs[t].end = n;
  }
  for (int t = 1; t < nthreads; ++t)
    if (pthread_create(&th[t], NULL, run_job, &jobs[t]) != 0) return -1;
  run_job(&jobs[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}
