/* A plain C99 consumer of include/roce_icrc.h: proves the header is valid C
 * and the library links without C++ or HIP headers on the caller's side.
 * Without a GPU it runs planning and argument checks only; with one it also
 * drives the GPU path through the C ABI (per-packet drop-in with and without
 * a context, a ragged batch
 * in compute and verify mode, and -- with two or more devices -- the
 * round-robin multi-device split).  Prints one line; exit status != 0 names
 * the failed check. */
#include <stdio.h>
#include <string.h>

#include "roce_icrc.h"

/* The sim_send_success SEND_ONLY: ICRC 0x1BE21D75,
 * wire bytes 75 1d e2 1b at the end. */
static const uint8_t kFrame[48] = {
    0x45, 0x00, 0x00, 0x30, 0x00, 0x01, 0x00, 0x00, 0x40, 0x11, 0x64, 0x7c, 0x0a, 0x01, 0x01, 0x30,
    0x0a, 0x01, 0x01, 0x0f, 0x00, 0x02, 0x12, 0xb7, 0x00, 0x1c, 0xfc, 0x40, 0x04, 0x30, 0xff, 0xff,
    0x00, 0x00, 0x00, 0x11, 0x80, 0x00, 0x00, 0x00, 0xff, 0x00, 0x00, 0x00, 0x75, 0x1d, 0xe2, 0x1b};
#define kIcrc 0x1BE21D75u

static int gpu_leg(ricrc_ctx* ctx, int ndev) {
  uint32_t icrc = 0;
  uint8_t st = 0xFF;
  if (ricrc_compute_one(ctx, kFrame, sizeof kFrame, &icrc, &st) != RICRC_OK) return 20;
  if (icrc != kIcrc || st != 0) return 21;
  icrc = 0;
  st = 0xFF;
  if (ricrc_icrc(kFrame, sizeof kFrame, &icrc, &st) != RICRC_OK) return 29;  /* no context */
  if (icrc != kIcrc || st != 0) return 30;
  /* a ragged batch: the frame, a copy with one payload bit flipped, the frame
   * again at an offset 4 bytes further */
  uint8_t buf[160];
  memset(buf, 0, sizeof buf);
  memcpy(buf, kFrame, 48);
  memcpy(buf + 48, kFrame, 48);
  buf[48 + 40] ^= 0x01;
  memcpy(buf + 100, kFrame, 48);
  const uint64_t offs[3] = {0, 48, 100};
  const uint32_t lens[3] = {48, 48, 48};
  uint32_t out[3] = {0, 0, 0};
  uint8_t ok[3] = {9, 9, 9};
  if (ricrc_compute_batch(ctx, buf, sizeof buf, offs, lens, 3, out, NULL) != RICRC_OK) return 22;
  if (out[0] != kIcrc || out[2] != kIcrc || out[1] == kIcrc) return 23;
  if (ricrc_verify_batch(ctx, buf, sizeof buf, offs, lens, 3, ok, NULL, NULL) != RICRC_OK)
    return 24;
  if (ok[0] != 1 || ok[1] != 0 || ok[2] != 1) return 25;
  {  /* the receive-side split, one context named twice (any box) */
    ricrc_ctx* same[2] = {ctx, ctx};
    uint8_t okm[3] = {9, 9, 9};
    uint32_t mm[3] = {0, 0, 0};
    if (ricrc_verify_batch_multi(same, 2, buf, sizeof buf, offs, lens, 3, okm, mm, NULL) !=
        RICRC_OK)
      return 31;
    if (okm[0] != 1 || okm[1] != 0 || okm[2] != 1 || mm[0] != out[0] || mm[1] != out[1])
      return 32;
  }
  {  /* ABI 5: the ragged variant of a context; host batches of 3 frames go to
      * the resident wave, so the kernel path is forced with the service off */
    int v = -1;
    if (ricrc_ctx_set_ragged_variant(ctx, 3) != RICRC_EINVAL) return 33;
    if (ricrc_ctx_last_ragged_variant(ctx, &v) != RICRC_OK || v != RICRC_RAGGED_AUTO) return 34;
    if (ricrc_ctx_set_service(ctx, 0) != RICRC_OK) return 35;
    if (ricrc_ctx_set_ragged_variant(ctx, RICRC_RAGGED_COMPACT) != RICRC_OK) return 36;
    uint32_t vc[3] = {0, 0, 0};
    if (ricrc_compute_batch(ctx, buf, sizeof buf, offs, lens, 3, vc, NULL) != RICRC_OK) return 37;
    if (vc[0] != out[0] || vc[1] != out[1] || vc[2] != out[2]) return 38;
    if (ricrc_ctx_last_ragged_variant(ctx, &v) != RICRC_OK || v != RICRC_RAGGED_COMPACT) return 41;
    if (ricrc_ctx_set_ragged_variant(ctx, RICRC_RAGGED_AUTO) != RICRC_OK) return 39;
    if (ricrc_ctx_set_service(ctx, 1000) != RICRC_OK) return 40;
  }
  if (ndev >= 2) {
    ricrc_ctx* c2 = NULL;
    if (ricrc_ctx_create(1, &c2) != RICRC_OK) return 26;
    ricrc_ctx* ctxs[2] = {ctx, c2};
    uint32_t m[3] = {0, 0, 0};
    const int rc = ricrc_compute_batch_multi(ctxs, 2, buf, sizeof buf, offs, lens, 3, m, NULL);
    ricrc_ctx_destroy(c2);
    if (rc != RICRC_OK) return 27;
    if (m[0] != out[0] || m[1] != out[1] || m[2] != out[2]) return 28;
  }
  return 0;
}

int main(void) {
  if (ricrc_abi_version() != RICRC_ABI_VERSION) return 1;
  if (strcmp(ricrc_strerror(RICRC_EINVAL), "invalid argument") != 0) return 2;
  if (ricrc_ctx_set_ragged_variant(NULL, RICRC_RAGGED_COMPACT) != RICRC_EINVAL) return 9;
  /* Util.compute_wr_pkt_num (src/roce_util.py:183-185): a 10000-byte SEND at
   * PMTU 4096 is 3 packets, a zero-length one 1 packet */
  ricrc_seg_wr wrs[2];
  memset(wrs, 0, sizeof wrs);
  wrs[0].op = RICRC_SEG_SEND;
  wrs[0].length = 10000;
  wrs[1].op = RICRC_SEG_RDMA_WRITE;
  wrs[1].length = 0;
  uint32_t npkts = 0, slot = 0;
  if (ricrc_segment_plan(wrs, 2, 4096, &npkts, &slot) != RICRC_OK) return 3;
  if (npkts != 4 || wrs[1].first_pkt != 3 || slot % 128 != 0) return 4;
  if (ricrc_segment_plan(wrs, 2, 1000, &npkts, &slot) != RICRC_EINVAL) return 5;
  ricrc_ctx* ctx = NULL;
  int rc = ricrc_ctx_create(0, &ctx);
  int ndev = -1;
  if (ricrc_device_count(&ndev) != RICRC_OK) return 6;
  if (ndev == 0 && (rc != RICRC_ENODEV || ctx != NULL)) return 7;
  if (ndev == 0) {
    uint32_t icrc = 0;
    if (ricrc_icrc(kFrame, sizeof kFrame, &icrc, NULL) != RICRC_ENODEV) return 8;
  }
  int gpu = -1;
  if (ctx) {
    gpu = gpu_leg(ctx, ndev);
    ricrc_ctx_destroy(ctx);
    if (gpu) return gpu;
  }
  printf("abi %d ok: %u packets, slot %u, devices %d, ctx_create %d, gpu leg %s\n",
         ricrc_abi_version(), npkts, slot, ndev, rc,
         gpu == 0 ? (ndev >= 2 ? "ok (multi-device)" : "ok") : "skipped");
  return 0;
}
