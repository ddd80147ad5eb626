/* Per-call latency of the host entry points from C (no Python): what a
 * cgo / JNI / N-API binding of include/roce_icrc.h sees.  ricrc_compute_one
 * (the per-packet drop-in of BTH.compute_icrc, src/roce.py:192) and small
 * ricrc_compute_batch bursts, with the resident service and with one kernel
 * launch per call, and the context-free ricrc_icrc; every service answer is
 * compared with the launch path's.
 *
 * build (from the repo root, after make -C roce-sim_amd):
 *   gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lroce-sim_amd/roce_icrc \
 *       -l:libroceicrc.so -Wl,-rpath,$PWD/roce-sim_amd/roce_icrc -o /tmp/latency_c
 * output: one JSON line per case (median and p99 in microseconds). */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "roce_icrc.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

/* An IPv4/UDP/BTH frame of `len` bytes (RC SEND_MIDDLE, payload from `seed`;
 * the trailer slot left zero): what the engine folds, as scapy builds it. */
static void make_frame(uint8_t* f, uint32_t len, uint32_t seed) {
  memset(f, 0, len);
  f[0] = 0x45;
  f[2] = (uint8_t)(len >> 8);
  f[3] = (uint8_t)len;
  f[5] = 1;     /* id 1 */
  f[8] = 64;    /* ttl */
  f[9] = 17;    /* UDP */
  f[12] = 10, f[15] = 1, f[16] = 10, f[19] = 2;
  f[22] = 0x12, f[23] = 0xB7; /* dport 4791 */
  f[24] = (uint8_t)((len - 20) >> 8);
  f[25] = (uint8_t)(len - 20);
  f[28] = 0x01; /* SEND_MIDDLE */
  f[30] = 0xFF, f[31] = 0xFF;
  f[35] = 0x11;
  uint32_t x = seed * 2654435761u + 1u;
  for (uint32_t i = 40; i + 4 < len; ++i) {
    x = x * 1664525u + 1013904223u;
    f[i] = (uint8_t)(x >> 24);
  }
}

#define REPS 500

static void report(const char* call, const char* what, int n, uint32_t svc, double* t) {
  qsort(t, REPS, sizeof(double), cmp_d);
  printf("{\"call\": \"%s\", \"frames\": \"%s\", \"n\": %d, \"service_idle_us\": %u, "
         "\"median_us\": %.2f, \"p99_us\": %.2f}\n",
         call, what, n, svc, t[REPS / 2], t[REPS * 99 / 100]);
  fflush(stdout);
}

int main(void) {
  ricrc_ctx* ctx = NULL;
  int rc = ricrc_ctx_create(0, &ctx);
  if (rc != RICRC_OK) {
    printf("ricrc_ctx_create: %s\n", ricrc_strerror(rc));
    return 1;
  }
  static uint8_t buf[1 << 17];
  static double t[REPS];
  uint64_t offs[64];
  uint32_t lens[64], out[64], ref[64];
  uint8_t st[64];
  const uint32_t sizes[] = {44, 1068, 4140};
  const uint32_t svcs[] = {1000, 0};
  int bad = 0;
  for (int si = 0; si < 2; ++si) {
    ricrc_ctx_set_service(ctx, svcs[si]);
    for (int k = 0; k < 3; ++k) {
      make_frame(buf, sizes[k], 7u + k);
      uint32_t want = 0;
      ricrc_ctx_set_service(ctx, 0);
      ricrc_compute_one(ctx, buf, sizes[k], &want, NULL);
      ricrc_ctx_set_service(ctx, svcs[si]);
      for (int w = 0; w < 50; ++w) ricrc_compute_one(ctx, buf, sizes[k], out, st);
      for (int r = 0; r < REPS; ++r) {
        const double t0 = now_us();
        ricrc_compute_one(ctx, buf, sizes[k], out, st);
        t[r] = now_us() - t0;
        bad += out[0] != want;
      }
      char what[32];
      snprintf(what, sizeof what, "%u B", sizes[k]);
      report("compute_one", what, 1, svcs[si], t);
    }
    /* bursts: 4 and 16 mixed-MTU frames, 64 ACK-sized frames */
    const int ns[] = {4, 16, 64};
    for (int c = 0; c < 3; ++c) {
      const int n = ns[c];
      size_t pos = 0;
      for (int i = 0; i < n; ++i) {
        const uint32_t L = n == 64 ? 48u : 296u + 256u * ((i * 7u) % 16u);
        make_frame(buf + pos, L, 100u + i);
        offs[i] = pos;
        lens[i] = L;
        pos += (L + 3u) & ~3u;
      }
      ricrc_ctx_set_service(ctx, 0);
      ricrc_compute_batch(ctx, buf, pos, offs, lens, n, ref, NULL);
      ricrc_ctx_set_service(ctx, svcs[si]);
      for (int w = 0; w < 50; ++w) ricrc_compute_batch(ctx, buf, pos, offs, lens, n, out, st);
      for (int r = 0; r < REPS; ++r) {
        const double t0 = now_us();
        ricrc_compute_batch(ctx, buf, pos, offs, lens, n, out, st);
        t[r] = now_us() - t0;
        for (int i = 0; i < n; ++i) bad += out[i] != ref[i];
      }
      report("compute_batch", n == 64 ? "ACK (48 B)" : "mixed-MTU", n, svcs[si], t);
    }
  }
  /* the context-free call (a library-owned context of this thread) */
  for (int k = 0; k < 3; ++k) {
    make_frame(buf, sizes[k], 7u + k);
    uint32_t want = 0;
    ricrc_ctx_set_service(ctx, 0);
    ricrc_compute_one(ctx, buf, sizes[k], &want, NULL);
    for (int w = 0; w < 50; ++w) ricrc_icrc(buf, sizes[k], out, st);
    for (int r = 0; r < REPS; ++r) {
      const double t0 = now_us();
      ricrc_icrc(buf, sizes[k], out, st);
      t[r] = now_us() - t0;
      bad += out[0] != want;
    }
    char what[32];
    snprintf(what, sizeof what, "%u B", sizes[k]);
    report("icrc", what, 1, 1000, t);
  }
  ricrc_ctx_destroy(ctx);
  printf("{\"mismatches_vs_launch_path\": %d}\n", bad);
  return bad != 0;
}
