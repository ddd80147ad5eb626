/* A plain C99 consumer of include/roce_icrc.h: proves the header is valid C
 * and the library links without C++ or HIP headers on the caller's side.
 * Runs without a GPU (planning and argument checks only); prints one line. */
#include <stdio.h>
#include <string.h>

#include "roce_icrc.h"

int main(void) {
  if (ricrc_abi_version() != RICRC_ABI_VERSION) return 1;
  if (strcmp(ricrc_strerror(RICRC_EINVAL), "invalid argument") != 0) return 2;
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
  if (npkts != 4 || wrs[1].first_pkt != 3 || slot % 256 != 0) return 4;
  if (ricrc_segment_plan(wrs, 2, 1000, &npkts, &slot) != RICRC_EINVAL) return 5;
  ricrc_ctx* ctx = NULL;
  int rc = ricrc_ctx_create(0, &ctx);
  int ndev = -1;
  if (ricrc_device_count(&ndev) != RICRC_OK) return 6;
  if (ndev == 0 && (rc != RICRC_ENODEV || ctx != NULL)) return 7;
  if (ctx) ricrc_ctx_destroy(ctx);
  printf("abi %d ok: %u packets, slot %u, devices %d, ctx_create %d\n", ricrc_abi_version(),
         npkts, slot, ndev, rc);
  return 0;
}
