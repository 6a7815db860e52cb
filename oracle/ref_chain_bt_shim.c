/* oracle/ref_chain_bt_shim.c -- TEST INFRASTRUCTURE ONLY.
 * Our own C entry point over the reference's UNMODIFIED minimap2-acceleration testbed
 * mm_chain_dp (tools/minimap2-acceleration/testbed/chain.c:25-219: chaining DP + backtrack +
 * reorder), compiled by oracle/Makefile with the testbed's misc.c (radix sorts) and kalloc.c into
 * oracle/_ref/libref_chain_bt.so. Pins oracle/chain_oracle.c's chain_oracle_backtrack. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "minimap.h"
#include "mmpriv.h"

/* One call: the DP computes avg_qspan itself (chain.c:40-41); max_iter 5000 and gap_scale 1 are
 * fixed in this version (chain.c:43-44). u_out gets the chains, bx/by the anchors (chain order).
 * Returns the chain count; *n_anchors = anchors written. */
int64_t ref_chain_dp_bt(int64_t n, int max_dist_x, int max_dist_y, int bw, int max_skip, int min_cnt, int min_sc,
                        int n_segs, const uint64_t *ax, const uint64_t *ay, uint64_t *u_out, uint64_t *bx,
                        uint64_t *by, int64_t *n_anchors) {
  *n_anchors = 0;
  if (n <= 0) return 0;
  mm128_t *a = (mm128_t *)malloc((size_t)n * sizeof(mm128_t));
  for (int64_t i = 0; i < n; i++) a[i].x = ax[i], a[i].y = ay[i];
  mm_mapopt_t opt;
  memset(&opt, 0, sizeof(opt));
  int n_u = 0;
  uint64_t *u = NULL;
  mm128_t *b = mm_chain_dp(max_dist_x, max_dist_y, bw, max_skip, min_cnt, min_sc, 0, n_segs, n, a, &n_u, &u, NULL,
                           &opt);
  int64_t k = 0;
  for (int i = 0; i < n_u; i++) {
    u_out[i] = u[i];
    for (int32_t q = 0; q < (int32_t)u[i]; q++, k++) bx[k] = b[k].x, by[k] = b[k].y;
  }
  *n_anchors = k;
  free(u);
  free(b);  /* mm_chain_dp frees `a` itself (kfree(km, a)) unless it returns early */
  return n_u;
}
