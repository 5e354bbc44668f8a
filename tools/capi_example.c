/* Plain-C use of the libyoda C-ABI (what the cgo binding does), run on the GPU box:
 *   gcc -O2 -I include -o /tmp/capi_example tools/capi_example.c \
 *       -L kubernetes-scheduler_amd/yoda_amd -lyoda -Wl,-rpath,$PWD/kubernetes-scheduler_amd/yoda_amd
 * Evaluates KAT 1 of SURVEY.md §8c (pod number=2, memory=8000, clock=1500 over three nodes)
 * and checks pick = node 1, raw score 4061, maxima {1200,1500,108,16000,400,32000}. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "yoda.h"

#define K 4
int main(void) {
  yoda_t* h = NULL;
  int rc = yoda_create(0, &h);
  if (rc) {
    printf("yoda_create failed: %d\n", rc);
    return 1;
  }
  uint64_t card_number[3] = {2, 4, 1}, free_sum[3] = {19000, 64000, 20000},
           total_sum[3] = {32000, 128000, 20000}, alloc[3] = {0, 16000, 0};
  uint32_t card_count[3] = {2, 4, 1};
  uint64_t fr[3 * K] = {10000, 9000, 0, 0, 16000, 16000, 16000, 16000, 20000};
  uint64_t to[3 * K] = {16000, 16000, 0, 0, 32000, 32000, 32000, 32000, 20000};
  uint64_t ck[3 * K] = {1500, 1500, 0, 0, 1500, 1500, 1500, 1500, 1500};
  uint64_t bw[3 * K] = {900, 900, 0, 0, 1200, 1200, 1200, 1200, 900};
  uint64_t co[3 * K] = {80, 80, 0, 0, 108, 108, 108, 108, 80};
  uint64_t pw[3 * K] = {300, 300, 0, 0, 400, 400, 400, 400, 300};
  uint8_t he[3 * K] = {1, 1, 0, 0, 1, 1, 1, 0, 1};
  yoda_node_soa nodes = {3, K, card_number, card_count, free_sum, total_sum, alloc,
                         fr, to, ck, bw, co, pw, he, NULL, NULL};
  if ((rc = yoda_upload_nodes(h, &nodes, 0, 0))) {
    printf("upload_nodes: %d %s\n", rc, yoda_last_error(h));
    return 1;
  }
  uint8_t one = 1;
  uint64_t number = 2, memory = 8000, clock = 1500;
  yoda_pod_soa pods = {1, &one, &number, &one, &memory, &one, &clock, NULL, NULL, NULL};
  int32_t pick = -9, status = -9;
  uint32_t nf = 0, ties = 0;
  int64_t top = 0;
  uint64_t maxima[6];
  yoda_eval_out out = {&pick, &status, &nf, &ties, &top, maxima};
  if ((rc = yoda_eval(h, &pods, YODA_MODE_SCV, &out))) {
    printf("eval: %d %s\n", rc, yoda_last_error(h));
    return 1;
  }
  const uint64_t want_max[6] = {1200, 1500, 108, 16000, 400, 32000};
  int ok = pick == 1 && status == YODA_STATUS_OK && nf == 2 && ties == 1 && top == 4061 &&
           memcmp(maxima, want_max, sizeof(want_max)) == 0;
  int64_t scores[3];
  uint32_t bits[1];
  if ((rc = yoda_score_rows(h, YODA_MODE_SCV, bits, 1, scores, 3))) return 1;
  ok = ok && bits[0] == 3u && scores[0] == 1718 && scores[1] == 4061 && scores[2] == -1;
  printf("KAT1 via C-ABI: pick=%d status=%d n_feasible=%u ties=%u top=%lld rows=[%lld %lld %lld] %s\n",
         pick, status, nf, ties, (long long)top, (long long)scores[0], (long long)scores[1],
         (long long)scores[2], ok ? "OK" : "MISMATCH");
  yoda_destroy(h);
  return ok ? 0 : 1;
}
