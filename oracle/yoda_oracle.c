/*
 * yoda_oracle.c — CPU restatement of the reference Yoda Filter/Score/select semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or the timed CPU
 * baseline).  The product path (libyoda, kubernetes-scheduler_amd/) never links or calls it.
 *
 * PARITY STATUS: parity unpinned by reference fixtures.  The reference
 * (Mr-LvGJ/kubernetes-scheduler, pure Go) holds no golden vectors or value-asserting tests
 * (SURVEY.md §4, §8c), and it cannot be built here (no Go toolchain; its deps
 * k8s.io/kubernetes v1.22.3 and NJUPT-ISL/SCV @46b36eeed646 are not vendored).  This file is
 * pinned instead by the known-answer tests hand-derived from the Go text (SURVEY.md §8c,
 * tests/test_oracle.py) and cross-checked against an independent pure-Python restatement
 * (oracle/pyoracle.py) on randomized clusters.
 *
 * Arithmetic follows Go on GOARCH=amd64 (reference Makefile:4): `uint` is uint64 with
 * wrap-around, integer division truncates, float64 ops are IEEE round-to-nearest with NO
 * fused multiply-add (build with -ffp-contract=off).
 *
 * Every function cites the reference file:line it restates.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/yoda.h"

#define GO_INT64_MAX 9223372036854775807LL

/* MaxValue — pkg/yoda/collection/collection.go:14-21 */
typedef struct {
  uint64_t bandwidth, clock, core, free_memory, power, total_memory;
} max_value;

/* score weights — pkg/yoda/score/algorithm.go:24-35 */
enum {
  W_BANDWIDTH = 1,
  W_CLOCK = 1,
  W_CORE = 2,
  W_POWER = 1,
  W_FREE_MEMORY = 3,
  W_TOTAL_MEMORY = 1,
  W_ACTUAL = 2,
  W_ALLOCATE = 3
};

typedef struct {
  uint64_t free_memory, total_memory, clock, bandwidth, core, power;
  int healthy;
} card_t;

static card_t get_card(const yoda_node_soa* nd, uint32_t n, uint32_t j) {
  size_t k = (size_t)n * nd->max_cards + j;
  card_t c;
  c.free_memory = nd->card_free_memory[k];
  c.total_memory = nd->card_total_memory[k];
  c.clock = nd->card_clock[k];
  c.bandwidth = nd->card_bandwidth[k];
  c.core = nd->card_core[k];
  c.power = nd->card_power[k];
  c.healthy = nd->card_healthy[k] != 0;
  return c;
}

/* CardFitsMemory — filter.go:52-54 */
static int card_fits_memory(uint64_t memory, const card_t* c) {
  return c->healthy && c->free_memory >= memory;
}

/* CardFitsClock — filter.go:56-58 (equality, not >=) */
static int card_fits_clock(uint64_t clock, const card_t* c) {
  return c->healthy && c->clock == clock;
}

/* PodFitsNumber — filter.go:11-16 */
static int pod_fits_number(const yoda_pod_soa* pd, uint32_t p, const yoda_node_soa* nd,
                           uint32_t n, uint64_t* number) {
  if (pd->has_number[p]) {
    *number = pd->number[p];
    return pd->number[p] <= nd->card_number[n];
  }
  *number = 1;
  return nd->card_number[n] > 0;
}

/* PodFitsMemory — filter.go:18-33 */
static int pod_fits_memory(uint64_t number, const yoda_pod_soa* pd, uint32_t p,
                           const yoda_node_soa* nd, uint32_t n, uint64_t* memory) {
  if (pd->has_memory[p]) {
    uint64_t fits = 0, m = pd->memory[p];
    for (uint32_t j = 0; j < nd->card_count[n]; ++j) {
      card_t c = get_card(nd, n, j);
      if (card_fits_memory(m, &c)) fits++;
    }
    *memory = m;
    return fits >= number;
  }
  *memory = 0;
  return 1;
}

/* PodFitsClock — filter.go:35-50 */
static int pod_fits_clock(uint64_t number, const yoda_pod_soa* pd, uint32_t p,
                          const yoda_node_soa* nd, uint32_t n, uint64_t* clock) {
  if (pd->has_clock[p]) {
    uint64_t fits = 0, c = pd->clock[p];
    for (uint32_t j = 0; j < nd->card_count[n]; ++j) {
      card_t cd = get_card(nd, n, j);
      if (card_fits_clock(c, &cd)) fits++;
    }
    *clock = c;
    return fits >= number;
  }
  *clock = 0;
  return 1;
}

/* The gating sequence of collection.go:41-44 (= algorithm.go:266-269): the Mode-A Filter.
 * Returns feasibility and the (memory, clock) thresholds of the card predicate. */
static int pod_fits_node(const yoda_pod_soa* pd, uint32_t p, const yoda_node_soa* nd, uint32_t n,
                         uint64_t* memory, uint64_t* clock) {
  uint64_t number;
  if (!pod_fits_number(pd, p, nd, n, &number)) return 0;
  int fm = pod_fits_memory(number, pd, p, nd, n, memory);
  int fc = pod_fits_clock(number, pd, p, nd, n, clock);
  return fc && fm;
}

/* ProcessMaxValueWithCard — collection.go:57-76 */
static void process_max_value_with_card(const card_t* c, max_value* v) {
  if (c->free_memory > v->free_memory) v->free_memory = c->free_memory;
  if (c->clock > v->clock) v->clock = c->clock;
  if (c->total_memory > v->total_memory) v->total_memory = c->total_memory;
  if (c->bandwidth > v->bandwidth) v->bandwidth = c->bandwidth;
  if (c->core > v->core) v->core = c->core;
  if (c->power > v->power) v->power = c->power;
}

/* CollectMaxValues — collection.go:30-55: floor 1 (:31-38), every SCV re-filtered
 * (:41-44), card predicate WITHOUT a health check and with >= clock (:46). */
static max_value collect_max_values(const yoda_pod_soa* pd, uint32_t p, const yoda_node_soa* nd) {
  max_value v = {1, 1, 1, 1, 1, 1};
  for (uint32_t n = 0; n < nd->n_nodes; ++n) {
    uint64_t memory, clock;
    if (!pod_fits_node(pd, p, nd, n, &memory, &clock)) continue;
    for (uint32_t j = 0; j < nd->card_count[n]; ++j) {
      card_t c = get_card(nd, n, j);
      if (c.free_memory >= memory && c.clock >= clock) process_max_value_with_card(&c, &v);
    }
  }
  return v;
}

/* CalculateCardScore — algorithm.go:280-291 (commented in the fork).  Note the quirk at
 * :283: clock is divided by MaxBandwidth.  uint64 wrap-around on every product. */
static uint64_t card_score(const max_value* v, const card_t* c) {
  uint64_t bandwidth = c->bandwidth * 100u / v->bandwidth;
  uint64_t clock = c->clock * 100u / v->bandwidth;
  uint64_t core = c->core * 100u / v->core;
  uint64_t power = c->power * 100u / v->power;
  uint64_t free_memory = c->free_memory * 100u / v->free_memory;
  uint64_t total_memory = c->total_memory * 100u / v->total_memory;
  return (bandwidth * W_BANDWIDTH + clock * W_CLOCK + core * W_CORE + power * W_POWER) +
         free_memory * W_FREE_MEMORY + total_memory * W_TOTAL_MEMORY;
}

/* CalculateBasicScore — algorithm.go:264-278 */
static uint64_t basic_score(const max_value* v, const yoda_pod_soa* pd, uint32_t p,
                            const yoda_node_soa* nd, uint32_t n) {
  uint64_t s = 0, memory, clock;
  if (pod_fits_node(pd, p, nd, n, &memory, &clock)) {
    for (uint32_t j = 0; j < nd->card_count[n]; ++j) {
      card_t c = get_card(nd, n, j);
      if (c.free_memory >= memory && c.clock >= clock) s += card_score(v, &c);
    }
  }
  return s;
}

/* CalculateActualScore — algorithm.go:293-295.  TotalMemorySum == 0 panics in Go. */
static uint64_t actual_score(const yoda_node_soa* nd, uint32_t n, int* div_zero) {
  uint64_t total = nd->total_memory_sum[n];
  if (total == 0) {
    *div_zero = 1;
    return 0;
  }
  return (nd->free_memory_sum[n] * 100u / total) * W_ACTUAL;
}

static uint64_t node_alloc(const yoda_node_soa* nd, uint32_t n) {
  return nd->alloc_memory ? nd->alloc_memory[n] : 0;
}

/* CalculateAllocateScore — algorithm.go:297-310 (alloc = Σ scv/memory of assigned pods,
 * :299-303, carried in alloc_memory). */
static uint64_t allocate_score(const yoda_node_soa* nd, uint32_t n, int* div_zero) {
  uint64_t total = nd->total_memory_sum[n], alloc = node_alloc(nd, n);
  if (total < alloc) return 0;
  if (total == 0) {
    *div_zero = 1;
    return 0;
  }
  return (total - alloc) * 100u / total * W_ALLOCATE;
}

/* Uint64ToInt64 — filter.go:84-86: FormatUint then Atoi; Atoi fails (-> 0) above MaxInt64. */
static int64_t uint64_to_int64(uint64_t u) {
  return u > (uint64_t)GO_INT64_MAX ? 0 : (int64_t)u;
}

/* amd64 CVTTSD2SQ: truncation, 0x8000000000000000 for NaN / out of range. */
static int64_t cvttsd2sq(double x) {
  if (isnan(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return INT64_MIN;
  return (int64_t)x;
}

/* Go's float64 -> uint64 conversion on amd64 (cmd/compile ssagen float64ToUint64). */
static uint64_t go_float64_to_uint64(double x) {
  const double cutoff = 9223372036854775808.0;
  if (x < cutoff) return (uint64_t)cvttsd2sq(x);
  double y = x - cutoff;
  return (uint64_t)cvttsd2sq(y) | 0x8000000000000000ull;
}

/* BalancedCpuDiskIOPriority — algorithm.go:99-119 for one (pod, node): the value returned
 * for the node being scored (:112-113), then Uint64ToInt64 (scheduler.go:154).
 * V = Cpu/100 (:73) and U = DiskIO/50 (:71) round-trip Redis exactly (go-redis formats
 * float64 with the shortest exact representation). */
static int64_t diskio_score(const yoda_pod_soa* pd, uint32_t p, const yoda_node_soa* nd, uint32_t n) {
  double rio = pd->rio[p];
  double rcpu = (double)pd->rcpu[p];
  double beta = 1.0 / (1.0 + rcpu / rio); /* :105 */
  double alpha = 1 - beta;                /* :106 */
  double v = nd->cpu[n] / 100.0;
  double u = nd->disk_io[n] / 50.0;
  double a = alpha * v;
  double b = beta * u;
  double l = fabs(a - b);        /* :110 */
  double t = 10.0 * l;
  double s = 10.0 - t;           /* :111 */
  return uint64_to_int64(go_float64_to_uint64(s));
}

/* B3 documentation mode — the Redis memo quirk of CalculateScore (algorithm.go:57-63,116,
 * SURVEY §8a B3).  Within one cycle (NormalizeScore flushes the DB, scheduler.go:160) the
 * first Score call misses "S-<node>", computes every node's S and stores it (:116); it
 * returns uint64(S) for its own node.  Every later call returns StrToUint64 (filter.go:67-73)
 * of the stored string: go-redis writes a float64 as FormatFloat(S, 'f', -1, 64), so Atoi
 * accepts it only when S is finite and integral; a negative integer wraps in uint64() and
 * then fails Uint64ToInt64 (scheduler.go:154); so the node scores S if S is a non-negative
 * integer, else 0.  Which call runs first depends on goroutine order: `first` fixes it. */
static int64_t diskio_score_memo(const yoda_pod_soa* pd, uint32_t p, const yoda_node_soa* nd,
                                 uint32_t n, int64_t first) {
  if ((int64_t)n == first) return diskio_score(pd, p, nd, n);
  double rio = pd->rio[p];
  double rcpu = (double)pd->rcpu[p];
  double beta = 1.0 / (1.0 + rcpu / rio);
  double alpha = 1 - beta;
  double v = nd->cpu[n] / 100.0;
  double u = nd->disk_io[n] / 50.0;
  double a = alpha * v;
  double b = beta * u;
  double s = 10.0 - 10.0 * fabs(a - b);
  if (!isfinite(s) || s != trunc(s)) return 0;           /* "NaN", "+Inf", "9.5": Atoi fails */
  if (s < 0 || s >= 9223372036854775808.0) return 0;     /* wraps / out of Atoi range -> 0 */
  return (int64_t)s;
}

/* Per-pod result of one scheduling cycle. */
typedef struct {
  int32_t pick, status;
  uint32_t n_feasible, n_ties;
  int64_t top_score;
  max_value maxima;
} cycle_result;

/* One kube-scheduler v1.22.3 cycle with only the yoda plugin scoring:
 *   Filter over all nodes (percentageOfNodesToScore 100) -> 0 feasible: Unschedulable;
 *   1 feasible: returned without PreScore/Score (generic_scheduler.go "only one node");
 *   else PreScore (CollectMaxValues), Score per feasible node, NormalizeScore
 *   (scheduler.go:158-183), range check [0,100] (framework RunScorePlugins), weight 1,
 *   selectHost.  selectHost breaks ties at random (rand.Intn); this restatement returns
 *   the LOWEST node index of the tie set and reports the tie set's size.
 * scratch: >= 2*N int64 + N uint32. */
static void schedule_one(const yoda_node_soa* nd, const yoda_pod_soa* pd, uint32_t p, int mode,
                         int64_t memo_first, int64_t* scores, uint32_t* feas, cycle_result* r) {
  uint32_t nf = 0;
  max_value mv = {1, 1, 1, 1, 1, 1};
  memset(r, 0, sizeof(*r));
  r->top_score = 0;
  for (uint32_t n = 0; n < nd->n_nodes; ++n) {
    uint64_t m, c;
    int ok = (mode == YODA_MODE_DISKIO) ? 1 /* Yoda.Filter pass-through, scheduler.go:96-99 */
                                        : pod_fits_node(pd, p, nd, n, &m, &c);
    if (ok) feas[nf++] = n;
  }
  r->n_feasible = nf;
  if (mode == YODA_MODE_SCV) {
    mv = collect_max_values(pd, p, nd);
  }
  r->maxima = mv;
  if (nf == 0) {
    r->pick = YODA_PICK_NONE;
    r->status = YODA_STATUS_UNSCHEDULABLE;
    return;
  }
  int div_zero = 0;
  for (uint32_t i = 0; i < nf; ++i) {
    uint32_t n = feas[i];
    if (mode == YODA_MODE_SCV) {
      /* algorithm.go:96 composition; Go evaluates left to right */
      uint64_t raw = basic_score(&mv, pd, p, nd, n);
      raw += allocate_score(nd, n, &div_zero);
      raw += actual_score(nd, n, &div_zero);
      scores[i] = uint64_to_int64(raw);
    } else if (memo_first >= 0) {
      scores[i] = diskio_score_memo(pd, p, nd, n, memo_first);
    } else {
      scores[i] = diskio_score(pd, p, nd, n);
    }
  }
  if (nf == 1) {
    r->pick = (int32_t)feas[0];
    r->status = YODA_STATUS_OK;
    r->n_ties = 1;
    r->top_score = scores[0];
    return;
  }
  if (div_zero) {
    r->pick = YODA_PICK_ERROR;
    r->status = YODA_STATUS_DIV_ZERO;
    return;
  }
  /* NormalizeScore — scheduler.go:158-183 */
  int64_t highest = 0, lowest = scores[0];
  for (uint32_t i = 0; i < nf; ++i) {
    if (scores[i] < lowest) lowest = scores[i];
    if (scores[i] > highest) highest = scores[i];
  }
  if (highest == lowest) lowest--;
  int64_t* norm = scores + nd->n_nodes;
  for (uint32_t i = 0; i < nf; ++i) {
    int64_t diff = scores[i] - lowest;                /* >= 0, no overflow (see DESIGN) */
    uint64_t prod = (uint64_t)diff * 100u;            /* Go int64 multiply wraps */
    norm[i] = (int64_t)prod / (highest - lowest);     /* truncates toward zero */
    if (norm[i] > 100 || norm[i] < 0) {               /* RunScorePlugins range check */
      r->pick = YODA_PICK_ERROR;
      r->status = YODA_STATUS_SCORE_RANGE;
      return;
    }
  }
  /* selectHost: max normalized score (weight 1), tie set, lowest index */
  int64_t best = norm[0];
  uint32_t bi = 0, ties = 1;
  for (uint32_t i = 1; i < nf; ++i) {
    if (norm[i] > best) {
      best = norm[i];
      bi = i;
      ties = 1;
    } else if (norm[i] == best) {
      ties++;
    }
  }
  r->pick = (int32_t)feas[bi];
  r->status = YODA_STATUS_OK;
  r->n_ties = ties;
  r->top_score = scores[bi];
}

static void write_result(const cycle_result* r, uint32_t p, yoda_eval_out* out) {
  if (out->pick) out->pick[p] = r->pick;
  if (out->status) out->status[p] = r->status;
  if (out->n_feasible) out->n_feasible[p] = r->n_feasible;
  if (out->n_ties) out->n_ties[p] = r->n_ties;
  if (out->top_score) out->top_score[p] = r->top_score;
  if (out->maxima) {
    uint64_t* m = out->maxima + (size_t)p * 6;
    m[0] = r->maxima.bandwidth;
    m[1] = r->maxima.clock;
    m[2] = r->maxima.core;
    m[3] = r->maxima.free_memory;
    m[4] = r->maxima.power;
    m[5] = r->maxima.total_memory;
  }
}

static int schedule_range(const yoda_node_soa* nd, const yoda_pod_soa* pd, int mode,
                          int64_t memo_first, uint32_t p0, uint32_t p1, int n_threads,
                          yoda_eval_out* out) {
  if (!nd || !pd || !out || p1 > pd->n_pods || p0 > p1) return YODA_ERR_INVALID_ARG;
  if (mode != YODA_MODE_SCV && mode != YODA_MODE_DISKIO) return YODA_ERR_INVALID_ARG;
  if (n_threads < 1) n_threads = 1;
  int err = 0;
#pragma omp parallel num_threads(n_threads)
  {
    int64_t* scores = (int64_t*)malloc(sizeof(int64_t) * 2 * ((size_t)nd->n_nodes + 1));
    uint32_t* feas = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)nd->n_nodes + 1));
    if (!scores || !feas) {
#pragma omp atomic write
      err = 1;
    } else {
#pragma omp for schedule(dynamic, 4)
      for (int64_t p = (int64_t)p0; p < (int64_t)p1; ++p) {
        cycle_result r;
        schedule_one(nd, pd, (uint32_t)p, mode, memo_first, scores, feas, &r);
        write_result(&r, (uint32_t)p, out);
      }
    }
    free(scores);
    free(feas);
  }
  return err ? YODA_ERR_INVALID_ARG : YODA_OK;
}

/* Schedule every pod independently against the snapshot (pods [p0, p1)). */
int oracle_schedule_range(const yoda_node_soa* nd, const yoda_pod_soa* pd, int mode, uint32_t p0,
                          uint32_t p1, int n_threads, yoda_eval_out* out) {
  return schedule_range(nd, pd, mode, -1, p0, p1, n_threads, out);
}

/* Mode B with the B3 memo quirk (diskio_score_memo): node `first` is the one whose Score
 * call runs first in every cycle.  Documentation mode only, not a product path. */
int oracle_schedule_memo(const yoda_node_soa* nd, const yoda_pod_soa* pd, uint32_t first,
                         int n_threads, yoda_eval_out* out) {
  if (!nd || first >= nd->n_nodes) return YODA_ERR_INVALID_ARG;
  return schedule_range(nd, pd, YODA_MODE_DISKIO, (int64_t)first, 0, pd ? pd->n_pods : 0,
                        n_threads, out);
}

int oracle_schedule(const yoda_node_soa* nd, const yoda_pod_soa* pd, int mode, int n_threads,
                    yoda_eval_out* out) {
  return oracle_schedule_range(nd, pd, mode, 0, pd ? pd->n_pods : 0, n_threads, out);
}

/* Per-node detail for one pod: feasibility, raw Score (after Uint64ToInt64; 0 where
 * infeasible) and normalized score (-1 where infeasible or not computed). */
int oracle_pod_detail(const yoda_node_soa* nd, const yoda_pod_soa* pd, uint32_t p, int mode,
                      uint8_t* feasible, int64_t* raw, int64_t* norm) {
  if (!nd || !pd || p >= pd->n_pods) return YODA_ERR_INVALID_ARG;
  max_value mv = {1, 1, 1, 1, 1, 1};
  if (mode == YODA_MODE_SCV) mv = collect_max_values(pd, p, nd);
  int div_zero = 0;
  int64_t highest = 0, lowest = 0;
  int first = 1;
  for (uint32_t n = 0; n < nd->n_nodes; ++n) {
    uint64_t m, c;
    int ok = (mode == YODA_MODE_DISKIO) ? 1 : pod_fits_node(pd, p, nd, n, &m, &c);
    feasible[n] = (uint8_t)ok;
    raw[n] = 0;
    norm[n] = -1;
    if (!ok) continue;
    if (mode == YODA_MODE_SCV) {
      uint64_t s = basic_score(&mv, pd, p, nd, n);
      s += allocate_score(nd, n, &div_zero);
      s += actual_score(nd, n, &div_zero);
      raw[n] = uint64_to_int64(s);
    } else {
      raw[n] = diskio_score(pd, p, nd, n);
    }
    if (first) {
      lowest = raw[n];
      first = 0;
    }
    if (raw[n] < lowest) lowest = raw[n];
    if (raw[n] > highest) highest = raw[n];
  }
  if (first) return YODA_OK;
  if (highest == lowest) lowest--;
  for (uint32_t n = 0; n < nd->n_nodes; ++n) {
    if (!feasible[n]) continue;
    uint64_t prod = (uint64_t)(raw[n] - lowest) * 100u;
    norm[n] = (int64_t)prod / (highest - lowest);
  }
  return div_zero ? YODA_STATUS_DIV_ZERO : YODA_OK;
}

/* Greedy batch: pods in queue order — sort.Less (sort.go:8-10), higher
 * scv/priority first, ties by input index (the build's deterministic stand-in for the
 * heap) — each pick "assumed" onto its node: alloc_memory += scv/memory (StrToUint64, only
 * when the label is present; algorithm.go:299-303).  flags & YODA_GREEDY_CARD_CAPACITY:
 * CardNumber -= number (saturating), the build-defined extension.  Mutates neither input. */
static const int64_t* g_prio;
static int cmp_queue(const void* a, const void* b) {
  uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  int64_t px = g_prio ? g_prio[x] : 0, py = g_prio ? g_prio[y] : 0;
  if (px != py) return px > py ? -1 : 1;
  return x < y ? -1 : (x > y ? 1 : 0);
}

int oracle_queue_order(const yoda_pod_soa* pd, uint32_t* order) {
  for (uint32_t i = 0; i < pd->n_pods; ++i) order[i] = i;
  g_prio = pd->priority;
  qsort(order, pd->n_pods, sizeof(uint32_t), cmp_queue);
  g_prio = NULL;
  return YODA_OK;
}

int oracle_greedy(const yoda_node_soa* nd_in, const yoda_pod_soa* pd, int mode, uint32_t flags,
                  int32_t* pick, int32_t* status) {
  if (!nd_in || !pd || !pick) return YODA_ERR_INVALID_ARG;
  uint32_t N = nd_in->n_nodes, P = pd->n_pods;
  yoda_node_soa nd = *nd_in;
  uint64_t* alloc = (uint64_t*)calloc((size_t)N + 1, sizeof(uint64_t));
  uint64_t* cardn = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)N + 1));
  int64_t* scores = (int64_t*)malloc(sizeof(int64_t) * 2 * ((size_t)N + 1));
  uint32_t* feas = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)N + 1));
  uint32_t* order = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)P + 1));
  if (!alloc || !cardn || !scores || !feas || !order) {
    free(alloc); free(cardn); free(scores); free(feas); free(order);
    return YODA_ERR_INVALID_ARG;
  }
  for (uint32_t n = 0; n < N; ++n) {
    alloc[n] = nd_in->alloc_memory ? nd_in->alloc_memory[n] : 0;
    cardn[n] = nd_in->card_number[n];
  }
  nd.alloc_memory = alloc;
  nd.card_number = cardn;
  oracle_queue_order(pd, order);
  for (uint32_t i = 0; i < P; ++i) {
    uint32_t p = order[i];
    cycle_result r;
    schedule_one(&nd, pd, p, mode, -1, scores, feas, &r);
    pick[p] = r.pick;
    if (status) status[p] = r.status;
    if (r.pick >= 0) {
      if (pd->has_memory[p]) alloc[r.pick] += pd->memory[p];
      if (flags & YODA_GREEDY_CARD_CAPACITY) {
        uint64_t num = pd->has_number[p] ? pd->number[p] : 1;
        cardn[r.pick] = cardn[r.pick] >= num ? cardn[r.pick] - num : 0;
      }
    }
  }
  free(alloc); free(cardn); free(scores); free(feas); free(order);
  return YODA_OK;
}

/* ---- node-parallel cycle (full-size fixtures) -----------------------------------------
 * schedule_one with its node loops split over OpenMP threads, for the full-size greedy
 * fixtures (config 5: 1M sequential cycles over 100k nodes).  Same functions, same order of
 * decisions: Filter per node (collection.go:41-44), the maxima over the feasible nodes'
 * cards (collection.go:46; MAX is order-free), the raw score per feasible node
 * (algorithm.go:96, scheduler.go:154), NormalizeScore's highest (init 0) and lowest (a
 * member of the list, so a plain MIN) (scheduler.go:162-175), the per-node normalized score
 * and range check (:178), and selectHost's maximum with the lowest node index and the tie
 * count.  Every reduction is MAX / MIN / SUM / lowest-index, so the result does not depend
 * on the thread count or schedule.  Scratch: raw[N] int64, ok[N] uint8. */

/* CalculateBasicScore's card loop (algorithm.go:270-276) for a node already known feasible */
static uint64_t basic_score_fit(const max_value* v, uint64_t memory, uint64_t clock,
                                const yoda_node_soa* nd, uint32_t n) {
  uint64_t s = 0;
  for (uint32_t j = 0; j < nd->card_count[n]; ++j) {
    card_t c = get_card(nd, n, j);
    if (c.free_memory >= memory && c.clock >= clock) s += card_score(v, &c);
  }
  return s;
}

static void schedule_one_par(const yoda_node_soa* nd, const yoda_pod_soa* pd, uint32_t p,
                             int n_threads, int64_t* raw, uint8_t* ok, cycle_result* r) {
  const int64_t N = nd->n_nodes;
  memset(r, 0, sizeof(*r));
  max_value mv = {1, 1, 1, 1, 1, 1};
  uint32_t nf = 0;
  int64_t first = -1;
  /* Filter + CollectMaxValues: one pass (the predicate is a pure function of the pair) */
#pragma omp parallel num_threads(n_threads)
  {
    max_value lv = {1, 1, 1, 1, 1, 1};
    uint32_t lnf = 0;
    int64_t lfirst = -1;
#pragma omp for schedule(static)
    for (int64_t n = 0; n < N; ++n) {
      uint64_t m, c;
      ok[n] = (uint8_t)pod_fits_node(pd, p, nd, (uint32_t)n, &m, &c);
      if (!ok[n]) continue;
      if (lfirst < 0) lfirst = n;
      lnf++;
      for (uint32_t j = 0; j < nd->card_count[n]; ++j) {
        card_t cd = get_card(nd, (uint32_t)n, j);
        if (cd.free_memory >= m && cd.clock >= c) process_max_value_with_card(&cd, &lv);
      }
    }
#pragma omp critical
    {
      nf += lnf;
      if (lfirst >= 0 && (first < 0 || lfirst < first)) first = lfirst;
      if (lv.bandwidth > mv.bandwidth) mv.bandwidth = lv.bandwidth;
      if (lv.clock > mv.clock) mv.clock = lv.clock;
      if (lv.core > mv.core) mv.core = lv.core;
      if (lv.free_memory > mv.free_memory) mv.free_memory = lv.free_memory;
      if (lv.power > mv.power) mv.power = lv.power;
      if (lv.total_memory > mv.total_memory) mv.total_memory = lv.total_memory;
    }
  }
  r->n_feasible = nf;
  r->maxima = mv;
  if (nf == 0) {
    r->pick = YODA_PICK_NONE;
    r->status = YODA_STATUS_UNSCHEDULABLE;
    return;
  }
  /* Score per feasible node (algorithm.go:96, left to right; Uint64ToInt64).  The card
   * predicate's thresholds are what pod_fits_node reports for any feasible node: the pod's
   * scv/memory and scv/clock, 0 when the label is absent (filter.go:18-50). */
  const uint64_t m_thr = pd->has_memory[p] ? pd->memory[p] : 0;
  const uint64_t c_thr = pd->has_clock[p] ? pd->clock[p] : 0;
  int div_zero = 0;
  int64_t highest = 0, lowest = INT64_MAX;
#pragma omp parallel num_threads(n_threads)
  {
    int ldz = 0;
    int64_t lhi = 0, llo = INT64_MAX;
#pragma omp for schedule(static)
    for (int64_t n = 0; n < N; ++n) {
      if (!ok[n]) continue;
      uint64_t s = basic_score_fit(&mv, m_thr, c_thr, nd, (uint32_t)n);
      s += allocate_score(nd, (uint32_t)n, &ldz);
      s += actual_score(nd, (uint32_t)n, &ldz);
      raw[n] = uint64_to_int64(s);
      if (raw[n] > lhi) lhi = raw[n];
      if (raw[n] < llo) llo = raw[n];
    }
#pragma omp critical
    {
      div_zero |= ldz;
      if (lhi > highest) highest = lhi;
      if (llo < lowest) lowest = llo;
    }
  }
  if (nf == 1) {
    r->pick = (int32_t)first;
    r->status = YODA_STATUS_OK;
    r->n_ties = 1;
    r->top_score = raw[first];
    return;
  }
  if (div_zero) {
    r->pick = YODA_PICK_ERROR;
    r->status = YODA_STATUS_DIV_ZERO;
    return;
  }
  if (highest == lowest) lowest--;
  int range_err = 0;
  int64_t best = -1, bi = -1;
  uint32_t ties = 0;
#pragma omp parallel num_threads(n_threads)
  {
    int lerr = 0;
    int64_t lbest = -1, lbi = -1;
    uint32_t lties = 0;
#pragma omp for schedule(static)
    for (int64_t n = 0; n < N; ++n) {
      if (!ok[n]) continue;
      uint64_t prod = (uint64_t)(raw[n] - lowest) * 100u;
      int64_t norm = (int64_t)prod / (highest - lowest);
      if (norm > 100 || norm < 0) lerr = 1;
      if (norm > lbest) {
        lbest = norm;
        lbi = n;
        lties = 1;
      } else if (norm == lbest) {
        lties++;
      }
    }
#pragma omp critical
    {
      range_err |= lerr;
      if (lbest > best) {
        best = lbest;
        bi = lbi;
        ties = lties;
      } else if (lbest == best && lbest >= 0) {
        if (lbi < bi) bi = lbi;
        ties += lties;
      }
    }
  }
  if (range_err) {
    r->pick = YODA_PICK_ERROR;
    r->status = YODA_STATUS_SCORE_RANGE;
    return;
  }
  r->pick = (int32_t)bi;
  r->status = YODA_STATUS_OK;
  r->n_ties = ties;
  r->top_score = raw[bi];
}

/* oracle_greedy with node-parallel cycles, for the full-size fixtures.  Pods in queue order
 * [q0, q1) only (q0 = 0, q1 = P: the whole batch), starting from the node state given (its
 * alloc_memory and card_number: a replayed state for a later block).  top_score / n_ties
 * optional. */
int oracle_greedy_mt(const yoda_node_soa* nd_in, const yoda_pod_soa* pd, uint32_t flags,
                     uint32_t q0, uint32_t q1, int n_threads, int32_t* pick, int32_t* status,
                     int64_t* top_score, uint32_t* n_ties) {
  if (!nd_in || !pd || !pick || q0 > q1 || q1 > pd->n_pods) return YODA_ERR_INVALID_ARG;
  if (n_threads < 1) n_threads = 1;
  uint32_t N = nd_in->n_nodes, P = pd->n_pods;
  yoda_node_soa nd = *nd_in;
  uint64_t* alloc = (uint64_t*)calloc((size_t)N + 1, sizeof(uint64_t));
  uint64_t* cardn = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)N + 1));
  int64_t* raw = (int64_t*)malloc(sizeof(int64_t) * ((size_t)N + 1));
  uint8_t* ok = (uint8_t*)malloc((size_t)N + 1);
  uint32_t* order = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)P + 1));
  if (!alloc || !cardn || !raw || !ok || !order) {
    free(alloc); free(cardn); free(raw); free(ok); free(order);
    return YODA_ERR_INVALID_ARG;
  }
  for (uint32_t n = 0; n < N; ++n) {
    alloc[n] = nd_in->alloc_memory ? nd_in->alloc_memory[n] : 0;
    cardn[n] = nd_in->card_number[n];
  }
  nd.alloc_memory = alloc;
  nd.card_number = cardn;
  oracle_queue_order(pd, order);
  for (uint32_t i = q0; i < q1; ++i) {
    uint32_t p = order[i];
    cycle_result r;
    schedule_one_par(&nd, pd, p, n_threads, raw, ok, &r);
    pick[p] = r.pick;
    if (status) status[p] = r.status;
    if (top_score) top_score[p] = r.top_score;
    if (n_ties) n_ties[p] = r.n_ties;
    if (r.pick >= 0) { /* the assume of oracle_greedy */
      if (pd->has_memory[p]) alloc[r.pick] += pd->memory[p];
      if (flags & YODA_GREEDY_CARD_CAPACITY) {
        uint64_t num = pd->has_number[p] ? pd->number[p] : 1;
        cardn[r.pick] = cardn[r.pick] >= num ? cardn[r.pick] - num : 0;
      }
    }
  }
  free(alloc); free(cardn); free(raw); free(ok); free(order);
  return YODA_OK;
}

int oracle_abi_version(void) { return YODA_ABI_VERSION; }
