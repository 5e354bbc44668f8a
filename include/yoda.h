/*
 * yoda.h — C-ABI of libyoda, the MI355X-native Yoda Filter/Score hot path.
 *
 * This is the drop-in boundary a Go kube-scheduler plugin binds through cgo (see
 * INTEGRATION.md).  It replaces the per-pair Go calls the scheduler framework makes into
 * the reference plugin with one call per pod batch:
 *
 *   reference (Mr-LvGJ/kubernetes-scheduler)            replaced by
 *   ---------------------------------------------       -----------------------------------
 *   filter.PodFitsNumber/Memory/Clock                   yoda_run  (K1: feasibility sweep)
 *     pkg/yoda/filter/filter.go:11-58
 *   collection.CollectMaxValues (PreScore)              yoda_run  (K1: per-pod maxima)
 *     pkg/yoda/collection/collection.go:30-76
 *   score.CalculateBasicScore/Card/Allocate/Actual      yoda_run  (K2: integer card score)
 *     pkg/yoda/score/algorithm.go:96,264-310
 *   score.BalancedCpuDiskIOPriority (live Mode B)       yoda_run  (mode YODA_MODE_DISKIO)
 *     pkg/yoda/score/algorithm.go:99-119
 *   Yoda.Score + filter.Uint64ToInt64                   yoda_run  (K2)
 *     pkg/yoda/scheduler.go:116-156, filter.go:84-86
 *   Yoda.NormalizeScore + k8s v1.22.3 selectHost        yoda_run  (K2 argmax + finalize)
 *     pkg/yoda/scheduler.go:158-183
 *   sort.Less / GetPodPriority (greedy batch order)     yoda_greedy
 *     pkg/yoda/sort/sort.go:8-18
 *
 * Conventions:
 *   - every entry point returns int: YODA_OK (0) or a negative YODA_ERR_* code; the
 *     message of the last failure is in yoda_last_error();
 *   - no C++ exception crosses the boundary; all buffers are caller-owned;
 *   - a handle is NOT thread-safe: one handle per goroutine, or guard it;
 *   - "d_" pointer arguments are device pointers (HIP global memory on the handle's
 *     device); everything else is host memory.
 *
 * Integer widths follow the reference on GOARCH=amd64 (Makefile:4): Go `uint` is 64-bit.
 */
#ifndef YODA_H_
#define YODA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YODA_ABI_VERSION 1

/* Maximum card slots per node (SCV Status.CardList length). */
#define YODA_MAX_CARDS 16

/* ---- status codes ------------------------------------------------------------------ */
#define YODA_OK 0
#define YODA_ERR_INVALID_ARG -1   /* NULL handle/pointer, bad size, bad mode            */
#define YODA_ERR_HIP -2           /* a HIP runtime call failed                          */
#define YODA_ERR_NO_NODES -3      /* yoda_run/yoda_eval before yoda_upload_nodes        */
#define YODA_ERR_NO_PODS -4       /* yoda_run before yoda_upload_pods                   */
#define YODA_ERR_RANGE -5         /* input outside what the library can represent       */
#define YODA_ERR_NO_DEVICE -6     /* no HIP device / bad device ordinal                 */
#define YODA_ERR_STATE -7         /* call out of sequence (e.g. phase2 before phase1)   */
#define YODA_ERR_SAME_DEVICE -8   /* two ranks of one communicator on the same GPU      */

/* ---- scoring modes ----------------------------------------------------------------- */
/* Mode A: the SCV GPU path (filter.go + collection.go + algorithm.go:264-310 composed as
 * algorithm.go:96).  Mode B: the score the shipped binary computes
 * (BalancedCpuDiskIOPriority, algorithm.go:99-119; Filter is a pass-through). */
#define YODA_MODE_SCV 0
#define YODA_MODE_DISKIO 1

/* ---- per-pod outcome (the framework Status the reference would produce) ------------ */
#define YODA_PICK_NONE (-1)  /* no feasible node: Unschedulable                          */
#define YODA_PICK_ERROR (-2) /* framework Error (see status)                             */

#define YODA_STATUS_OK 0             /* pick is a node index                              */
#define YODA_STATUS_UNSCHEDULABLE 1  /* no node passed Filter                              */
#define YODA_STATUS_DIV_ZERO 2       /* a scored node has TotalMemorySum == 0: the
                                        reference panics (algorithm.go:294 / :309)        */
#define YODA_STATUS_SCORE_RANGE 3    /* NormalizeScore produced a score outside [0,100]
                                        (int64 overflow at scheduler.go:178); k8s rejects */

/* Node snapshot, struct-of-arrays.  Node i's card slot j lives at [i * max_cards + j];
 * slots j >= card_count[i] are ignored.  Mirrors the SCV CRD Status
 * (github.com/NJUPT-ISL/SCV api/v1 @46b36eeed646, types pinned by use: filter.go:13,22,53,57,
 * collection.go:14-20, algorithm.go:294,305-309). */
typedef struct yoda_node_soa {
  uint32_t n_nodes;
  uint32_t max_cards;                /* stride of the card arrays, 1..YODA_MAX_CARDS        */
  const uint64_t* card_number;       /* [N] Status.CardNumber                              */
  const uint32_t* card_count;        /* [N] len(Status.CardList), <= max_cards             */
  const uint64_t* free_memory_sum;   /* [N] Status.FreeMemorySum                           */
  const uint64_t* total_memory_sum;  /* [N] Status.TotalMemorySum                          */
  const uint64_t* alloc_memory;      /* [N] sum of scv/memory labels of pods already bound
                                        to the node (algorithm.go:299-303); may be NULL=0   */
  const uint64_t* card_free_memory;  /* [N*K] Card.FreeMemory                              */
  const uint64_t* card_total_memory; /* [N*K] Card.TotalMemory                             */
  const uint64_t* card_clock;        /* [N*K] Card.Clock                                   */
  const uint64_t* card_bandwidth;    /* [N*K] Card.Bandwidth                               */
  const uint64_t* card_core;         /* [N*K] Card.Core                                    */
  const uint64_t* card_power;        /* [N*K] Card.Power                                   */
  const uint8_t* card_healthy;       /* [N*K] Card.Health == "Healthy"                     */
  /* Mode B inputs: advisor.NodeInfo (advisor.go:26-32).  May be NULL for Mode A. */
  const double* cpu;                 /* [N] NodeInfo.Cpu   (percent)                       */
  const double* disk_io;             /* [N] NodeInfo.DiskIO (MB/s)                         */
} yoda_node_soa;

/* Pod requests, struct-of-arrays, already parsed from labels with the reference's Go
 * semantics (strconv.Atoi; negative values wrap to uint64 — filter.go:60-74). */
typedef struct yoda_pod_soa {
  uint32_t n_pods;
  const uint8_t* has_number;   /* [P] label scv/number present (filter.go:12)               */
  const uint64_t* number;      /* [P] strToUint(scv/number)                                */
  const uint8_t* has_memory;   /* [P] label scv/memory present (filter.go:19)               */
  const uint64_t* memory;      /* [P] StrToUint64(scv/memory)                              */
  const uint8_t* has_clock;    /* [P] label scv/clock present (filter.go:36)                */
  const uint64_t* clock;       /* [P] strToUint(scv/clock)                                 */
  const int64_t* priority;     /* [P] Atoi(scv/priority) (sort.go:12-18); may be NULL = 0   */
  /* Mode B: may be NULL for Mode A. */
  const double* rio;           /* [P] ParseFloat(annotations["diskIO"], 32) (algorithm.go:103) */
  const int64_t* rcpu;         /* [P] CalculatePodResourceRequest(cpu) millicores (:104,238) */
} yoda_pod_soa;

/* Per-pod outputs of yoda_eval / yoda_download.  Any pointer may be NULL. */
typedef struct yoda_eval_out {
  int32_t* pick;         /* [P] node index (global), YODA_PICK_NONE or YODA_PICK_ERROR     */
  int32_t* status;       /* [P] YODA_STATUS_*                                              */
  uint32_t* n_feasible;  /* [P] nodes that passed Filter                                   */
  uint32_t* n_ties;      /* [P] nodes sharing the top normalized score (the set k8s
                            selectHost draws from at random)                              */
  int64_t* top_score;    /* [P] raw Score (after Uint64ToInt64) of the picked node         */
  uint64_t* maxima;      /* [P*6] Mode A PreScore maxima in MaxValue order (collection.go:
                            14-21): Bandwidth, Clock, Core, FreeMemory, Power, TotalMemory */
} yoda_eval_out;

typedef struct yoda_handle yoda_t;

/* ---- lifecycle ---------------------------------------------------------------------- */
int yoda_abi_version(void);
/* One handle drives one GPU (device ordinal).  Multi-GPU: one handle per GPU, each holding
 * a node shard, merged by the caller's collectives through the yoda_shard_* entry points. */
int yoda_create(int device, yoda_t** out);
int yoda_destroy(yoda_t* h);
const char* yoda_last_error(const yoda_t* h);
/* Launch all work on this HIP stream (hipStream_t passed as void*; NULL = the HIP null
 * stream, e.g. PyTorch's default stream).  Until called, the handle uses a non-blocking
 * stream of its own; yoda_use_own_stream switches back to it.  Work the handle already
 * queued on its previous stream (e.g. an upload's copies) is ordered before the new
 * stream's next work (an event wait on the device, no host synchronization). */
int yoda_set_stream(yoda_t* h, void* hip_stream);
int yoda_use_own_stream(yoda_t* h);
int yoda_synchronize(yoda_t* h);

/* ---- node snapshot ------------------------------------------------------------------ */
/* Upload a node snapshot (or a shard of one).  node_offset is the global index of this
 * shard's first node: picks are reported as node_offset + local index.  Replaces the
 * previous snapshot.  Chooses the narrowest exact record format the value ranges allow
 * (DESIGN.md §Exactness). */
#define YODA_UPLOAD_FORCE_GENERIC 1u /* always the exact-u64 path                     */
#define YODA_UPLOAD_FORCE_F64 2u     /* never the narrow path (tests)                 */
#define YODA_UPLOAD_NO_UNIFORM 4u    /* disable the per-node GPU-model factoring (tests) */
#define YODA_UPLOAD_PER_NODE_K1 8u   /* N32: per-node K1 sweep instead of the block-
                                        classified one (tests, A/B measurements)      */
#define YODA_UPLOAD_PER_NODE_K2 16u  /* N32: per-pod K2 scoring instead of the block-
                                        classified one (tests, A/B measurements)      */
#define YODA_UPLOAD_NO_GTAB 32u      /* N32: no G table (the block K2 computes every
                                        node's card terms itself; tests, A/B)         */
#define YODA_UPLOAD_MEM_RANKS 64u    /* N32: memory ranks even when every memory field
                                        fits 32 bits (tests, A/B)                     */
#define YODA_UPLOAD_F64_QUOTIENTS 128u /* N32: small-field quotients in f64 even when
                                        every bandwidth/clock/core/power <= 55738 --
                                        for a node shard whose peers hold wider
                                        fields (yoda_small_field_max); a shard with
                                        mixed-model nodes then takes YODA_PATH_F64    */
int yoda_upload_nodes(yoda_t* h, const yoda_node_soa* nodes, uint32_t node_offset,
                      uint32_t flags);
/* 1 if the uploaded snapshot runs on the generic (u64) path, 0 on a fast path. */
int yoda_uses_generic_path(const yoda_t* h);
/* Record format of the uploaded snapshot: YODA_PATH_N32 (u32 fields; f32 or f64 quotients,
 * DESIGN.md §5), YODA_PATH_F64 (exact f64) or YODA_PATH_U64 (exact uint64 wrap-around). */
#define YODA_PATH_N32 0
#define YODA_PATH_F64 1
#define YODA_PATH_U64 2
int yoda_record_path(const yoda_t* h);
/* 1 if the N32 snapshot holds its FreeMemory / TotalMemory as ranks (fields beyond 32 bits,
 * e.g. bytes: the u32 fields keep every comparison and maximum, value tables give the
 * quotients and the maxima -- DESIGN.md §3), 0 if as values; -1 for a NULL handle.  The
 * PreScore maxima returned and exchanged are values either way. */
int yoda_memory_ranks(const yoda_t* h);
/* The largest bandwidth, clock, core or power of any card of the uploaded snapshot.  N32
 * computes their quotients in f32 while every maximum it divides by is <= 55738 and in f64
 * beyond (every bandwidth/clock/core/power up to 2^32 - 2 stays on N32 when every node holds
 * one GPU model with one TotalMemory).  Node shards exchange maxima, so all shards must agree:
 * when the MAX of this over the shards exceeds 55738, re-upload the others with
 * YODA_UPLOAD_F64_QUOTIENTS (yoda_amd/dist.py agree_on_path) before agreeing on the record
 * path.  0 for a NULL handle. */
uint64_t yoda_small_field_max(const yoda_t* h);
/* An upper bound on every raw Score of the uploaded snapshot whatever its allocated memory
 * (Basic at the largest clock + the largest Allocate 300 + Actual); ~0 when unbounded.  The
 * sharded merge packs (score, node) into one 64-bit key when it fits (yoda_amd/dist.py). */
uint64_t yoda_score_bound(const yoda_t* h);
/* Replace alloc_memory (the Allocate-score input) without re-uploading the cards. */
int yoda_update_alloc(yoda_t* h, const uint64_t* alloc_memory);

/* ---- one-shot evaluation ------------------------------------------------------------ */
/* Schedule every pod independently against the uploaded snapshot (each pod sees the same
 * snapshot: a batch of independent scheduling cycles).  Equivalent to
 * yoda_upload_pods + yoda_run + yoda_download. */
int yoda_eval(yoda_t* h, const yoda_pod_soa* pods, int mode, yoda_eval_out* out);

/* ---- split evaluation (device-resident timing, multi-GPU) --------------------------- */
int yoda_upload_pods(yoda_t* h, const yoda_pod_soa* pods);
/* Run filter+prescore+score+normalize+select for the uploaded pods; results stay on the
 * device until yoda_download.  Asynchronous on the handle's stream. */
#define YODA_RUN_BITMASK 1u /* also materialise the feasibility bitmask for download      */
int yoda_run(yoda_t* h, int mode, uint32_t flags);
int yoda_download(yoda_t* h, yoda_eval_out* out);
/* Feasibility bitmask of the last yoda_run with YODA_RUN_BITMASK: bit (n & 31) of
 * words[p * ((N + 31) / 32) + n / 32] is set iff node n (local) passed Filter for pod p. */
int yoda_download_bitmask(yoda_t* h, uint32_t* words, uint64_t n_words);

/* Framework-plugin row mode: for the uploaded pods (a handful — one per
 * scheduling cycle), return the Filter result and the raw Score of EVERY node, so the
 * plugin's Filter and Score become lookups and NormalizeScore/selectHost stay the
 * reference's code.  bitmask: [P][ceil(N/32)] as yoda_download_bitmask; scores: [P][N]
 * int64, the value Yoda.Score returns (after Uint64ToInt64), -1 where Filter fails.
 * Also leaves the picks for yoda_download.  Either output may be NULL. */
int yoda_score_rows(yoda_t* h, int mode, uint32_t* bitmask, uint64_t n_bitmask_words,
                    int64_t* scores, uint64_t n_scores);
/* yoda_score_rows plus the normalized scores, computed on the device: norm [P][N] int64 =
 * Yoda.NormalizeScore (scheduler.go:158-183) over each pod's feasible nodes -- highest =
 * max(0, max raw), lowest = min raw, lowest-- when equal, (raw - lowest) * 100 /
 * (highest - lowest) in Go's int64 arithmetic -- and -1 where Filter fails.  k8s then adds
 * the plugin weight and validates [0, 100] (RunScorePlugins). */
int yoda_score_rows_norm(yoda_t* h, int mode, uint32_t* bitmask, uint64_t n_bitmask_words,
                         int64_t* scores, uint64_t n_scores, int64_t* norm, uint64_t n_norm);

/* Sharded evaluation.  Each rank holds a node shard; between phases the caller reduces
 * the exchange buffers across ranks (RCCL all-reduce) with the op named per buffer.
 *   phase1 -> d_maxima [6*P] u64 (MAX), d_counts [2*P] u32 (SUM: n_feasible, n_zero_total)
 *   phase2 (reads reduced maxima/counts) -> d_best [P] i64 (MAX), d_idx [P] u32, d_ties [P]
 *            u32, d_lowest [P] i64 (MIN)
 *   prepare_merge (reads reduced d_best) -> masks d_idx (MIN) and d_ties (SUM) in place
 *   finalize (reads reduced buffers) -> picks into the handle, then yoda_download. */
/* yoda_shard_exchange_order(h, 1): the exchange buffers above are in the CALLER's pod order
 * (the order of yoda_upload_pods), so each shard sorts its pods and nodes privately -- the
 * padded counting order and block-grouped node order of yoda_run -- instead of the
 * reproducible radix order all shards must otherwise share (one shard of config 3: 5.7x
 * faster).  Every shard of a batch must use the same setting.  Evaluation batches only (the
 * greedy-window entry points below refuse it); the U64 record path ignores it.  Default 0. */
int yoda_shard_exchange_order(yoda_t* h, int caller_order);
int yoda_shard_phase1(yoda_t* h, int mode, uint64_t* d_maxima, uint32_t* d_counts);
int yoda_shard_phase2(yoda_t* h, int mode, const uint64_t* d_maxima, const uint32_t* d_counts,
                      int64_t* d_best, uint32_t* d_idx, uint32_t* d_ties, int64_t* d_lowest);
int yoda_shard_prepare_merge(yoda_t* h, const int64_t* d_best_global, const int64_t* d_best_local,
                             uint32_t* d_idx, uint32_t* d_ties);
int yoda_shard_finalize(yoda_t* h, int mode, const uint32_t* d_counts, const int64_t* d_best,
                        const uint32_t* d_idx, const uint32_t* d_ties, const int64_t* d_lowest);
/* Generic path only: pods whose NormalizeScore can overflow int64 are re-evaluated with
 * the exact normalize (scheduler.go:176-179).  Returns the number of such pods in *n_pods
 * (after yoda_shard_finalize: nonzero means the exchange below is needed). */
int yoda_shard_overflow_count(yoda_t* h, uint32_t* n_pods);
/* When yoda_shard_overflow_count reports pods after yoda_shard_finalize, their exact normalize
 * is split across the shards: yoda_shard_exact_records writes this shard's per-pod records
 * (d_rec: [P] x 24 bytes, device), the caller ALL-GATHERS them over the ranks in rank order
 * (d_all: [world][P] x 24 bytes) and yoda_shard_exact_merge folds them into the picks (best
 * normalized score, lowest node, ties summed, a score outside [0, 100] -> STATUS_SCORE_RANGE),
 * completing the step.  yoda_comm_run does this itself. */
int yoda_shard_exact_records(yoda_t* h, void* d_rec);
int yoda_shard_exact_merge(yoda_t* h, const void* d_all, int world);

/* ---- multi-GPU without a host framework: RCCL inside libyoda ------------------------
 * For callers that have no torch.distributed (the Go plugin through cgo, C).  One handle per
 * GPU holds a node shard (yoda_upload_nodes with its node_offset) and the same pod batch.
 * Rank 0 calls yoda_comm_unique_id and hands the id to the other ranks out of band (a file,
 * the k8s API, MPI ...); every rank then calls yoda_comm_init (collective).  yoda_comm_run is
 * one whole sharded step on the handle's stream -- phase 1; ONE group of all-reduces: MAX of
 * the maxima (+ two agreement words: score bits, node-id bits) and SUM of the counts; phase 2;
 * on the fast record paths the packed-key merge: all-reduce(MAX) of each shard's
 * (best << ib | 2^ib - 1 - node) key, then all-reduce(SUM) of the winners' tie counts (the
 * U64 path in Mode A all-gathers (best, index, ties, lowest) records instead); finalize --
 * and leaves the picks for yoda_download, like yoda_run.  All shards must run the same
 * record path.  librccl.so.1 is opened at the first call (not a link dependency).
 * yoda_comm_run_local runs the same step for `world` shard handles of ONE process on one
 * device, with device copies as the transport (tests, single-process use). */
#define YODA_COMM_ID_BYTES 128
int yoda_comm_unique_id(uint8_t* id);
int yoda_comm_init(yoda_t* h, const uint8_t* id, int rank, int world);
/* RCCL refuses two ranks on one GPU ("invalid usage").  Before yoda_comm_init every rank
 * exchanges its device key (yoda_device_key, YODA_DEVICE_KEY_BYTES, NUL-terminated: a 16-hex
 * hash of the hostname and boot id, '/', the PCI bus id of yoda_device_bus_id -- bus ids alone
 * repeat across identical servers) along with the communicator id, and checks the gathered keys
 * (rank-major, `stride` bytes apart): YODA_ERR_SAME_DEVICE when two ranks share one, with
 * *rank_a < *rank_b the first such pair (either pointer may be NULL).  Host only: no HIP call. */
#define YODA_BUS_ID_BYTES 32
#define YODA_DEVICE_KEY_BYTES 64
int yoda_device_bus_id(const yoda_t* h, char* out, int len);
int yoda_device_key(const yoda_t* h, char* out, int len);
int yoda_comm_check_devices(const char* bus_ids, int world, int stride, int* rank_a,
                            int* rank_b);
int yoda_comm_run(yoda_t* h, int mode);
int yoda_comm_run_local(yoda_t* const* handles, int world, int mode);
/* The greedy batch (yoda_greedy's semantics) over the ranks' node shards, driven inside libyoda
 * (collective: every rank passes the same pods and the SAME full snapshot `all_nodes`, which the
 * host-side resolve reads; its handle holds this rank's shard).  Per window the maxima / counts
 * (capacity mode: and the maxima witnesses) are all-reduced and the shards' top-k candidate
 * lists all-gathered; an uncertified pod is scored on every shard and the (score, node)
 * candidates all-gathered.  U64 snapshots: every pod one sharded exact step.  pick [P]: global
 * node ids in input order.  The shards' node state is restored at the end.  The C/cgo twin of
 * the Python driver dist.sharded_greedy (the Go plugin's ShardedGreedy calls it); the same
 * picks, but its capacity windows take yoda_greedy's deeper lists (each shard's merged to 64,
 * the union cut where it stops being certain), so it runs fewer windows than the Python driver.
 * _local: the same over `world` handles of this process on one device (tests). */
int yoda_comm_greedy(yoda_t* h, const yoda_node_soa* all_nodes, const yoda_pod_soa* pods,
                     int mode, uint32_t flags, int32_t* pick);
/* Work counters of the last yoda_comm_greedy[_local] on this handle (the first handle for
 * _local): out[5] = {windows, pods evaluated one by one (exchanges), capacity restarts,
 * mid-window list refreshes, collective calls}. */
int yoda_comm_greedy_stats(const yoda_t* h, uint32_t* out);
int yoda_comm_greedy_local(yoda_t* const* handles, int world, const yoda_node_soa* all_nodes,
                           const yoda_pod_soa* pods, int mode, uint32_t flags, int32_t* pick);

/* ---- batch ordering ---------------------------------------------------------------- */
/* Mode A runs of more than 128 pods (yoda_run, yoda_score_rows, yoda_shard_phase1) sort the
 * batch on the device by the Filter's inputs so that whole wavefronts skip infeasible nodes;
 * every output is returned in the caller's pod order, so results never depend on it.
 * enable = 0 turns the ordering off; 1 (default) orders, a private run (yoda_run) padding each
 * (clock, number, has-memory) group to a wave boundary when that adds at most 1/8 of the
 * batch; 2 orders without the padding.  Takes effect from the next run. */
int yoda_set_pod_order(yoda_t* h, int enable);
/* The batch order (diagnostic): out[4] = {(clock, number, has-memory) groups of the uploaded
 * batch (0: too many for the counting sort), its sorted positions with every group padded to
 * a wave, the sorted positions of the last run, how that run was ordered (0 not, 1 radix sort,
 * 2 counting sort)}. */
int yoda_order_info(const yoda_t* h, uint32_t* out);
/* The node snapshot's order in private runs (diagnostic): *grouped = 1 when its one-model nodes
 * are dealt into 64-node blocks of one clock for yoda_run (copies of the summaries in that
 * order; YODA_NODE_PERM=0 disables), 0 when the upload order is used. */
int yoda_node_order(const yoda_t* h, uint32_t* grouped);

/* ---- kernel timing ----------------------------------------------------------------- */
/* enable != 0: every subsequent K1 / K2 launch is bracketed by HIP events recorded on the
 * launch stream.  yoda_profile_read synchronizes, returns the summed K1 and K2 durations
 * (ms) and launch count since the last read, and clears them. */
int yoda_profile(yoda_t* h, int enable);
int yoda_profile_read(yoda_t* h, double* k1_ms, double* k2_ms, uint32_t* n_launches);

/* ---- work classes ------------------------------------------------------------------ */
/* Device counters of how the block-classified kernels (N32 path) split the
 * (pod wave, node) pairs of the runs made while enabled (one atomic per wave and chunk).
 * read: {K1 ALL, K1 NONE, K1 PART, K2 U, K2 FAST, K2 EXACT, K2 skipped,
 * K2 (wave, chunk)s with uniform maxima, K2 (wave, chunk)s, (wave, node) pairs,
 * K2 FAST pairs served by node records, K2 per-pod pairs of non-uniform waves,
 * the most per-pod nodes of one (wave, chunk), K1 (wave, 64-node block)s the block summaries
 * decide NONE, ... decide ALL, K1 (wave, block)s classified node by node, K2 (wave, block)s
 * pruned by their bound,
 * K2 (wave, block)s worked on}: out[18]; resets them. */
int yoda_class_stats_enable(yoda_t* h, int enable);
int yoda_class_stats_read(yoda_t* h, uint64_t* out);
/* Diagnostic: with YODA_K2_TRACE=<slots> set when the counters are enabled, the block K2
 * records per (pod wave, chunk) {start, end (100 MHz clock), per-pod nodes, uniform maxima}
 * at slot wave * chunks + chunk; out[4 * n_slots]. */
int yoda_k2_trace_read(yoda_t* h, uint64_t* out, uint64_t n_slots);

/* ---- greedy batch ------------------------------------------------------------------- */
/* Schedule the pods one after another in queue order (sort.go:8-10: scv/priority
 * descending, then input index), each pick feeding the next cycle through the node's
 * Allocate score (alloc_memory += scv/memory, algorithm.go:299-303; the scheduler-cache
 * "assume" of SURVEY §3.4).  YODA_GREEDY_CARD_CAPACITY additionally decrements the picked
 * node's CardNumber by the pod's number (saturating at 0): a build-defined extension,
 * batched as well (a window restarts at the first pod the capacity certificate cannot
 * clear).  The uploaded snapshot is left unchanged. */
#define YODA_GREEDY_CARD_CAPACITY 1u
int yoda_greedy(yoda_t* h, const yoda_pod_soa* pods, int mode, uint32_t flags, int32_t* pick);
/* Work counters of the last yoda_greedy: GPU top-k windows, pods evaluated one by one
 * (uncertified candidates, or every pod on the exact sequential path), and host wall time
 * (ms) in times_ms[0..2] = {window candidate passes, sequential resolve, exact fallbacks}
 * (times_ms may be NULL). */
int yoda_greedy_stats(const yoda_t* h, uint32_t* windows, uint32_t* fallbacks,
                      double* times_ms);
/* YODA_GREEDY_CARD_CAPACITY: windows of the last yoda_greedy that ended early at a pod the
 * capacity certificate could not clear (that pod then opens the next window).  The capacity
 * mode restarts on every uncertified pod by default (no exact fallbacks: the fallback count
 * stays 0); the YODA_GREEDY_FAIL_DIV environment knob re-enables one-by-one fallbacks for
 * A/B runs. */
int yoda_greedy_restarts(const yoda_t* h, uint32_t* restarts);
/* flags == 0: mid-window list refreshes of the last yoda_greedy (the window's top-k lists
 * recomputed against the current state once many of its remaining pods had gone uncertified;
 * DESIGN.md §5). */
int yoda_greedy_refreshes(const yoda_t* h, uint32_t* refreshes);

/* ---- sharded greedy batch (node shards on several GPUs) ------------------------------
 * yoda_greedy's windowed algorithm split at its exchange points, so each rank's handle holds
 * a node shard (reference semantics as yoda_greedy: sort.go:8-10 order, the scheduler-cache
 * assume of algorithm.go:299-303).  Per window of W pods, on every rank:
 *   yoda_upload_pods(window) ; yoda_shard_phase1 ; all-reduce maxima MAX, counts SUM ;
 *   yoda_shard_topk -> the shard's best yoda_topk_k() (score, global node) per pod, sorted by
 *     score desc / node asc, -1.0 / 0xFFFFFFFF padding, plus the reduced counts, all in the
 *     window's pod order ;
 *   merge the shards' lists (keep the first yoda_topk_k() of their union in that order) ;
 *   yoda_gs_begin_window ; loop { yoda_gs_resolve -> next ; if next == W break ;
 *     [mid-window refresh, every 8th such pod: when yoda_gs_uncertified(next + 1, 256) >= 16,
 *      push yoda_gs_take_dirty, yoda_shard_topk again on every shard (the window's phase-1
 *      masks and maxima stay valid: only static scores change), merge as above and
 *      yoda_gs_refresh(next, merged) -- then resolve again] ;
 *     push yoda_gs_take_dirty to every shard (yoda_set_node_state) ;
 *     yoda_shard_best_one(next) on every shard ; pick = max score, lowest node ;
 *     yoda_gs_assign(ws + next, pick) } ; push yoda_gs_take_dirty.
 * That is the flags == 0 protocol on the fast record paths (N32 / F64).  With
 * YODA_GREEDY_CARD_CAPACITY each window runs the witness phase 1 below instead, and the first
 * pod the session cannot certify opens the next window (sized by yoda_greedy_next_window);
 * no pod is evaluated one by one.  On the U64 path every pod is one exact sharded step
 * (yoda_shard_phase1 / phase2 / finalize over a one-pod batch) fed to yoda_gs_assign. */
int yoda_topk_k(void);
/* The capacity windows' list depth: yoda_shard_topk returns this many candidates per pod after
 * yoda_shard_phase1_witness (yoda_topk_k() after yoda_shard_phase1). */
int yoda_topk_k_capacity(void);
/* Set the allocated memory (and CardNumber) of the listed nodes (GLOBAL ids; ids outside
 * this handle's shard are ignored) and refresh their static score on the device. */
int yoda_set_node_state(yoda_t* h, uint32_t count, const uint32_t* nodes, const uint64_t* alloc,
                        const uint64_t* card_number);
/* After yoda_shard_phase1 (or _phase1_witness) and the caller's reduction of its buffers
 * (d_maxima, d_counts as there).  k = the list depth of that phase 1, yoda_shard_topk_depth(h)
 * (yoda_topk_k() after yoda_shard_phase1, yoda_topk_k_capacity() after the witness phase 1);
 * any other k is rejected with YODA_ERR_INVALID_ARG, so the caller's buffers always match.
 * Host outputs: counts [2][P] (n_feasible, n_zero_total), top_score [k][P] (f64, exact
 * integers), top_node [k][P]. */
int yoda_shard_topk_depth(const yoda_t* h);
int yoda_shard_topk(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_counts, uint32_t k,
                    uint32_t* counts, double* top_score, uint32_t* top_node);
/* Capacity windows across shards (the window sequence of yoda_comm_greedy and yoda_greedy):
 * yoda_shard_topk after yoda_shard_phase1_witness, but the lists are `deep` long
 * (yoda_greedy_cap_depth()) -- the chunks' lists merged deeper, exact down to their last entry
 * and 0xFFFFFFFF-ended past it; top_score / top_node are [deep][P]. */
int yoda_greedy_cap_depth(void);
int yoda_shard_topk_deep(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_counts,
                         uint32_t k, uint32_t deep, uint32_t* counts, double* top_score,
                         uint32_t* top_node);
/* The shards' list merge of the sharded greedy (host only, no handle): scores / nodes are the
 * world's gathered lists, [world][kl][wn] in shard order (yoda_shard_topk[_deep]'s layout);
 * out_score / out_node [kl][wn] get, for window pods [from, wn), the first kl of the union in
 * (score desc, node asc) order, -1.0 / 0xFFFFFFFF past its end.  Deep lists (kl >
 * yoda_topk_k_capacity()) are cut where a node some shard left unlisted could enter (after the
 * first yoda_topk_k(), at the latest of the shards' last entries).  yoda_comm_greedy merges
 * with this same function. */
int yoda_merge_shard_lists(uint32_t world, uint32_t wn, uint32_t kl, uint32_t from,
                           const double* scores, const uint32_t* nodes, double* out_score,
                           uint32_t* out_node);
/* Exact best node of pod `pod` (index in the batch of the last yoda_shard_topk) over this
 * shard against the CURRENT node state: *node = global id or -1 (no feasible node here),
 * *score = its raw score (lowest node among equal scores). */
int yoda_shard_best_one(yoda_t* h, uint32_t pod, double* score, int32_t* node);

/* YODA_GREEDY_CARD_CAPACITY across shards (fast record paths).  Per window, instead of
 * yoda_shard_phase1: yoda_shard_phase1_witness also writes d_wit [2][6][P] u32 -- per PreScore
 * maxima field the shard's witness count (nodes whose qualifying cards reach the shard's
 * maximum) and its lowest witness (GLOBAL id).  Exchange: keep a copy of the local d_maxima,
 * all-reduce d_maxima MAX and d_counts SUM, yoda_shard_witness_prepare(global, local, d_wit)
 * (clears the fields where this shard does not reach the global maximum), then SUM-reduce
 * d_wit[0, 6P) and MIN-reduce (unsigned) d_wit[6P, 12P).  yoda_shard_topk with
 * k = yoda_topk_k_capacity() (the deeper lists of the capacity windows); then
 * yoda_shard_witness_download gives maxima [6][P] and wit [12][P] in the caller's pod order
 * for yoda_gs_set_witness.  A pod the session cannot certify starts the next window. */
int yoda_shard_phase1_witness(yoda_t* h, uint64_t* d_maxima, uint32_t* d_counts,
                              uint32_t* d_wit);
int yoda_shard_witness_prepare(yoda_t* h, const uint64_t* d_maxima_global,
                               const uint64_t* d_maxima_local, uint32_t* d_wit);
int yoda_shard_witness_download(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_wit,
                                uint64_t* maxima, uint32_t* wit);

/* Host-side sequential resolve over the GLOBAL node set (no GPU); identical on every rank. */
typedef struct yoda_greedy_session yoda_gs_t;
/* nodes: the full snapshot (card_number, free/total memory sums, alloc_memory (may be NULL)
 * are read); pods: the whole batch (number/memory/priority are read). */
int yoda_gs_create(const yoda_node_soa* nodes, const yoda_pod_soa* pods, uint32_t flags,
                   yoda_gs_t** out);
int yoda_gs_destroy(yoda_gs_t* g);
/* order[q] = input index of the pod at queue position q (sort.go:8-10). */
int yoda_gs_queue_order(const yoda_gs_t* g, uint32_t* order);
/* Window = queue positions [ws, ws + wn); arrays in window order as yoda_shard_topk's.  A
 * pod's list may end (0xFFFFFFFF entries) before min(counts[i], k) entries: it then holds its
 * best nodes only down to its last entry (every unlisted node scored at most that, in score
 * desc / node asc order), which becomes the pod's threshold, and is never taken for the whole
 * feasible set (libyoda's own capacity windows pass such lists, merged deeper than exact). */
int yoda_gs_begin_window(yoda_gs_t* g, uint32_t ws, uint32_t wn, uint32_t k,
                         const uint32_t* counts, const double* top_score,
                         const uint32_t* top_node);
/* YODA_GREEDY_CARD_CAPACITY sessions: the window's PreScore maxima [6][wn] with their
 * witnesses -- per field the number of window-start feasible nodes whose qualifying cards
 * reach the maximum, and the lowest such node (GLOBAL id, 0xFFFFFFFF if none) -- window
 * order as yoda_gs_begin_window's arrays; call after it.  Without them a capacity session
 * certifies a pod only while no node it could use has lost cards in the window. */
int yoda_gs_set_witness(yoda_gs_t* g, const uint64_t* maxima, const uint32_t* wit_count,
                        const uint32_t* wit_node);
/* Resolve the window in queue order; *next = the first window pod it cannot certify (wn when
 * the window is done).  flags == 0: the caller scores that pod exactly against the current
 * state (yoda_shard_best_one) and feeds it to yoda_gs_assign.  YODA_GREEDY_CARD_CAPACITY:
 * the caller starts the next window at that pod instead (the certificate of DESIGN.md §5
 * also tracks CardNumber decrements: feasibility and, through the witnesses, the maxima). */
int yoda_gs_resolve(yoda_gs_t* g, uint32_t* next);
int yoda_gs_assign(yoda_gs_t* g, uint32_t queue_pos, int32_t pick);
/* flags == 0: *count = window pods [from, from + scan) with >= 2 feasible nodes whose lists no
 * longer certify them (they stay so: scores only drop) -- the refresh trigger; 0 once some
 * node's Allocate has wrapped (no list certifies then, so a refresh cannot help).
 * YODA_ERR_STATE for capacity sessions. */
int yoda_gs_uncertified(const yoda_gs_t* g, uint32_t from, uint32_t scan, uint32_t* count);
/* New candidate lists for window pods [from, wn) ([k][wn] in window order, as
 * yoda_gs_begin_window's, scored against the CURRENT node state with the window's phase-1
 * masks and maxima): each list's threshold becomes its refresh-time k-th score.  Every listed
 * node is validated first (YODA_ERR_RANGE leaves the session unchanged); capacity sessions
 * restart windows instead and get YODA_ERR_STATE. */
int yoda_gs_refresh(yoda_gs_t* g, uint32_t from, const double* top_score,
                    const uint32_t* top_node);
/* YODA_GREEDY_CARD_CAPACITY: the size of the window that a restart at window index `progress`
 * opens (130 % of the progress in whole waves, at least 64, at most wmax) -- the one rule of
 * yoda_greedy, yoda_comm_greedy and the Python driver. */
uint32_t yoda_greedy_next_window(uint32_t progress, uint32_t wmax);
/* Nodes whose state changed since the last call (at most cap), with their current state. */
int yoda_gs_take_dirty(yoda_gs_t* g, uint32_t cap, uint32_t* nodes, uint64_t* alloc,
                       uint64_t* card_number, uint32_t* count);
/* Every node the session ever changed, with its ORIGINAL state (to restore the shards). */
int yoda_gs_touched_original(const yoda_gs_t* g, uint32_t cap, uint32_t* nodes, uint64_t* alloc,
                             uint64_t* card_number, uint32_t* count);
/* pick [P] in input order; pods certified from candidate lists; pods assigned by the caller. */
int yoda_gs_picks(const yoda_gs_t* g, int32_t* pick, uint32_t* resolved, uint32_t* assigned);

#ifdef __cplusplus
}
#endif

#endif /* YODA_H_ */
