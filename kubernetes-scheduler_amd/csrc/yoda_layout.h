// yoda_layout.h — device-resident data layout shared by the HIP kernels and the host side
// of libyoda.  See DESIGN.md §Data layout in HBM.
//
// Node records are array-of-structs, one record per node, because every wavefront walks
// the nodes in lock-step and reads a node's record through the SCALAR path (s_load into
// SGPRs, broadcast to all 64 lanes = 64 pods).  Inside a record the card fields are
// grouped field-major so the feasibility sweep touches only the first two groups.
#pragma once
#include <stdint.h>

namespace yoda {

constexpr int kBlock = 256;             // threads per workgroup = 4 waves = 256 pods
constexpr int kWave = 64;
constexpr uint32_t kChunkAlign = 64;    // node-chunk granularity (one K1 node block)

// Three exact record formats, chosen per snapshot by the host:
//   N32  every card field <= 0xFFFFFFFE (memory beyond that: ranks, MemTab) and the card score
//        below 2^32 / K: K1 runs on u32, every K2 quotient in f64 (300 x + M < 2^53: the
//        quotient lemma; tools/check_div_lemma.c), the card score accumulates in u32.
//   F64  every card field <= 2^44 and every score < 2^52: everything in exact f64.
//   U64  anything else: Go's uint64 wrap-around arithmetic verbatim.
enum class Path : int { N32 = 0, F64 = 1, U64 = 2 };
constexpr uint64_t kFastFieldMax = 1ull << 44;
constexpr uint64_t kFastScoreMax = 1ull << 52;
constexpr uint64_t kN32FieldMax = 0xFFFFFFFEull;
// bandwidth, clock, core, power <= this: 301 * 55738 < 2^24, the f32 quotient lemma holds
constexpr uint64_t kF32SmallMax = 55738;

// Record header of the fast path (32 B).  Cards follow: 6 groups of K doubles:
//   free[K], clock[K], total[K], bandwidth[K], core[K], power[K].
struct alignas(16) NodeHdrF {
  double static_score;    // CalculateAllocateScore + CalculateActualScore (exact)
  uint64_t card_number;   // Status.CardNumber
  uint32_t healthy_mask;  // bit j: card j Healthy
  uint32_t zero_total;    // Status.TotalMemorySum == 0 (reference panics if scored)
  uint32_t real_mask;     // bit j: j < len(CardList) (slots beyond are padding)
  uint32_t flags;         // kNodeUniform4, ...
};
// Every real card of the node has the same clock, bandwidth, core and power (one GPU
// model per node, the common case): K1 takes those maxima once per node and K2 computes
// their quotients once per node (N32 path).
constexpr uint32_t kNodeUniform4 = 1u;
// ... and also the same TotalMemory on every real card: the total-memory maximum and
// quotient are per node too.
constexpr uint32_t kNodeUniformTotal = 2u;
static_assert(sizeof(NodeHdrF) == 32, "NodeHdrF layout");

// Generic (exact uint64) path: same shape with uint64 card fields.
struct alignas(16) NodeHdrG {
  uint64_t static_score;  // (Allocate + Actual) mod 2^64
  uint64_t card_number;
  uint32_t healthy_mask;
  uint32_t zero_total;
  uint32_t real_mask;
  uint32_t flags;
};
static_assert(sizeof(NodeHdrG) == 32, "NodeHdrG layout");

enum CardField { kFree = 0, kClock = 1, kTotal = 2, kBandwidth = 3, kCore = 4, kPower = 5 };
constexpr int kCardFields = 6;

// F64 / U64 record: header + 6 groups of K 8-byte fields in CardField order.
__host__ __device__ constexpr uint32_t node_stride(int k) { return 32u + 48u * (uint32_t)k; }

// N32 record: header (NodeHdrF) + 6 groups of K u32 in CardField order (K1, the K2 card
// predicate and the small-field quotients) + 2 groups of K f64 {free, total}: the memory
// values (memory ranks: the u32 groups hold ranks) for the K2 quotients.
__host__ __device__ constexpr uint32_t n32_stride(int k) { return 32u + 40u * (uint32_t)k; }
__host__ __device__ constexpr uint32_t n32_u32_off(int field, int k) {
  return 32u + 4u * (uint32_t)(field * k);
}
enum N32F64 { kF64Free = 0, kF64Total = 1 };
__host__ __device__ constexpr uint32_t n32_f64_off(int g, int k) {
  return 32u + 24u * (uint32_t)k + 8u * (uint32_t)(g * k);
}

// K1 node summary (N32 path): the Filter / PreScore facts of one node in a few u32 words,
// read by the block-classified K1 with lane = node (k1_block_n32).  One record per node,
// k1sum_stride(K) bytes, words:
//   cn_lo, cn_hi      Status.CardNumber
//   clock             the clock of every real card (valid when kSumUni4)
//   meta              kSumUni4 | kSumUniTotal | kSumZeroTotal | (healthy count << 8)
//   mrf1              1 + max FreeMemory over the real cards (0: empty CardList)
//   total, bw, core, power   the per-node values (valid under kSumUni4 / kSumUniTotal)
//   hfs[K]            1 + FreeMemory of the HEALTHY cards, sorted descending, 0-padded:
//                     #healthy cards with free >= m  >= need  <=>  hfs[need-1] > m
enum K1SumWord {
  kSumCnLo = 0, kSumCnHi = 1, kSumClock = 2, kSumMeta = 3, kSumMrf1 = 4, kSumTotal = 5,
  kSumBw = 6, kSumCore = 7, kSumPower = 8, kSumHfs = 12
};
constexpr uint32_t kSumUni4 = 1u, kSumUniTotal = 2u, kSumZeroTotal = 4u;
__host__ __device__ constexpr uint32_t k1sum_stride(int k) {
  return (48u + 4u * (uint32_t)k + 15u) & ~15u;
}

// K2 node summary (N32 path), read by the block K2 (k2_block_n32) with lane = node and, for
// single nodes, through the scalar path.  k2sum_stride(K) bytes, u32 words:
//   static (f64, words 0-1)   CalculateAllocateScore + CalculateActualScore
//   clock, meta, bw, core, power   meta = kSumUni4 | (len(CardList) << 8)
//   fs[K]   FreeMemory of the REAL cards, sorted descending (0-padded)
//   ts[K]   TotalMemory of the same cards, in the same order
// The qualifying cards of a one-model node (algorithm.go:271) are then a prefix of that
// order: nq(m) = #{fs >= m} (capped at len(CardList)).
//   minclk  the lowest clock over the REAL cards (0xFFFFFFFF: empty CardList)
enum K2SumWord { kS2Static = 0, kS2Clock = 2, kS2Meta = 3, kS2Bw = 4, kS2Core = 5, kS2Power = 6,
                 kS2MinClk = 7, kS2Fs = 8 };
__host__ __device__ constexpr uint32_t k2sum_stride(int k) { return 32u + 8u * (uint32_t)k; }

// Block summary (N32 path): bounds over the REAL nodes of one 64-node block of a summary
// order (the snapshot order, or the block-grouped copy's), so that the block K1 can decide
// whole blocks for a wave -- every node NONE, or every node ALL with one maxima contribution
// -- before any per-node work, 64 blocks at a time (lane = block).  u32 words, stored in tiles
// of 64 blocks word-major like the node summaries (sum_index(block, word, bsum_stride(K))):
//   cn_min, cn_max      CardNumber bounds, saturated to 32 bits (0xFFFFFFFF: >= that);
//                       k_set_static keeps them valid bounds with atomics, k_bsum_cn makes
//                       them tight again
//   flags    kBsOneModel: every node one GPU model with one TotalMemory (kSumUni4|UniTotal);
//            kBsUni4: every node kSumUni4
//   ck_min, ck_max      the nodes' clock (one-model nodes) / card clocks (others)
//   hck_min, hck_max    the clocks of the HEALTHY cards (~0 / 0: none)
//   nh_min, nh_max      healthy cards per node
//   mrf_min, mrf_max    1 + max FreeMemory per node (K1Sum mrf1)
//   nreal, nzt          real nodes in the block, of them TotalMemorySum == 0
//   mx[6]   per MaxValue field (kMax* order) the max over the nodes of the contribution a
//           one-model node makes when some card qualifies (its model values, max free)
//   wc[6]   nodes reaching mx[f];  wl[6]  the lowest of them (offset in the block)
//   sat      the min over the nodes of 1 + the free of the card (in descending free order)
//            where the prefix maxima of the six MaxValue fields reach the node's all-card
//            maxima: a pod with scv/memory m < sat (and scv/clock <= every card's clock)
//            qualifies that prefix, so every node contributes its all-card maxima (one-model
//            nodes of one TotalMemory: 1 + max free, as mrf)
//   hc[4]    per distinct HEALTHY-card clock of the block (flags: kBsHcTab, entries << 8):
//            clock | (min over the nodes of their healthy cards of that clock << 16) | (max << 24)
//   tmin[K], tmax[K]    bounds of hfs[k] (K1Sum: 1 + free of the k-th healthy card by free)
// mx[6] of a node that is not one model with one TotalMemory: its all-card maxima.
enum BlockSumWord {
  kBsCnMin = 0, kBsCnMax = 1, kBsFlags = 2, kBsCkMin = 3, kBsCkMax = 4, kBsHckMin = 5,
  kBsHckMax = 6, kBsNhMin = 7, kBsNhMax = 8, kBsMrfMin = 9, kBsMrfMax = 10, kBsNReal = 11,
  kBsNzt = 12, kBsMx = 13, kBsWc = 19, kBsWl = 25, kBsSat = 31, kBsHc = 32, kBsT = 36
};
constexpr uint32_t kBsOneModel = 1u, kBsUni4 = 2u, kBsHcTab = 4u;
__host__ __device__ constexpr uint32_t bsum_stride(int k) { return 4u * (kBsT + 2u * (uint32_t)k); }

// K2 block bounds (N32 path; waves whose reciprocals are the G table's): per 64-node block of a
// summary order, u32 words (kbub_stride(K) bytes a block), in tiles of 64 blocks word-major
// (sum_index(block, word, kbub_stride(K))) so that a wave reads 64 blocks' bounds coalesced:
//   ub[j]    (f64, words 2j, 2j + 1; j = 0..K)  the max over the block's real nodes of
//            static + B_G[min(j, len(CardList))] -- no pod with at most j qualifying cards on
//            every node of the block scores more there (basic <= B_G[nq], nq <= j)
//   fmax[k]  (u32, from word 2K + 2; k < K)  the max over the nodes of fs[k] (K2 summary): a
//            pod with scv/memory m qualifies at most #{k : fmax[k] >= m} cards on any of them
//   lv[l]    (f64, words kbub_lvl(K) + 2l, 2l + 1; l < kKbLevels)  the max over the block's real
//            nodes of static + B_G[nq(t_l)], nq(t) = min(#{fs >= t}, len(CardList)), at the
//            snapshot's free levels t_0 = 0 < t_1 < ... < t_{L-1} = 0xFFFFFFFF (kb_levels):
//            - an UPPER bound for a wave whose smallest scv/memory is >= t_l (each pod qualifies
//              at most nq(t_l) cards, B_G is non-decreasing in q): the argmax K2's pruning;
//            - a LOWER bound on every pod's best score for a wave whose largest scv/memory is
//              <= t_l when every node of the block is feasible for every pod of the wave (the
//              maximising node scores at least that for each of them): the block K1's seed.
// Built from the K2 summaries and the G table on the device (k_block_ub), again whenever the
// static scores changed (k_set_static).
constexpr uint32_t kKbLevels = 32;
__host__ __device__ constexpr uint32_t kbub_fmax(int k) { return 2u * (uint32_t)k + 2u; }
__host__ __device__ constexpr uint32_t kbub_lvl(int k) { return kbub_fmax(k) + (uint32_t)k; }
__host__ __device__ constexpr uint32_t kbub_stride(int k) {
  return (4u * (kbub_lvl(k) + 2u * kKbLevels) + 15u) & ~15u;
}

// K2 block bounds for waves whose maxima M are NOT the G maxima (N32 path, one reciprocal set;
// e.g. clock-labelled pods, whose feasible nodes are one GPU model): B_M has no table, so the
// bound decouples the basic score per card (algorithm.go:280-291) into its model part and its
// memory part, each bounded over the block's real nodes independently:
//   basic_M(n, q) <= q shared_M(n) + (300 / M_free) F_n[q] + (100 / M_total) T_n[q]
// (floor(x 100 / M) <= x r with r = RU(100 / M)), F / T the sums of free / total over the q
// cards of largest free.  u32 words, tiles of 64 blocks (sum_index(block, word, kbdec_stride)):
//   ok            1: every real node of the block is one GPU model (kSumUni4), values, not ranks
//   bw, ck, co, pw   the max over the block's nodes of the model values (shared_M is monotone)
//   stat (f64)    the max static score
//   ql[l]         the max over the nodes of nq(t_l) (kb_levels, as kbub's lv[])
//   fl[l] (f64)   the max over the nodes of the sum of the frees >= t_l
//   tl[l] (f64)   the max over the nodes of the sum of the totals of those cards
// so that static + nq shared + 3 r_free F + r_total T <= stat + ql shared(bw, ck, co, pw) +
// 3 r_free fl + r_total tl for every pod whose smallest scv/memory is >= t_l.
enum KbDecWord { kDecOk = 0, kDecBw = 1, kDecCk = 2, kDecCo = 3, kDecPw = 4, kDecStat = 5, kDecQl = 7 };
__host__ __device__ constexpr uint32_t kbdec_fl(uint32_t l) { return kDecQl + kKbLevels + 2u * l; }
__host__ __device__ constexpr uint32_t kbdec_tl(uint32_t l) { return kDecQl + 3u * kKbLevels + 2u * l; }
__host__ __device__ constexpr uint32_t kbdec_stride() {
  return (4u * (kDecQl + 5u * kKbLevels) + 15u) & ~15u;
}

// Per-card GPU models of every node (N32 path), in the K2 summary's descending-free card order,
// read with lane = node by the block kernels for the nodes whose cards are not all one model
// (no kSumUni4): u32 words
//   ck[K], bw[K], co[K], pw[K]   Clock, Bandwidth, Core, Power of the j-th card in free order
//   hm                           bit j: that card is Healthy
// (zeros past len(CardList)).  Tile layout like the summaries (sum_index).
enum MixWord { kMixCk = 0, kMixBw = 1, kMixCo = 2, kMixPw = 3 };
__host__ __device__ constexpr uint32_t mix_word(int field, int j, int k) {
  return (uint32_t)(field * k + j);
}
__host__ __device__ constexpr uint32_t mix_hm(int k) { return 4u * (uint32_t)k; }
__host__ __device__ constexpr uint32_t mix_stride(int k) { return 4u * (4u * (uint32_t)k + 1u); }

// K1 tile of the nodes whose cards are not all one model (N32 path; read by k1_block_n32 with
// lane = node), REAL cards in the K2 summary's descending-free order, u32 words:
//   chg      bit q (1..K): the prefix maxima below differ between q - 1 and q cards (bit 1
//            whenever a card exists); bit 31: more than 4 distinct healthy-card clocks
//   ch[4]    clock | (healthy cards with that clock << 16), distinct clocks (0: unused)
//   pm[q-1]  for q = 1..K, the maxima over the first q cards of (clock | bandwidth << 16)
//            and (core | power << 16) per 16-bit half, and of TotalMemory (K2 summary code)
//   cd[t]    card t's (clock | bandwidth << 16), (core | power << 16)
// (a snapshot with such nodes keeps clock, bandwidth, core and power <= 65535: yoda_capi.cpp
// n32_ok.)  Tile layout
// like the summaries (sum_index).
enum K1MixWord { kX1Chg = 0, kX1Ch = 1, kX1Pm = 5 };
__host__ __device__ constexpr uint32_t x1_pm(int q1, int f) { return kX1Pm + 3u * (uint32_t)q1 + (uint32_t)f; }
__host__ __device__ constexpr uint32_t x1_cd(int t, int f, int k) {
  return kX1Pm + 3u * (uint32_t)k + 2u * (uint32_t)t + (uint32_t)f;
}
__host__ __device__ constexpr uint32_t x1_stride(int k) { return 4u * (kX1Pm + 5u * (uint32_t)k); }
constexpr uint32_t kX1ChgMany = 1u << 31;

// Both summaries are stored in tiles of 64 nodes, word-major inside a tile (AoSoA): word w
// of node n is u32 number sum_index(n, w, stride).  The block kernels read them with
// lane = node, so loading one word for 64 nodes is one contiguous 256-B access (2 cache
// lines) instead of 64 strided ones (a 16-B load over an 80-B stride touches 40 lines).
// The last tile is padded to 64 nodes (zeros; the kernels mask those lanes).
__host__ __device__ constexpr size_t sum_index(uint32_t n, uint32_t w, uint32_t stride) {
  return ((size_t)(n >> 6) * (stride / 4u) + w) * 64u + (n & 63u);
}
__host__ __device__ constexpr size_t sum_words(uint32_t n_nodes, uint32_t stride) {
  return (size_t)((n_nodes + 63u) >> 6) * 64u * (stride / 4u);
}

// Feasibility bitmask: one u64 per (pod wave, node), bit l = pod 64 w + l (in the order the
// kernels see the pods) feasible on node n, at bm[w * bm_stride + n]; bm_stride = N rounded
// up to 64.  K1 writes it coalesced (lane = node); K2 reads one wave's mask per node through
// the scalar path and skips the node when it is 0.
__host__ __device__ constexpr uint32_t bm_row(uint32_t n_nodes) { return (n_nodes + 63u) & ~63u; }
// Sparse form written by the block-classified K1 (N32 path), so the [wave][node] array is
// not streamed through HBM in full: per (pod wave, 64-node block) one BlockMask,
//   nz   bit j: node 64 b + j has a feasible pod of the wave,
//   full bit j: every live pod of the wave is feasible on it (mask == the wave's live mask),
// at bs[w * bs_row(N) + b], written for every block of the wave's chunks; bm[w][n] is then
// written (and read) only for the PARTIAL nodes, nz & ~full.  Mask of (w, n):
//   full ? live(w) : nz ? bm[w][n] : 0.
struct alignas(16) BlockMask {
  uint64_t nz, full;
};
__host__ __device__ constexpr uint32_t bs_row(uint32_t n_nodes) { return (n_nodes + 63u) / 64u; }
// Non-empty node blocks: u64 blk[wave][w], bit b % 64 of word b / 64 set when node block b
// (nodes 64 b .. 64 b + 63) has a feasible pod of the wave.  Written by the block K1, read by
// the block K2 to visit only those blocks.
__host__ __device__ constexpr uint32_t blk_row(uint32_t n_nodes) {
  return ((n_nodes + 63u) / 64u + 63u) / 64u;
}

// The block-grouped copies of the node summaries (private batch runs) that k_set_static keeps
// current with the originals: inv[node] = its internal position.
struct PermCopy {
  const uint32_t* inv = nullptr;
  unsigned char* sum = nullptr;
  unsigned char* sum2 = nullptr;
  // and the block summaries' CardNumber bounds (BlockSumWord), of the snapshot order and of
  // the block-grouped order, widened with atomics so that they stay valid bounds
  uint32_t* bsum = nullptr;
  uint32_t* bsum_p = nullptr;
  uint32_t bsum_words = 0;  // bsum_stride(K) / 4
};

// Mode B node record: V = Cpu/100, U = DiskIO/50 (algorithm.go:71,73).
struct alignas(16) NodeRecB {
  double v, u;
};

// Mode B score levels.  With d = alpha*V - beta*U (algorithm.go:109), the score
// trunc(10 - 10*|d|) (>= 1, else 0; :110-111 then Uint64ToInt64) is a non-increasing function
// of |d| under IEEE rounding (each operation is monotone), so score >= k  <=>  |d| <= t[k] for
// k = 1..10; t[11] = -1 (no level above 10), t[0] unused.  Computed once on the host by
// bisection over the double bit patterns (yoda_capi.cpp diskio_levels).
struct DiskLevels {
  double t[12];
};
// Mode B per (node chunk, pod class) partial: level << 28 | nodes at that level in the chunk.
constexpr uint32_t kDiskCountBits = 28;
// Mode B batch launch plan (yoda_kernels.hip diskio_plan): C chunks of `chunk` nodes.
struct DiskPlan {
  uint32_t chunk, C;
  bool node_lanes;
};

// One pod evaluated alone against the CURRENT node state (greedy fallbacks), lane = node:
// its Filter / card-predicate operands, passed by value (yoda_kernels.hip k_one_*).
struct OnePod {
  uint64_t number;            // PodFitsNumber operand: label value or 1
  uint32_t need_mem, need_clk;  // healthy cards required (0: label absent)
  uint32_t m32, c32;          // N32 thresholds (clamped to 0xFFFFFFFF)
  double mf, cf;              // F64 thresholds (clamped to 2^53)
};
// Results of the two k_one_* launches (device, then copied to the host in one piece).
struct alignas(16) OneOut {
  uint64_t maxima[6];         // PreScore maxima, MaxValue order (floor 1)
  uint32_t nf, nz, first, pad;  // feasible nodes, of them TotalMemorySum == 0, lowest one
  double rcp[5];              // RU(100/M): bw, core, power, free, total
  double best, low;           // highest / lowest raw score over the feasible nodes
  uint32_t idx, ties;         // lowest node reaching best, nodes reaching it
};

// Multi-GPU step inside libyoda (yoda_comm_*): a shard's per-pod result of phase 2, all-
// gathered across ranks (global node index; best / low as int64 raw scores).
struct alignas(8) ShardRec {
  int64_t best;       // highest raw score over the shard's feasible nodes (-1: none)
  uint32_t idx, ties; // lowest global node reaching it, nodes reaching it
  int64_t low;        // lowest raw score (INT64_MAX: none)
};
static_assert(sizeof(ShardRec) == 24, "ShardRec layout");
// Up to this many handles share one in-process exchange (yoda_comm_run_local).
constexpr int kMaxLocalShards = 16;
struct PtrList {
  const void* p[kMaxLocalShards];
};

// Per-pod device parameters (struct of arrays, length P each).
// The "G table" of an N32 snapshot (yoda_kernels.hip k_gtable / k2_block_n32): per-node terms
// under the snapshot-wide maxima G, and G's reciprocals (f64 bw, core, power, free, total).
struct GTab {
  const uint32_t* tab;
  double r_bw, r_core, r_pow, r_free, r_tot;
  float f_bw, f_core, f_pow;  // RU32 of r_bw, r_core, r_pow (the f32-quotient block K2's)
};
__host__ __device__ constexpr uint32_t gtab_stride(int k) { return 4u * (uint32_t)k; }

// Memory ranks (N32 snapshots whose FreeMemory / TotalMemory exceed 32 bits, e.g. bytes): the
// u32 memory fields of the records and summaries hold RANKS instead of values -- free ->
// 2 + its index among the snapshot's distinct card frees (ascending), total -> 2 + its index
// among the distinct totals -- and scv/memory becomes 2 + #{distinct frees < m}, so every
// comparison free >= m, every max and every sort order is unchanged.  vf[r] / vt[r] give the
// value of rank r (index 0, 1: 0).  Values are needed only for the quotients (CalculateCard
// Score) and the maxima themselves: a maximum of rank r is max(1, v[r]) (r < 2: the floor
// 1 of collection.go:31-38).  vf == nullptr: plain values.
struct MemTab {
  const double* vf = nullptr;
  const double* vt = nullptr;
  uint32_t nf = 0;  // distinct card frees (vf[2 .. nf + 1])
};

struct PodParams {
  // Filter / card predicate thresholds
  double* m_f;         // fast: scv/memory clamped to 2^53 (0 if absent)
  double* c_f;         // fast: scv/clock clamped to 2^53 (0 if absent)
  uint64_t* m_u;       // generic: scv/memory (0 if absent)
  uint64_t* c_u;       // generic: scv/clock  (0 if absent)
  uint32_t* m_32;      // narrow: scv/memory clamped to 0xFFFFFFFF
  uint32_t* c_32;      // narrow: scv/clock clamped to 0xFFFFFFFF
  uint64_t* number;    // PodFitsNumber operand: label value or 1
  uint32_t* need_mem;  // healthy cards with free >= m required (0 if label absent)
  uint32_t* need_clk;  // healthy cards with clock == c required (0 if label absent)
  // Mode B
  double* alpha;
  double* beta;
  // the snapshot's G table (N32 with node summaries; tab == nullptr: none)
  GTab g = {};
  // the snapshot's per-card models in free order (N32; yoda_layout.h MixWord)
  const uint32_t* mix = nullptr;
  // the snapshot's K1 tile of mixed-model nodes (N32; yoda_layout.h K1MixWord)
  const uint32_t* x1 = nullptr;
  // every node of the snapshot is one GPU model with one TotalMemory (N32: the K1 without
  // per-card branches serves it)
  bool one_model = false;
  // every node of the snapshot is one GPU model (kSumUni4; N32: the K2 without mixed rows)
  bool all_uni4 = false;
  // private runs over the block-grouped node order (yoda_capi.cpp node_perm): the local node
  // id of each internal position (the argmax ties compare these, not positions); nullptr: none
  const uint32_t* ids = nullptr;
  // the snapshot's memory ranks (MemTab; vf == nullptr: none)
  MemTab mt = {};
  // 64-node block summaries of the order the run visits (BlockSumWord; nullptr: none)
  const uint32_t* bsum = nullptr;
  // K2 block bounds of that order (kbub_stride; nullptr: none -- the argmax K2 prunes with them)
  const uint32_t* kbub = nullptr;
  // the blocks of that order with the highest bounds (bit words, as the K1 block list)
  const uint64_t* hot = nullptr;
  // the block K1's partial words: kNarrowWords (small fields <= kPack16Max) or kWideWords
  uint32_t nwords = 4;
  // the block K2's small-field quotients in f32 (every small field <= kF32SmallMax), else f64
  bool q32 = true;
  // heaviest-first pod blocks: K1 adds per-wave weights into lpt_w, k_lpt_order sorts them into
  // lpt_order, the argmax block K2 visits its pod blocks in that order (nullptr: none)
  uint32_t* lpt_w = nullptr;
  const uint32_t* lpt_order = nullptr;
  // the block K1's heaviest-first pod blocks (k1_probe + k_lpt_order; nullptr: launch order)
  const uint32_t* k1_order = nullptr;
  // K2 pruning seeds [waves] u64 (zeroed with the block list before the block K1): a lower
  // bound on every live pod's best raw score under the G maxima, found by the block K1 on the
  // nodes every pod of the wave passes (nullptr: none); the snapshot's free levels kb_levels
  // [kKbLevels] of the kbub lv[] bounds; kbub_exact: those bounds are current (not loose), so
  // the block K1 may take seeds from them
  uint64_t* seed = nullptr;
  const uint32_t* kb_levels = nullptr;
  bool kbub_exact = false;
  // the non-G block bounds (kbdec_*) of the order the run visits (nullptr: none), and the
  // argmax K2's per-pod best so far shared across its node chunks ([P] u64: score + 1, zeroed
  // with the block list; nullptr: none)
  const uint32_t* kbdec = nullptr;
  uint64_t* gbest = nullptr;
  // per pod wave a bit per node chunk that wrote its partials (K1: some pod has a feasible
  // node there; the argmax K2: some pod may hold its pick or a tie there): the reduces read
  // only those chunks (<= 48 chunks, the plain reduces; nullptr: every chunk writes)
  uint64_t* cmask1 = nullptr;
  uint64_t* cmask2 = nullptr;
};

// Per-pod state produced between kernels (length P each unless noted).
struct PodState {
  uint64_t* maxima;    // [6][P] MaxValue in collection.go field order (see kMax* below)
  uint32_t* counts;    // [2][P] n_feasible, n_zero_total
  double* rcp;         // [5][P] RU(100 / M) for bw, core, power, free, total (f64)
  int64_t* best;       // [P] highest raw score over feasible nodes (-1: none)
  uint32_t* idx;       // [P] lowest global node index reaching it
  uint32_t* ties;      // [P] nodes reaching it
  int64_t* lowest;     // [P] lowest raw score over feasible nodes (INT64_MAX: none)
  int32_t* pick;       // [P]
  int32_t* status;     // [P]
  uint32_t* flagged;   // [P] generic path: pods needing the exact normalize
  uint32_t* n_flagged; // [1]
};

// MaxValue field order (collection.go:14-21) used for the [6][P] maxima buffer.
enum MaxField { kMaxBw = 0, kMaxClock = 1, kMaxCore = 2, kMaxFree = 3, kMaxPower = 4, kMaxTotal = 5 };

// Chunk partials: [field][chunk][P].  The block K1 (N32) writes its maxima as u32 words, read
// back by k_reduce1<true>: packed into kNarrowWords (bandwidth | clock << 16, core | power << 16,
// free, total) when the four small fields are <= 65535, else kWideWords (one per field).
constexpr uint32_t kNarrowWords = 4;
constexpr uint32_t kWideWords = 6;
constexpr uint64_t kPack16Max = 0xFFFF;
struct Partials {
  uint64_t* max_u;     // [6][C][P]
  uint32_t* cnt;       // [2][C][P]
  double* best_f;      // [C][P]
  int64_t* best_i;     // [C][P] (generic; also used for exact normalize)
  uint32_t* idx;       // [C][P]
  uint32_t* ties;      // [C][P]
  double* low_f;       // [C][P]
  int64_t* low_i;      // [C][P]
  uint32_t* err;       // [C][P] exact normalize: score out of range seen
};

// Per-pod array table for the batch permutation (yoda_order.hip).
constexpr int kPermArrays = 16;
// Counting-sort pod order (yoda_order.hip): the batch's distinct group keys (ascending;
// key = clock24 << 9 | number8 << 1 | has-memory), each group's first sorted position, and
// the memory buckets per group (1 << nb_log2; bucket = min(m, 2^32 - 1) >> m_shift).
struct OrderMeta {
  const uint64_t* groups;
  const uint32_t* gstart;
  uint32_t n_groups, nb_log2, m_shift;
  const uint32_t* m32 = nullptr;  // memory ranks: the pods' rank thresholds (MemTab)
};

// k_finalize of an ordered run: the caller-order outputs (perm == nullptr: none, the
// outputs stay in sorted order); n_out = caller pods, the row stride of counts / maxima.
struct FinalScatter {
  const uint32_t* perm;
  uint32_t n_out;
  uint32_t* counts;          // [2][n_out]
  int64_t* best;             // [n_out]
  uint64_t* maxima;          // [6][n_out], or none (left in sorted order)
  const uint64_t* maxima_in; // [6][n_pods] sorted
};

struct PermTable {
  const void* src[kPermArrays];
  void* dst[kPermArrays];
  uint32_t bytes[kPermArrays];
  uint32_t n;
};

}  // namespace yoda
