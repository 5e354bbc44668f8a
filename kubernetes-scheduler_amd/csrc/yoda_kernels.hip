// yoda_kernels.hip — CDNA4 (gfx950) kernels of the Yoda Filter/Score hot path.
//
// Mapping: one LANE = one POD, one workgroup = 256 pods, grid.y = node
// chunks.  Every wave walks its node chunk in lock-step; the node record's address is
// wave-uniform, so it is read through the scalar path (s_load -> SGPR) and broadcast to the
// 64 pods, while each lane keeps its pod's thresholds / reciprocals and running reductions
// in VGPRs.  Per-pod reductions (maxima, argmax, ties, min) therefore never cross lanes
// inside the hot loop; chunk partials are merged by small per-pod kernels.
//
//   K1  k1_filter_maxima   filter.go:11-58 + collection.go:30-76  (feasibility bitmask,
//                          n_feasible, per-pod maxima)
//   K2  k2_score_*         algorithm.go:264-310 composed as :96, scheduler.go:154,
//                          argmax/ties/min for NormalizeScore + selectHost
//   K2B k2_diskio          algorithm.go:99-119 (live Mode B)
//   K3  k3_exact_normalize scheduler.go:176-179 with int64 wrap (generic path only)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "yoda_layout.h"

// The YODA_ABL_* ablations remove work whose results the path needs (written masks, summaries,
// whole classes): counter and timing builds only.  They compile only beside the A/B knobs
// (tools/build_ab.sh), never into a release libyoda.
#if !defined(YODA_AB_KNOBS) &&                                                         \
    (defined(YODA_ABL_K1_NOGEN) || defined(YODA_ABL_K1_NOHC) || defined(YODA_ABL_K1_NOPART) || \
     defined(YODA_ABL_K1_NOBS) || defined(YODA_ABL_K1_NOBM))
#error "YODA_ABL_* ablations give wrong results: build them with -DYODA_AB_KNOBS (tools/build_ab.sh)"
#endif

#pragma clang fp contract(off)

namespace yoda {

constexpr int64_t kI64Max = 0x7fffffffffffffffll;

static inline dim3 pod_grid(uint32_t n) { return dim3((n + kBlock - 1) / kBlock); }

// Record policies (yoda_layout.h): field type of the K1 sweep and where its groups live.
template <Path P>
struct Rec;
template <>
struct Rec<Path::N32> {
  using T = uint32_t;
  static constexpr uint32_t stride(int k) { return n32_stride(k); }
  static constexpr uint32_t off(int field, int k) { return n32_u32_off(field, k); }
};
template <>
struct Rec<Path::F64> {
  using T = double;
  static constexpr uint32_t stride(int k) { return node_stride(k); }
  static constexpr uint32_t off(int field, int k) { return 32u + 8u * (uint32_t)(field * k); }
};
template <>
struct Rec<Path::U64> {
  using T = uint64_t;
  static constexpr uint32_t stride(int k) { return node_stride(k); }
  static constexpr uint32_t off(int field, int k) { return 32u + 8u * (uint32_t)(field * k); }
};

// K values of one card-field group, read with ONE wide scalar load (the address is
// wave-uniform), so a node costs a handful of s_load_dwordx8/x16 and one wait.
template <class T, int K>
struct alignas(sizeof(T) >= 4 ? sizeof(T) : 4) Group {
  T v[K];
};
template <class T, int K>
__device__ __forceinline__ Group<T, K> load_group(const unsigned char* p) {
  return *reinterpret_cast<const Group<T, K>*>(p);
}

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// Memory ranks (yoda_layout.h MemTab): a maximum in rank space -> its value: max(1, v[r]), the CollectMaxValues floor for r < 2.
__device__ __forceinline__ uint64_t rank_value(uint64_t r, const double* v) {
  if (r < 2u) return 1u;
  const uint64_t x = (uint64_t)v[r];
  return x > 1u ? x : 1u;
}

// max of two non-NaN doubles in ONE v_max_f64.  fmax() under the default IEEE mode first
// canonicalizes both operands (two extra v_max_f64 per call); card fields and maxima are
// exact non-negative integers, never NaN, so the canonicalization is dead work.
// x must be wave-uniform (a node-record field read through the scalar path).
__device__ __forceinline__ double dmax(double acc, double x) {
  double r;
  asm volatile("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(acc), "s"(x));  // x: uniform (SGPR)
  return r;
}
__device__ __forceinline__ uint32_t fmax_t(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ double fmax_t(double a, double b) { return dmax(a, b); }
__device__ __forceinline__ uint64_t fmax_t(uint64_t a, uint64_t b) { return umax64(a, b); }

// ---------------------------------------------------------------------------------------
// K1: Filter (PodFitsNumber ∧ PodFitsMemory ∧ PodFitsClock, collection.go:41-44) and the
// PreScore maxima (CollectMaxValues).  k1_node evaluates ONE node record for every pod lane
// of the wave: it returns the lane's feasibility and folds the node into the lane's maxima
// and counts.  Branch-free in the card loop: a short-circuit `healthy && free >= m` would
// make every field load conditional and serialise one scalar-load round trip per card.
template <int K, Path PATH>
__device__ __forceinline__ bool k1_node(const unsigned char* rec, typename Rec<PATH>::T m,
                                        typename Rec<PATH>::T c, uint64_t number,
                                        uint32_t need_mem, uint32_t need_clk,
                                        typename Rec<PATH>::T (&mx)[6], uint32_t& nf,
                                        uint32_t& nz) {
  using R = Rec<PATH>;
  using T = typename R::T;
  const NodeHdrG hd = *reinterpret_cast<const NodeHdrG*>(rec);
  const Group<T, K> fr = load_group<T, K>(rec + R::off(kFree, K));
  const Group<T, K> ck = load_group<T, K>(rec + R::off(kClock, K));
  // one GPU model on the node (scalar flag, so the branch is wave-uniform)
  bool uniform = false;
  if constexpr (PATH == Path::N32) uniform = (hd.flags & kNodeUniform4) != 0u;
  uint32_t cm = 0, cc = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t hj = (hd.healthy_mask >> j) & 1u;
    cm += (uint32_t)(fr.v[j] >= m) & hj;   // CardFitsMemory (filter.go:52-54)
  }
  if (uniform) {
    // every real card has clock ck[0]: CardFitsClock counts all healthy cards or none
    cc = (ck.v[0] == c) ? (uint32_t)__builtin_popcount(hd.healthy_mask) : 0u;
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j)
      cc += (uint32_t)(ck.v[j] == c) & ((hd.healthy_mask >> j) & 1u);  // filter.go:56-58
  }
  const bool feas = (number <= hd.card_number) & (cm >= need_mem) & (cc >= need_clk);
  if (feas && uniform) {
    ++nf;
    nz += hd.zero_total;
    // qualifying cards (collection.go:46) = real cards with free >= m, if clock >= c
    if (ck.v[0] >= c) {
      uint32_t any = 0;
      if (hd.flags & kNodeUniformTotal) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const uint32_t q = ((hd.real_mask >> j) & 1u) & (uint32_t)(fr.v[j] >= m);
          mx[kMaxFree] = fmax_t(mx[kMaxFree], q ? fr.v[j] : T(0));
          any |= q;
        }
      } else {
        const Group<T, K> to = load_group<T, K>(rec + R::off(kTotal, K));
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const uint32_t q = ((hd.real_mask >> j) & 1u) & (uint32_t)(fr.v[j] >= m);
          mx[kMaxFree] = fmax_t(mx[kMaxFree], q ? fr.v[j] : T(0));
          mx[kMaxTotal] = fmax_t(mx[kMaxTotal], q ? to.v[j] : T(0));
          any |= q;
        }
      }
      if (any) {
        const T* g = reinterpret_cast<const T*>(rec);
        if (hd.flags & kNodeUniformTotal)
          mx[kMaxTotal] = fmax_t(mx[kMaxTotal], g[R::off(kTotal, K) / sizeof(T)]);
        mx[kMaxBw] = fmax_t(mx[kMaxBw], g[R::off(kBandwidth, K) / sizeof(T)]);
        mx[kMaxClock] = fmax_t(mx[kMaxClock], ck.v[0]);
        mx[kMaxCore] = fmax_t(mx[kMaxCore], g[R::off(kCore, K) / sizeof(T)]);
        mx[kMaxPower] = fmax_t(mx[kMaxPower], g[R::off(kPower, K) / sizeof(T)]);
      }
    }
  } else if (feas) {
    ++nf;
    nz += hd.zero_total;
    const Group<T, K> bw = load_group<T, K>(rec + R::off(kBandwidth, K));
    const Group<T, K> co = load_group<T, K>(rec + R::off(kCore, K));
    const Group<T, K> pw = load_group<T, K>(rec + R::off(kPower, K));
    const Group<T, K> to = load_group<T, K>(rec + R::off(kTotal, K));
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if ((fr.v[j] >= m) & (ck.v[j] >= c)) {  // collection.go:46: no health check, >= clock
        mx[kMaxBw] = fmax_t(mx[kMaxBw], bw.v[j]);
        mx[kMaxClock] = fmax_t(mx[kMaxClock], ck.v[j]);
        mx[kMaxCore] = fmax_t(mx[kMaxCore], co.v[j]);
        mx[kMaxFree] = fmax_t(mx[kMaxFree], fr.v[j]);
        mx[kMaxPower] = fmax_t(mx[kMaxPower], pw.v[j]);
        mx[kMaxTotal] = fmax_t(mx[kMaxTotal], to.v[j]);
      }
    }
  }
  return feas;
}

// k1_node for the block-classified N32 K1's undecided MIXED-model nodes (one-model nodes are
// decided from the node summary there): the same predicates and maxima, but the maxima
// fields are read one card at a time, so the rare path holds ~2K + 6 SGPRs instead of 6K
// and does not push the whole kernel into SGPR spills.
template <int K>
__device__ __forceinline__ bool k1_node_lean(const unsigned char* rec, uint32_t m, uint32_t c,
                                             uint64_t number, uint32_t need_mem,
                                             uint32_t need_clk, uint32_t (&mx)[6], uint32_t& nf,
                                             uint32_t& nz) {
  const NodeHdrG hd = *reinterpret_cast<const NodeHdrG*>(rec);
  const uint32_t* g = reinterpret_cast<const uint32_t*>(rec + n32_u32_off(0, K));
  uint32_t cm = 0, cc = 0;
#pragma unroll 1
  for (int j = 0; j < K; ++j) {
    const uint32_t hj = (hd.healthy_mask >> j) & 1u, fj = g[kFree * K + j], cj = g[kClock * K + j];
    cm += (uint32_t)(fj >= m) & hj;   // CardFitsMemory (filter.go:52-54)
    cc += (uint32_t)(cj == c) & hj;   // CardFitsClock (filter.go:56-58)
  }
  const bool feas = (number <= hd.card_number) & (cm >= need_mem) & (cc >= need_clk);
  if (feas) {
    ++nf;
    nz += hd.zero_total;
#pragma unroll 1
    for (int j = 0; j < K; ++j) {
      const uint32_t fj = g[kFree * K + j], cj = g[kClock * K + j];
      if ((fj >= m) & (cj >= c)) {  // collection.go:46: no health check, >= clock
        mx[kMaxBw] = max(mx[kMaxBw], g[kBandwidth * K + j]);
        mx[kMaxClock] = max(mx[kMaxClock], cj);
        mx[kMaxCore] = max(mx[kMaxCore], g[kCore * K + j]);
        mx[kMaxFree] = max(mx[kMaxFree], fj);
        mx[kMaxPower] = max(mx[kMaxPower], g[kPower * K + j]);
        mx[kMaxTotal] = max(mx[kMaxTotal], g[kTotal * K + j]);
      }
    }
  }
  return feas;
}

__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
// per-16-bit-half maximum of two packed pairs (v_pk_max_u16)
__device__ __forceinline__ uint32_t max16x2(uint32_t a, uint32_t b) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  const us2 m = __builtin_elementwise_max(__builtin_bit_cast(us2, a), __builtin_bit_cast(us2, b));
  return __builtin_bit_cast(uint32_t, m);
}
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ uint32_t uniform_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  return (uint64_t)uniform_u32((uint32_t)v) | ((uint64_t)uniform_u32((uint32_t)(v >> 32)) << 32);
}
// Workgroup -> (pod block, node chunk), XCD-aware.  The grid is (pod blocks, chunks);
// workgroups are dealt round-robin over the 8 XCDs in linear order, so with C a multiple of
// 8 the linear id is remapped to give each XCD whole chunks (chunk % 8 == its slot), visited
// one chunk at a time across all pod blocks: the chunk's node records and summaries stay in
// that XCD's L2 while every pod block reads them.  Placement only affects speed.
struct Tile {
  uint32_t pb, chunk;
};
#ifndef YODA_TILE_POD_MAJOR
#define YODA_TILE_POD_MAJOR 1
#endif
__device__ __forceinline__ Tile tile() {
  const uint32_t PB = gridDim.x, C = gridDim.y;
  if ((C & 7u) != 0u) return {blockIdx.x, blockIdx.y};
  const uint32_t L = blockIdx.x + blockIdx.y * PB;
  const uint32_t i = L >> 3;
  // XCD (L & 7) owns chunks (L & 7) + 8 g.  Pod-major: it takes all its chunks of one pod
  // block before the next, so the pod block's parameters are read from HBM once per XCD
  // (its C / 8 chunks' node summaries -- ~1 MB -- stay in the XCD's 4 MB L2 meanwhile);
  // chunk-major walks one chunk across all pod blocks at a time.
  if (YODA_TILE_POD_MAJOR) {
    const uint32_t G = C >> 3;
    return {i / G, (i % G) * 8u + (L & 7u)};
  }
  return {i % PB, (i / PB) * 8u + (L & 7u)};
}

// Wave-wide reductions (every lane gets the result).  The block kernels run them in every
// (wave, chunk) task's set-up and epilogue -- ~20 per task, which at config 3's ~38k tasks per
// launch made them a large part of the fixed per-task cost -- so with the whole wave active
// they take no LDS round trip: the cross-row steps are the CDNA4 half/row swaps
// (v_permlane32_swap, v_permlane16_swap), the in-row steps DPP moves (row_ror:8,
// row_half_mirror, quad_perm), ~2 VALU each instead of a dependent ds_bpermute.  Step s pairs
// lane l with l ^ {32, 16, 8, 7, 2, 1}[s]: the six masks span the six lane bits, so after all
// six every lane holds the reduction over the wave, for any commutative, associative op.
// A wave with lanes switched off (exec partial: a DPP / permlane read of an off lane is not
// its value) takes the ds_bpermute butterfly instead.
__device__ __forceinline__ bool exec_full() { return __builtin_amdgcn_read_exec() == ~0ull; }
template <int S>
__device__ __forceinline__ uint32_t xlane_u32(uint32_t v) {
  if constexpr (S == 0) {  // l ^ 32
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32u) ? r[0] : r[1];
  } else if constexpr (S == 1) {  // l ^ 16
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16u) ? r[0] : r[1];
  } else if constexpr (S == 2) {  // l ^ 8: rotate the 16-lane row by 8
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);
  } else if constexpr (S == 3) {  // l ^ 7: mirror within each 8-lane half row
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);
  } else if constexpr (S == 4) {  // l ^ 2: quad_perm [2, 3, 0, 1]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);
  } else {  // l ^ 1: quad_perm [1, 0, 3, 2]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);
  }
}
template <int S>
__device__ __forceinline__ uint64_t xlane_u64(uint64_t v) {
  return (uint64_t)xlane_u32<S>((uint32_t)v) | ((uint64_t)xlane_u32<S>((uint32_t)(v >> 32)) << 32);
}
// op(v, partner) over the six steps (whole wave active), else the xor butterfly
template <class T, class Op>
__device__ __forceinline__ T wave_allreduce(T v, Op op) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit lanes");
  using U = std::conditional_t<sizeof(T) == 4, uint32_t, uint64_t>;
  auto x = [](T a, auto step) -> T {
    constexpr int S = decltype(step)::value;
    if constexpr (sizeof(T) == 4) return __builtin_bit_cast(T, xlane_u32<S>(__builtin_bit_cast(U, a)));
    else return __builtin_bit_cast(T, xlane_u64<S>(__builtin_bit_cast(U, a)));
  };
  if (exec_full()) {
    v = op(v, x(v, std::integral_constant<int, 0>{}));
    v = op(v, x(v, std::integral_constant<int, 1>{}));
    v = op(v, x(v, std::integral_constant<int, 2>{}));
    v = op(v, x(v, std::integral_constant<int, 3>{}));
    v = op(v, x(v, std::integral_constant<int, 4>{}));
    v = op(v, x(v, std::integral_constant<int, 5>{}));
    return v;
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const U u = (U)__shfl_xor(__builtin_bit_cast(std::conditional_t<sizeof(T) == 4, int, long long>, v), o, kWave);
    v = op(v, __builtin_bit_cast(T, u));
  }
  return v;
}
struct OpMaxU32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return max(a, b); } };
struct OpMaxU64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; } };
struct OpSumU32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpMaxF64 { __device__ double operator()(double a, double b) const { return fmax(a, b); } };
struct OpMinF64 { __device__ double operator()(double a, double b) const { return fmin(a, b); } };
struct OpMaxF32 { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  return uniform_u32(wave_allreduce(v, OpMaxU32{}));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return ~wave_max_u32(~v); }
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  return uniform_u64(wave_allreduce(v, OpMaxU64{}));
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) { return ~wave_max_u64(~v); }
// The same reductions left in VGPRs (every lane holds the result; the compiler does not know
// it is uniform): for wave bounds that are only VALU operands, so that a kernel with many of
// them does not run out of SGPRs (spills, lower occupancy).
__device__ __forceinline__ uint32_t wave_max_u32v(uint32_t v) { return wave_allreduce(v, OpMaxU32{}); }
__device__ __forceinline__ uint32_t wave_min_u32v(uint32_t v) { return ~wave_max_u32v(~v); }
__device__ __forceinline__ uint64_t wave_max_u64v(uint64_t v) { return wave_allreduce(v, OpMaxU64{}); }
__device__ __forceinline__ uint64_t wave_min_u64v(uint64_t v) { return ~wave_max_u64v(~v); }
__device__ __forceinline__ double wave_max_f64(double v) { return wave_allreduce(v, OpMaxF64{}); }
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) { return wave_allreduce(v, OpSumU32{}); }

// Lane j of (lo, hi) := the 64-bit wave mask b (j wave-uniform).
__device__ __forceinline__ void set_lane(uint32_t& lo, uint32_t& hi, uint64_t b, uint32_t j) {
  const bool me = lane_id() == j;
  lo = me ? (uint32_t)b : lo;
  hi = me ? (uint32_t)(b >> 32) : hi;
}

// Stores of the per-(wave, node) feasibility masks: lane j of (lo, hi) holds node nb + j.
__device__ __forceinline__ void bm_store(uint64_t* __restrict__ bm_row_w, uint32_t nb,
                                         uint32_t n_end, uint32_t lo, uint32_t hi) {
  const uint32_t n = nb + lane_id();
  if (n < n_end) bm_row_w[n] = ((uint64_t)hi << 32) | lo;
}

// K1, per-node sweep (F64 / U64 record paths): every wave evaluates every node of its chunk
// with k1_node; the wave's feasibility ballot of node n goes to lane n % 64 of (lo, hi) and
// 64 nodes' masks are stored with one coalesced store.
template <int K, Path PATH>
__global__ __launch_bounds__(kBlock) void k1_filter_maxima(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const typename Rec<PATH>::T* __restrict__ m_in, const typename Rec<PATH>::T* __restrict__ c_in,
    const uint64_t* __restrict__ number_in, const uint32_t* __restrict__ need_mem_in,
    const uint32_t* __restrict__ need_clk_in, uint32_t n_pods, uint64_t* __restrict__ pmax,
    uint32_t* __restrict__ pcnt, uint64_t* __restrict__ bm, uint32_t bm_stride) {
  using R = Rec<PATH>;
  using T = typename R::T;
  const Tile tl = tile();
  const uint32_t p = tl.pb * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk, C = gridDim.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  if (ballot(live) == 0) return;  // a wave past the batch: no bitmask row, no partials
  uint64_t* bmw = bm + (size_t)uniform_u32(p >> 6) * bm_stride;

  T m = 0, c = 0;
  uint64_t number = ~0ull;
  uint32_t need_mem = 0, need_clk = 0;
  if (live) {
    m = m_in[p];
    c = c_in[p];
    number = number_in[p];
    need_mem = need_mem_in[p];
    need_clk = need_clk_in[p];
  }
  T mx[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) mx[f] = T(1);  // floor 1 (collection.go:31-38)
  uint32_t nf = 0, nz = 0, lo = 0, hi = 0;
  for (uint32_t n = n0; n < n1; ++n) {
    const bool f = k1_node<K, PATH>(nodes + (size_t)n * R::stride(K), m, c, number, need_mem,
                                    need_clk, mx, nf, nz) && live;
    const uint64_t b = ballot(f);
    const int j = (int)(n & 63u);
    set_lane(lo, hi, b, (uint32_t)j);
    if (j == 63 || n + 1 == n1) bm_store(bmw, n & ~63u, n1, lo, hi);
  }
  if (!live) return;
#pragma unroll
  for (int f = 0; f < 6; ++f) pmax[((size_t)f * C + chunk) * n_pods + p] = (uint64_t)mx[f];
  pcnt[((size_t)0 * C + chunk) * n_pods + p] = nf;
  pcnt[((size_t)1 * C + chunk) * n_pods + p] = nz;
}

// K1 for the capacity-decrement greedy windows (YODA_GREEDY_CARD_CAPACITY, fast record
// paths): the per-node sweep of k1_filter_maxima, plus, per PreScore maxima field, the number
// of feasible nodes whose qualifying cards reach the pod's maximum and the lowest such node
// ("witnesses").  A pick only lowers CardNumber, so later pods of the window lose feasible
// nodes, never gain any; a maximum of CollectMaxValues (collection.go:30-76) can only move
// when every one of its witnesses is lost -- the host resolve checks that instead of
// re-evaluating the pod (greedy).  Dense masks, chunk partials
// pmax [6][C][P], pwit [2][6][C][P] (count, lowest local node), pcnt [2][C][P].
template <int K, Path PATH>
__global__ __launch_bounds__(kBlock) void k1_witness(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const typename Rec<PATH>::T* __restrict__ m_in, const typename Rec<PATH>::T* __restrict__ c_in,
    const uint64_t* __restrict__ number_in, const uint32_t* __restrict__ need_mem_in,
    const uint32_t* __restrict__ need_clk_in, uint32_t n_pods, uint64_t* __restrict__ pmax,
    uint32_t* __restrict__ pwit, uint32_t* __restrict__ pcnt, uint64_t* __restrict__ bm,
    uint32_t bm_stride) {
  using R = Rec<PATH>;
  using T = typename R::T;
  const Tile tl = tile();
  const uint32_t p = tl.pb * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk, C = gridDim.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  if (ballot(live) == 0) return;
  uint64_t* bmw = bm + (size_t)uniform_u32(p >> 6) * bm_stride;
  T m = 0, c = 0;
  uint64_t number = ~0ull;
  uint32_t need_mem = 0, need_clk = 0;
  if (live) {
    m = m_in[p];
    c = c_in[p];
    number = number_in[p];
    need_mem = need_mem_in[p];
    need_clk = need_clk_in[p];
  }
  T mx[6];
  uint32_t wc[6], wn[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    mx[f] = T(1);  // floor 1 (collection.go:31-38)
    wc[f] = 0u;
    wn[f] = 0xffffffffu;
  }
  uint32_t nf = 0, nz = 0, lo = 0, hi = 0;
  for (uint32_t n = n0; n < n1; ++n) {
    const unsigned char* rec = nodes + (size_t)n * R::stride(K);
    const NodeHdrG hd = *reinterpret_cast<const NodeHdrG*>(rec);
    const Group<T, K> fr = load_group<T, K>(rec + R::off(kFree, K));
    const Group<T, K> ck = load_group<T, K>(rec + R::off(kClock, K));
    uint32_t cm = 0, cc = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t hj = (hd.healthy_mask >> j) & 1u;
      cm += (uint32_t)(fr.v[j] >= m) & hj;  // CardFitsMemory (filter.go:52-54)
      cc += (uint32_t)(ck.v[j] == c) & hj;  // CardFitsClock (filter.go:56-58)
    }
    const bool feas =
        live && (number <= hd.card_number) & (cm >= need_mem) & (cc >= need_clk);
    bool uniform = false;  // one GPU model (scalar flag: a wave-uniform branch)
    if constexpr (PATH == Path::N32) uniform = (hd.flags & kNodeUniform4) != 0u;
    if (feas && uniform) {
      ++nf;
      nz += hd.zero_total;
      // the qualifying cards (collection.go:46) are the real cards with free >= m when the
      // common clock is >= c (padding slots hold zeros: they never raise a maximum, as in
      // k1_node); the four per-model fields are then the node's own, or 0 with no card
      auto vmax = [](T x, T y) { return x > y ? x : y; };  // per-lane operands
      T v[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};
      uint32_t any = 0;
      if (ck.v[0] >= c) {
        const T* g = reinterpret_cast<const T*>(rec);
        if (hd.flags & kNodeUniformTotal) {
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const uint32_t q = ((hd.real_mask >> j) & 1u) & (uint32_t)(fr.v[j] >= m);
            v[kMaxFree] = vmax(v[kMaxFree], q ? fr.v[j] : T(0));
            any |= q;
          }
          v[kMaxTotal] = any ? g[R::off(kTotal, K) / sizeof(T)] : T(0);
        } else {
          const Group<T, K> to = load_group<T, K>(rec + R::off(kTotal, K));
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const uint32_t q = ((hd.real_mask >> j) & 1u) & (uint32_t)(fr.v[j] >= m);
            v[kMaxFree] = vmax(v[kMaxFree], q ? fr.v[j] : T(0));
            v[kMaxTotal] = vmax(v[kMaxTotal], q ? to.v[j] : T(0));
            any |= q;
          }
        }
        v[kMaxBw] = any ? g[R::off(kBandwidth, K) / sizeof(T)] : T(0);
        v[kMaxClock] = any ? ck.v[0] : T(0);
        v[kMaxCore] = any ? g[R::off(kCore, K) / sizeof(T)] : T(0);
        v[kMaxPower] = any ? g[R::off(kPower, K) / sizeof(T)] : T(0);
      }
      if (any) {
#pragma unroll
        for (int f = 0; f < 6; ++f) {
          if (v[f] > mx[f]) {  // nodes in increasing order: the first witness is the lowest
            mx[f] = v[f];
            wc[f] = 1u;
            wn[f] = n;
          } else if (v[f] == mx[f]) {
            ++wc[f];
          }
        }
      }
    } else if (feas) {
      ++nf;
      nz += hd.zero_total;
      const Group<T, K> bw = load_group<T, K>(rec + R::off(kBandwidth, K));
      const Group<T, K> co = load_group<T, K>(rec + R::off(kCore, K));
      const Group<T, K> pw = load_group<T, K>(rec + R::off(kPower, K));
      const Group<T, K> to = load_group<T, K>(rec + R::off(kTotal, K));
      // this node's contribution: the max of each field over its qualifying cards
      T v[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};
      uint32_t any = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const bool q = (fr.v[j] >= m) & (ck.v[j] >= c);  // collection.go:46
        any |= (uint32_t)q;
        v[kMaxBw] = (q && bw.v[j] > v[kMaxBw]) ? bw.v[j] : v[kMaxBw];
        v[kMaxClock] = (q && ck.v[j] > v[kMaxClock]) ? ck.v[j] : v[kMaxClock];
        v[kMaxCore] = (q && co.v[j] > v[kMaxCore]) ? co.v[j] : v[kMaxCore];
        v[kMaxFree] = (q && fr.v[j] > v[kMaxFree]) ? fr.v[j] : v[kMaxFree];
        v[kMaxPower] = (q && pw.v[j] > v[kMaxPower]) ? pw.v[j] : v[kMaxPower];
        v[kMaxTotal] = (q && to.v[j] > v[kMaxTotal]) ? to.v[j] : v[kMaxTotal];
      }
      if (any) {
#pragma unroll
        for (int f = 0; f < 6; ++f) {
          if (v[f] > mx[f]) {  // nodes in increasing order: the first witness is the lowest
            mx[f] = v[f];
            wc[f] = 1u;
            wn[f] = n;
          } else if (v[f] == mx[f]) {
            ++wc[f];
          }
        }
      }
    }
    const uint64_t b = ballot(feas);
    const int j = (int)(n & 63u);
    set_lane(lo, hi, b, (uint32_t)j);
    if (j == 63 || n + 1 == n1) bm_store(bmw, n & ~63u, n1, lo, hi);
  }
  if (!live) return;
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    const size_t o = ((size_t)f * C + chunk) * n_pods + p;
    pmax[o] = (uint64_t)mx[f];
    pwit[o] = wc[f];
    pwit[(size_t)6 * C * n_pods + o] = wn[f];
  }
  pcnt[((size_t)0 * C + chunk) * n_pods + p] = nf;
  pcnt[((size_t)1 * C + chunk) * n_pods + p] = nz;
}

// Merge of k1_witness partials, one wave per pod: maxima [6][P], counts [2][P], and per field
// the witness count (summed over the chunks reaching the maximum) and the lowest witness
// (global id; 0xFFFFFFFF when no node reaches it, i.e. the floor of 1).
__global__ __launch_bounds__(kWave) void k_reduce_wit(const uint64_t* __restrict__ pmax,
                                                       const uint32_t* __restrict__ pwit,
                                                       const uint32_t* __restrict__ pcnt,
                                                       uint32_t C, uint32_t n_pods,
                                                       uint32_t node_offset,
                                                       uint64_t* __restrict__ maxima,
                                                       uint32_t* __restrict__ counts,
                                                       uint32_t* __restrict__ wcount,
                                                       uint32_t* __restrict__ wnode, MemTab mt) {
  const uint32_t p = blockIdx.x, lane = threadIdx.x;
  for (int f = 0; f < 6; ++f) {
    uint64_t mx = 1;
    uint32_t wc = 0, wn = 0xffffffffu;
    auto merge = [&](uint64_t m2, uint32_t c2, uint32_t n2) {
      if (m2 > mx) {
        mx = m2;
        wc = c2;
        wn = n2;
      } else if (m2 == mx) {
        wc += c2;
        wn = min(wn, n2);
      }
    };
    for (uint32_t c = lane; c < C; c += kWave) {
      const size_t o = ((size_t)f * C + c) * n_pods + p;
      merge(pmax[o], pwit[o], pwit[(size_t)6 * C * n_pods + o]);
    }
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const uint64_t m2 = __shfl_xor(mx, o, kWave);
      const uint32_t c2 = __shfl_xor(wc, o, kWave), n2 = __shfl_xor(wn, o, kWave);
      merge(m2, c2, n2);
    }
    if (mt.vf && f == kMaxFree) mx = rank_value(mx, mt.vf);  // memory ranks -> values
    if (mt.vf && f == kMaxTotal) mx = rank_value(mx, mt.vt);
    if (lane == 0) {
      maxima[(size_t)f * n_pods + p] = mx;
      wcount[(size_t)f * n_pods + p] = wc;
      wnode[(size_t)f * n_pods + p] = wn == 0xffffffffu ? wn : wn + node_offset;
    }
  }
  for (int f = 0; f < 2; ++f) {
    uint32_t sum = 0;
    for (uint32_t c = lane; c < C; c += kWave) sum += pcnt[((size_t)f * C + c) * n_pods + p];
    for (int o = kWave / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, kWave);
    if (lane == 0) counts[(size_t)f * n_pods + p] = sum;
  }
}

// K1, block-classified sweep (N32 path).  The batch is sorted by the Filter's inputs
// (yoda_order.hip), so the 64 pods of a wave usually share their clock / number labels and
// span a narrow memory range.  The wave first reduces its pods' thresholds to bounds
// (max/min of number, scv/memory, scv/clock, card counts needed), then walks its chunk in
// blocks of 64 nodes with LANE = NODE, reading the node summaries (K1Sum) coalesced, and
// classifies every node for the whole wave:
//   NONE  the bounds prove every pod of the wave infeasible (e.g. CardNumber < min number,
//         or the need_min-th largest healthy free < min memory);
//   ALL   the bounds prove every pod feasible AND the node's maxima contribution is the same
//         for every pod (one GPU model, uniform TotalMemory or no qualifying card);
//   PART  anything else: the node is evaluated exactly for every pod lane with k1_node.
// NONE and ALL are exact statements about every (pod, node) pair of the block, not
// approximations: ALL nodes fold their contribution into node-lane maxima that are reduced
// across the wave once per chunk, and both write their 64-bit masks with one store.
#ifndef YODA_K1_GEN_UNROLL
#define YODA_K1_GEN_UNROLL 1
#endif
// MIX = false: a snapshot whose every node is one GPU model with one TotalMemory (no per-card
// work in K1 at all): the same kernel with the per-card branches compiled out.
// WIT (capacity greedy windows, with MIX = false): also the witnesses of every maximum (how
// many nodes reach it, the lowest one; k1_witness's outputs), in k1_witness's partial layout:
// pmax [6][C][P] u64, pwit [2][6][C][P], pcnt [2][C][P].
// Packed N32 partial word w (k1_block_n32's epilogue) -> the MaxValue fields it holds:
// w 0: bandwidth | clock << 16, w 1: core | power << 16 (per-half max), w 2: free, w 3: total.
// nw = kNarrowWords when the four small fields fit 16 bits (<= 65535); with a wider one the
// partials hold one u32 word per MaxValue field, kMax* order (nw = kWideWords).
__device__ __forceinline__ uint32_t narrow_max(uint32_t a, uint32_t b, int w,
                                               uint32_t nw = kNarrowWords) {
  return (nw == kNarrowWords && w < 2) ? max16x2(a, b) : max(a, b);
}
__device__ __forceinline__ uint32_t narrow_floor(int w, uint32_t nw) {  // floor 1 per field
  return (nw == kNarrowWords && w < 2) ? 0x00010001u : 1u;
}

// SUB = 4 (the argmax runs): the workgroup's four waves hold the SAME 64 pods, each over its own
// quarter of the chunk (chunk_nodes = the quarter), and merge their partials in LDS at the end:
// a quarter of the partial bytes (and of k_reduce1's reads) for the same (wave, node-range)
// tasks -- 24 B per (pod, chunk) written once per chunk instead of once per quarter.
// The wave bounds K1's whole-block decisions compare against (k1_block_class), from the wave's
// pods: scv/number, scv/memory (m, the need in cards), scv/clock (c, the need in cards).
struct K1Wave {
  uint64_t num_min, num_max;
  uint32_t mpm_min, mpm_max;  // m over the pods with the scv/memory label
  uint32_t m_min, m_max, c_min, c_max;
  uint32_t cpc_max, nc_min, nc_max;  // c and the need over the pods with the scv/clock label
  uint32_t bs_tn, bs_ta;  // BlockSumWord words: the q-th healthy free's min / max for the needs
  bool any_pm, all_pm, any_pc, all_pc, c_uni, hfs_all_ok, hfs_none_ok;
};
// K1's whole-block decision for a block (its BlockSumWord words at B[64 w]): every node NONE
// (PodFitsNumber, PodFitsMemory or PodFitsClock fails for every pod of the wave), or every node
// ALL (one-model, feasible for every pod, its cards all qualifying -- allq -- or none).  Every
// word is loaded up front and tested bitwise: one memory round trip per 64 blocks.  (As short-
// circuit tests each load was issued only once the test before it had its answer: ~10 dependent
// round trips per 64 blocks -- most of a K1 task's block pass.)  Shared by the block K1 and its
// cost probe (k1_probe), so both classify alike.  Sufficient conditions of the per-node tests.
struct K1BlockClass {
  bool none, all, allq;
  uint32_t nreal;  // the block's real nodes (0 for an invalid lane)
};
// mix_all = false: whole-block ALL for one-model blocks only (k1_probe's cost weights: with the
// other blocks' ALL counted as per-node work the heaviest-first order comes out better --
// mixed50 K1 0.91 vs 1.10 ms; the blocks they decide are not what makes a wave long)
__device__ __forceinline__ K1BlockClass k1_block_class(const uint32_t* B, bool bv,
                                                       const K1Wave& w, bool mix_all = true) {
  const uint32_t fl = B[64 * kBsFlags], ckmin = B[64 * kBsCkMin], ckmax = B[64 * kBsCkMax];
  const uint32_t cn_min = B[64 * kBsCnMin], cn_max = B[64 * kBsCnMax];
  const uint32_t nreal_w = B[64 * kBsNReal], t_none = B[64 * w.bs_tn], t_all = B[64 * w.bs_ta];
  const uint32_t hck_min = B[64 * kBsHckMin], hck_max = B[64 * kBsHckMax];
  const uint32_t nh_min = B[64 * kBsNhMin], nh_max = B[64 * kBsNhMax];
  const uint32_t mrf_min = B[64 * kBsMrfMin], mrf_max = B[64 * kBsMrfMax];
  const uint32_t sat = B[64 * kBsSat];
  uint32_t hcw[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) hcw[e] = B[64 * (kBsHc + e)];
  K1BlockClass r;
  r.nreal = bv ? nreal_w : 0u;
  // the block's healthy cards of the wave's one scv/clock per node, min / max (hc table)
  const bool tab = (fl & kBsHcTab) != 0u;
  const uint32_t n_hc = (fl >> 8) & 7u;
  uint32_t hc_lo = 0u, hc_hi = 0u;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bool hit = ((uint32_t)e < n_hc) & ((hcw[e] & 0xffffu) == w.cpc_max);
    hc_lo = hit ? (hcw[e] >> 16) & 0xffu : hc_lo;
    hc_hi = hit ? hcw[e] >> 24 : hc_hi;
  }
  const bool one = (fl & kBsOneModel) != 0u;
  bool bnone = (cn_max != 0xffffffffu) & (w.num_min > (uint64_t)cn_max);
  bnone |= w.all_pm & (!w.hfs_none_ok | (t_none <= w.mpm_min));
  if (w.all_pc && w.c_uni) {
    // no healthy card of the block has the wave's clock (hc = 0 < need), or one-model nodes
    // of that clock with too few healthy cards, or no node with enough of them (hc table)
    bnone |= (w.cpc_max < hck_min) | (w.cpc_max > hck_max) |
             (((fl & kBsUni4) != 0u) & (ckmin == ckmax) & (ckmin == w.cpc_max) &
              (nh_max < w.nc_min)) |
             (tab & (hc_hi < w.nc_min));
  }
  bool ball = (w.num_max <= (uint64_t)cn_min);
  ball &= !w.any_pm | (w.hfs_all_ok & (t_all > w.mpm_max));
  ball &= !w.any_pc |
          (w.c_uni & (one ? (ckmin == ckmax) & (ckmin == w.cpc_max) & (nh_min >= w.nc_max)
                          : tab & (hc_lo >= w.nc_max)));
  // every pod's qualifying cards (collection.go:46) reach each node's all-card maxima: every
  // card passes the clock test and the scv/memory is below the saturation free (one-model
  // nodes of one total: sat = mrf, the old rule)
  r.allq = (ckmin >= w.c_max) & (sat > w.m_max);
  const bool noq = (ckmax < w.c_min) | (mrf_max <= w.m_min);
  // (other blocks: no clock-only noq -- the seed's level bound assumes every card passes)
  ball &= (r.allq | (one ? noq : mrf_max <= w.m_min)) & !bnone & (one | mix_all);
#ifdef YODA_AB_NO_MIXALL  // (A/B build: whole-block ALL for one-model blocks only, as round 5)
  ball &= one;
#endif
  r.none = bnone & bv & (r.nreal > 0u);
  r.all = ball & bv & (r.nreal > 0u);
  return r;
}

template <int K, bool STATS, bool MIX = true, bool WIT = false, int SUB = 1>
#ifndef YODA_K1_WAVES
#define YODA_K1_WAVES 6  // (7: 9 VGPRs spilled, ~90 MB of scratch writes per launch; r05j)
#endif
// (waves per SIMD: 6 for one-model tiles -- no VGPR spills; 6 with the mixed-model tiles too
// since their PART nodes are staged in LDS (round 6): mixed50 K1 0.75 vs 0.80 ms at 7 waves,
// profiles/r06/mixed/ab_staged.txt; 7 paid while the per-node loop was a chain of scalar loads)
#ifndef YODA_K1_MIX_WAVES
#define YODA_K1_MIX_WAVES 6
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WIT ? 4 : (K >= 16 ? 5 : (MIX ? YODA_K1_MIX_WAVES : YODA_K1_WAVES))))) void k1_block_n32(
    const unsigned char* __restrict__ nodes, const unsigned char* __restrict__ sum,
    const uint32_t* __restrict__ sum2w, const uint32_t* __restrict__ mixw,
    const uint32_t* __restrict__ x1w,
    uint32_t n_nodes, uint32_t chunk_nodes, const uint32_t* __restrict__ m_in,
    const uint32_t* __restrict__ c_in, const uint64_t* __restrict__ number_in,
    const uint32_t* __restrict__ need_mem_in, const uint32_t* __restrict__ need_clk_in,
    uint32_t n_pods, uint64_t* __restrict__ pmax, uint32_t* __restrict__ pcnt,
    uint64_t* __restrict__ bm, uint32_t bm_stride, BlockMask* __restrict__ bs,
    uint32_t bs_stride, uint64_t* __restrict__ blk, uint32_t blk_stride,
    unsigned long long* __restrict__ stats, uint32_t* __restrict__ pwit = nullptr,
    const uint32_t* __restrict__ bsm = nullptr, uint32_t nwords = kNarrowWords,
    uint32_t* __restrict__ wts = nullptr, const uint32_t* __restrict__ gtab = nullptr,
    const uint32_t* __restrict__ kbub = nullptr, const uint32_t* __restrict__ levels = nullptr,
    unsigned long long* __restrict__ seed_out = nullptr,
    unsigned long long* __restrict__ cmask = nullptr,
    const uint32_t* __restrict__ ids = nullptr,
    const uint32_t* __restrict__ pb_order = nullptr) {
  static_assert(!(WIT && MIX), "the witness K1 serves one-model snapshots");
  static_assert(SUB == 1 || (SUB == kBlock / kWave && !WIT), "SUB: 1, or one pod wave per workgroup");
  constexpr uint32_t SS = k1sum_stride(K);
  constexpr uint32_t NS = n32_stride(K);
  constexpr uint32_t S2 = k2sum_stride(K), MS = mix_stride(K), XS = x1_stride(K);
  constexpr uint32_t HW = K + 1;  // LDS words per node: hfs[0..K-1], 0
  // + a 10-word record per one-model PART node (below): the per-pod pass reads it from LDS
  constexpr uint32_t REC = 10, RECS = kWave * HW;
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[kBlock / kWave][RECS + kWave * REC];
  uint32_t* lds = lds_all[threadIdx.x >> 6];
  const uint32_t lane = lane_id();
  const Tile tl = tile();
  const uint32_t sub = SUB > 1 ? threadIdx.x >> 6 : 0u;
  // pb_order: the pod blocks heaviest first (k1_probe + k_lpt_order), so the long tasks do not
  // start last (SUB = 1)
  const uint32_t pbk = (SUB == 1 && pb_order != nullptr) ? pb_order[tl.pb] : tl.pb;
  const uint32_t p = SUB > 1 ? tl.pb * kWave + lane : pbk * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk, C = gridDim.y;
  const uint32_t n0 = (chunk * SUB + sub) * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  const uint64_t live_mask = ballot(live);
  // a wave past the batch: no bitmask row, no partials (SUB: the whole workgroup, together)
  if (live_mask == 0) return;
  uint64_t* bmw = bm + (size_t)uniform_u32(p >> 6) * bm_stride;
  BlockMask* bsw = bs + (size_t)uniform_u32(p >> 6) * bs_stride;
  // STATS with stats[15] == 2: per-(wave, chunk) timing trace only (no counter atomics)
  // (stats[15] >> 8 = the trace slots allocated: every slot index is bounded by it)
  const bool trace = STATS && (stats[15] & 0xffull) == 2ull;
  const uint64_t t_start = STATS ? wall_clock64() : 0ull;
  uint32_t npart = 0, nblk = 0;  // (trace: PART nodes, blocks classified node by node)

  uint32_t m = 0, c = 0, need_mem = 0, need_clk = 0;
  uint64_t number = ~0ull;
  if (live) {
    m = m_in[p];
    c = c_in[p];
    number = number_in[p];
    need_mem = need_mem_in[p];
    need_clk = need_clk_in[p];
  }
  // ---- wave bounds (pm: pods with the scv/memory label, pc: with scv/clock) ----
  const bool pm = live && need_mem > 0, pc = live && need_clk > 0;
  const uint64_t pm_mask = ballot(pm), pc_mask = ballot(pc);
  const bool any_pm = pm_mask != 0, all_pm = pm_mask == live_mask;
  const bool any_pc = pc_mask != 0, all_pc = pc_mask == live_mask;
  const uint64_t num_max = wave_max_u64(live ? number : 0ull);
  const uint64_t num_min = wave_min_u64(live ? number : ~0ull);
  const uint32_t nm_max = wave_max_u32(pm ? need_mem : 0u);
  const uint32_t nm_min = wave_min_u32(pm ? need_mem : ~0u);
  // (bounds compared only against node-lane values stay in VGPRs: fewer SGPR spills, whose
  // v_readlane reloads cost issue slots in every block; profiles/r02/final/k1_occupancy_ab.txt)
  const uint32_t mpm_max = wave_max_u32v(pm ? m : 0u);
  const uint32_t mpm_min = wave_min_u32v(pm ? m : ~0u);
  const uint32_t nc_max = wave_max_u32(pc ? need_clk : 0u);
  const uint32_t nc_min = wave_min_u32(pc ? need_clk : ~0u);
  const uint32_t cpc_max = wave_max_u32(pc ? c : 0u);
  const uint32_t cpc_min = wave_min_u32(pc ? c : ~0u);
  const uint32_t m_max = wave_max_u32v(live ? m : 0u), m_min = wave_min_u32v(live ? m : ~0u);
  const uint32_t c_max = wave_max_u32v(live ? c : 0u), c_min = wave_min_u32v(live ? c : ~0u);
  const bool c_uni = cpc_min == cpc_max;
  // hfs slot of the (1-based) need; a need beyond the K slots has no such card (hfs = 0)
  const bool hfs_all_ok = nm_max <= (uint32_t)K, hfs_none_ok = nm_min <= (uint32_t)K;
  const uint32_t hfs_all = kSumHfs + (any_pm && hfs_all_ok ? nm_max - 1u : 0u);
  const uint32_t hfs_none = kSumHfs + (hfs_none_ok ? nm_min - 1u : 0u);
  // Every pod of the wave needs the same number of memory-fitting cards (or none has the
  // scv/memory label): the per-pod pass reads that card's threshold hfs[need-1] from the
  // node lane (t_all) instead of an LDS row of all K, and the rows are not staged at all.
  const bool need_uni = uniform_u32(!any_pm || (all_pm && nm_min == nm_max)) != 0u;

  // (trace: the end of the set-up, the end of the block pass)
  const uint64_t t_setup = STATS ? wall_clock64() : 0ull;
  uint32_t mx[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) mx[f] = 1u;  // floor 1 (collection.go:31-38)
  uint32_t nf = 0, nz = 0;
  // node-lane maxima of the ALL nodes (their contribution is the same for every pod lane)
  uint32_t a_bw = 0, a_ck = 0, a_core = 0, a_free = 0, a_pw = 0, a_tot = 0;
  uint32_t nf_all = 0, nz_all = 0;
  // WIT: per field, the pod lane's witness count / lowest witness of mx (per-pod nodes), and
  // the node lane's maximum / count / lowest node over the ALL nodes it holds
  uint32_t wc[WIT ? 6 : 1], wn[WIT ? 6 : 1], aw[WIT ? 6 : 1], ac[WIT ? 6 : 1], al[WIT ? 6 : 1];
  if constexpr (WIT) {
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      wc[f] = ac[f] = 0u;
      wn[f] = al[f] = 0xffffffffu;
      aw[f] = 1u;
    }
  }
  // blocks with a feasible pod of this wave, for K2 (bit b of word b/64; flushed with an
  // atomic OR when the word changes -- neighbouring chunks may share a word)
  uint64_t* blkw = blk + (size_t)uniform_u32(p >> 6) * blk_stride;
  uint32_t blk_wi = (n0 >> 6) >> 6;
  uint64_t blk_bits = 0;
  auto blk_flush = [&]() {
    if (blk_bits != 0 && lane == 0)
      atomicOr(reinterpret_cast<unsigned long long*>(blkw + blk_wi), (unsigned long long)blk_bits);
  };

#ifndef YODA_K1_PF
#define YODA_K1_PF 0
#endif
  // the summary words a block's classification reads (YODA_K1_PF = 1: the next block
  // node_block visits is loaded while this one is classified; off: the extra live registers
  // spill, K1 0.211-0.219 ms without against 0.230-0.235 with, same box)
  uint4 pf0 = make_uint4(0u, 0u, 0u, 0u), pf1 = pf0;
  uint32_t pf_pw = 0, pf_ta = 0, pf_tn = 0;
  auto load_sum = [&](uint32_t nb) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(sum) + sum_index(nb, 0, SS) + lane;
    pf0 = make_uint4(s[64 * kSumCnLo], s[64 * kSumCnHi], s[64 * kSumClock], s[64 * kSumMeta]);
    pf1 = make_uint4(s[64 * kSumMrf1], s[64 * kSumTotal], s[64 * kSumBw], s[64 * kSumCore]);
    pf_pw = s[64 * kSumPower];
    pf_ta = s[64 * hfs_all];
    pf_tn = s[64 * hfs_none];
  };
  // Whole-block decisions from the block summaries (BlockSumWord, scalar reads): the bounds
  // of the block's nodes against the wave's bounds prove every node NONE, or every node ALL
  // with one contribution (all qualifying: the block's maxima; none qualifying: nothing).
  // Sufficient conditions of the per-node tests below, so the outcome is the same.
  constexpr uint32_t BST = bsum_stride(K);
  const uint32_t s_mpm_max = uniform_u32(mpm_max), s_mpm_min = uniform_u32(mpm_min);
  const uint32_t s_m_max = uniform_u32(m_max), s_m_min = uniform_u32(m_min);
  const uint32_t s_c_max = uniform_u32(c_max), s_c_min = uniform_u32(c_min);
  // K2 pruning seed (PodParams::seed): the most any node that EVERY live pod of the wave passes
  // scores for all of them under the G maxima -- static + B_G[q], q = the cards that qualify
  // for the wave's largest scv/memory (so for every pod: B_G is non-decreasing in q), one-model
  // nodes only (a feasible one has the pods' scv/clock, so every card passes the clock test).
  // Taken over the ALL blocks (lane = block, kbub's lv[] at the wave's largest scv/memory);
  // YODA_K1_NODE_SEEDS (A/B) adds the ALL nodes of the blocks classified node by node.
#ifdef YODA_K1_NOSEED  // (A/B build: the seed code compiled out)
  const bool seeding = false;
#else
  const bool seeding = !WIT && seed_out != nullptr && gtab != nullptr;
#endif
  // (kept in LDS, one word per wave, max-updated by the lanes: no registers across the loops)
  __shared__ unsigned long long lds_seed[kBlock / kWave];
  unsigned long long* sdw = lds_seed + (threadIdx.x >> 6);
  if (seeding && lane == 0) *sdw = 0ull;
  // ALL blocks: kbub's lv[l_hi], l_hi = the smallest free level >= the wave's largest scv/memory
  uint32_t l_hi = kKbLevels - 1u;
  if (seeding && kbub != nullptr && levels != nullptr)
    for (uint32_t l = kKbLevels - 1u; l-- > 0u;) l_hi = levels[l] >= s_m_max ? l : l_hi;
  const uint32_t bs_tn = kBsT + (uint32_t)K + (hfs_none_ok && nm_min > 0u ? nm_min - 1u : 0u);
  const uint32_t bs_ta = kBsT + (any_pm && hfs_all_ok && nm_max > 0u ? nm_max - 1u : 0u);
  const K1Wave kw{num_min, num_max, s_mpm_min, s_mpm_max, s_m_min, s_m_max, s_c_min, s_c_max,
                  cpc_max, nc_min, nc_max, bs_tn, bs_ta, any_pm, all_pm, any_pc, all_pc, c_uni,
                  hfs_all_ok, hfs_none_ok};
  // per-node classification of one 64-node block (below: only the blocks the block summaries
  // leave undecided)
  // (nxt: the block node_block visits next, whose summary words are loaded here -- the
  // caller loaded nb's before the first call; ~0u: none)
  auto node_block = [&](uint32_t nb, uint32_t nxt) {
    if (STATS) ++nblk;
    const uint32_t n = nb + lane;
    const bool valid = n < n1;
    // this block's tile of summaries (nb is a multiple of 64): word w at s[64 w]
    const uint32_t* s = reinterpret_cast<const uint32_t*>(sum) + sum_index(nb, 0, SS) + lane;
    if (!YODA_K1_PF) load_sum(nb);
    const uint4 w0 = pf0, w1 = pf1;
    const uint32_t pw0 = pf_pw, t_all = pf_ta, t_none = pf_tn;
    if (YODA_K1_PF && nxt != ~0u) load_sum(nxt);
    if (!need_uni) {  // the node's healthy frees for the per-pod pass: lds[node][need - 1] (slot K: 0)
      // (all K loads in flight before the first LDS write: one round trip, not K / 2)
      uint32_t hv[K];
#pragma unroll
      for (int t = 0; t < K; ++t) hv[t] = s[64 * (kSumHfs + t)];
#pragma unroll
      for (int t = 0; t < K; ++t) lds[lane * HW + t] = hv[t];
      lds[lane * HW + K] = 0u;
    }
    const uint64_t cn = (uint64_t)w0.x | ((uint64_t)w0.y << 32);
    const uint32_t meta = w0.w;
    // the node's model values; for the per-card nodes below, overwritten with their maxima
    // contribution (those nodes never take the one-model record path, the only other reader)
    uint32_t ck = w0.z, mrf1 = w1.x, tot = w1.y, bw = w1.z, core = w1.w, pw = pw0;
    const bool uni4 = (meta & kSumUni4) != 0u, unit = (meta & kSumUniTotal) != 0u;
    const bool one_model = uni4 && unit;
    const uint32_t nh = (meta >> 8) & 0xffu;
    // PodFitsNumber / PodFitsMemory for every pod of the wave at once
    const bool mem_all = !any_pm || (hfs_all_ok && t_all > mpm_max);
    const bool mem_none = all_pm && (!hfs_none_ok || t_none <= mpm_min);
    const bool num_none = num_min > cn;
    // hc: the node's healthy cards whose clock is the wave's scv/clock (PodFitsClock's count,
    // filter.go:56-58; meaningful when every pod with the label asks for one clock, c_uni)
    uint32_t hc = (uni4 && ck == cpc_max) ? nh : 0u;
    // mixed-model nodes: count hc over the per-card clocks (free order, with health bits),
    // only when it decides something (some pod has the label, all of them one clock) and
    // the number / memory bounds leave the node open
    const uint32_t* xw = x1w + sum_index(nb, 0, XS) + lane;
    if (any_pc && c_uni) {
#ifdef YODA_ABL_K1_NOHC
      const bool cnt_clk = false;
#else
      const bool cnt_clk = MIX && valid && !uni4 && !num_none && !mem_none;
#endif
      if (ballot(cnt_clk) != 0ull) {
        if (cnt_clk) {  // the node's healthy-card count per distinct clock (K1MixWord ch)
          if ((xw[64 * kX1Chg] & kX1ChgMany) == 0u) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t w = xw[64 * (kX1Ch + e)];
              hc += (w & 0xffffu) == cpc_max ? w >> 16 : 0u;
            }
          } else {  // more than 4 distinct clocks: the cards one by one
            const uint32_t* mxw = mixw + sum_index(nb, 0, MS) + lane;
            const uint32_t hm = mxw[64 * mix_hm(K)];
#pragma unroll
            for (int t = 0; t < K; ++t)
              hc += ((hm >> t) & 1u) & (uint32_t)(mxw[64 * mix_word(kMixCk, t, K)] == cpc_max);
          }
        }
      }
    }
    // PodFitsClock for every pod of the wave at once
    const bool clk_all = !any_pc || (c_uni && hc >= nc_max);
    const bool clk_none = all_pc && c_uni && hc < nc_min;
    const bool feas_all = (num_max <= cn) && mem_all && clk_all;
    const bool feas_none = num_none || mem_none || clk_none;
    // The node's CollectMaxValues contribution (collection.go:46: cards with free >= m and
    // clock >= c, no health check) is the same for every pod of the wave when the SMALLEST
    // qualifying set (the wave's largest m and c) and the LARGEST (its smallest m and c) give
    // the same six maxima: every pod's set lies between the two.  One-model node with one
    // TotalMemory: some card qualifies  <=>  clock >= c  and  max free >= m, and then the
    // maxima are the node's own model values.
    bool qual = ck >= c_max && mrf1 > m_max;
    bool same = qual || ck < c_min || mrf1 <= m_min;
    // Any other node (mixed GPU models, or per-card TotalMemory) that every pod of the wave
    // passes: a loop over its free-ordered cards (K2 summary frees / totals, per-card models),
    // lane = node -- the smallest set's maxima, then whether a card of the largest set but
    // not the smallest raises one of them.
#ifdef YODA_ABL_K1_NOGEN
    const bool gen = false;
#else
    const bool gen = MIX && valid && !one_model && feas_all && !feas_none;
#endif
    if (ballot(gen) != 0ull) {
      if (gen) {
        // The cards in free order (K2 summary): the smallest set is {t < qs, clock >= c_max},
        // the largest {t < ql, clock >= c_min}, qs / ql = cards with free >= m_max / m_min.
        const uint32_t* s2 = sum2w + sum_index(nb, 0, S2) + lane;
        const uint32_t cnt = (s2[64 * kS2Meta] >> 8) & 0xffu, minclk = s2[64 * kS2MinClk];
        uint32_t qs = 0, ql = 0;
#pragma unroll
        for (int t = 0; t < K; ++t) {
          const uint32_t f = s2[64 * (kS2Fs + t)];
          qs += (uint32_t)(f >= m_max);
          ql += (uint32_t)(f >= m_min);
        }
        qs = min(qs, cnt);
        ql = min(ql, cnt);
        if (c_max <= minclk) {
          // every card passes every pod's clock test: both sets are prefixes, whose maxima
          // are tabled (K1MixWord pm) with the cards where they change (chg)
          const uint32_t chg = xw[64 * kX1Chg];
          same = ((chg >> (qs + 1u)) & ((1u << (ql - qs)) - 1u)) == 0u;
          bw = ck = core = mrf1 = pw = tot = 0u;
          if (qs > 0u) {
            const uint32_t* pm = xw + 64 * x1_pm((int)qs - 1, 0);
            const uint32_t a = pm[0], b = pm[64], t = pm[128];
            ck = a & 0xffffu;
            bw = a >> 16;
            core = b & 0xffffu;
            pw = b >> 16;
            tot = t;
            mrf1 = s2[64 * kS2Fs] + 1u;  // the first card has the largest free
          }
        } else {
          // per card, both sets' maxima at once (clock|bandwidth and core|power per 16-bit
          // half); the contribution is the same for every pod iff they are equal
          uint32_t sa = 0, sb = 0, st = 0, sf = 0, la = 0, lb = 0, lt = 0, lf = 0;
#pragma unroll YODA_K1_GEN_UNROLL
          for (int t = 0; t < K; ++t) {
            const uint32_t f = s2[64 * (kS2Fs + t)], to = s2[64 * (kS2Fs + K + t)];
            const uint32_t a = xw[64 * x1_cd(t, 0, K)], b = xw[64 * x1_cd(t, 1, K)];
            const uint32_t cj = a & 0xffffu;
            const bool real = (uint32_t)t < cnt;
            const bool in_s = real & (f >= m_max) & (cj >= c_max);
            const bool in_l = real & (f >= m_min) & (cj >= c_min);
            sa = max16x2(sa, in_s ? a : 0u);
            sb = max16x2(sb, in_s ? b : 0u);
            st = max(st, in_s ? to : 0u);
            sf = max(sf, in_s ? f + 1u : 0u);
            la = max16x2(la, in_l ? a : 0u);
            lb = max16x2(lb, in_l ? b : 0u);
            lt = max(lt, in_l ? to : 0u);
            lf = max(lf, in_l ? f + 1u : 0u);
          }
          same = (sa == la) & (sb == lb) & (st == lt) & (sf == lf);
          ck = sa & 0xffffu;
          bw = sa >> 16;
          core = sb & 0xffffu;
          pw = sb >> 16;
          tot = st;
          mrf1 = sf;
        }
        qual = true;
      }
    }
    const bool is_none = valid && feas_none;
    const bool is_all = valid && !feas_none && feas_all && same;
#ifdef YODA_K1_NODE_SEEDS  // (A/B: per-node seeds too -- +35 % K1 time for little K2 gain)
    if (seeding) {
      const bool sdl = valid && feas_all && !feas_none && uni4;
      if (ballot(sdl) != 0ull && sdl) {
        uint32_t q = 0;  // healthy cards with free >= the largest m (<= the qualifying cards)
#pragma unroll
        for (int t = 0; t < K; ++t) q += s[64 * (kSumHfs + t)] > m_max ? 1u : 0u;
        const uint32_t* s2 = sum2w + sum_index(nb, 0, k2sum_stride(K)) + lane;
        const double st = __longlong_as_double(
            (long long)((uint64_t)s2[64 * kS2Static] | ((uint64_t)s2[64 * (kS2Static + 1)] << 32)));
        const uint32_t bq = q > 0u ? gtab[sum_index(nb + lane, q - 1u, gtab_stride(K))] : 0u;
        atomicMax(sdw, (unsigned long long)((uint64_t)st + (uint64_t)bq));
      }
    }
#endif
    const uint64_t all_b = ballot(is_all), none_b = ballot(is_none);
    uint64_t part_b = ballot(valid) & ~all_b & ~none_b;
    if (STATS && !trace) {  // class counts of (wave, node) pairs: ALL, NONE; whole blocks
      if (lane == 0) {
        atomicAdd(stats + 0, (unsigned long long)__builtin_popcountll(all_b));
        atomicAdd(stats + 1, (unsigned long long)__builtin_popcountll(none_b));
        atomicAdd(stats + 12, 1ull);
      }
    }
    nf_all += (uint32_t)__builtin_popcountll(all_b);
    nz_all += (uint32_t)__builtin_popcountll(ballot(is_all && (meta & kSumZeroTotal)));
    if (is_all && qual) {
      a_bw = max(a_bw, bw);
      a_ck = max(a_ck, ck);
      a_core = max(a_core, core);
      a_free = max(a_free, mrf1 - (mrf1 != 0u ? 1u : 0u));
      a_pw = max(a_pw, pw);
      a_tot = max(a_tot, tot);
      if constexpr (WIT) {  // nodes in increasing order per lane: the first witness is lowest
        const uint32_t v[6] = {bw, ck, core, mrf1 - (mrf1 != 0u ? 1u : 0u), pw, tot};
#pragma unroll
        for (int f = 0; f < 6; ++f) {
          const bool gt = v[f] > aw[f], eq = v[f] == aw[f];
          ac[f] = gt ? 1u : ac[f] + (eq ? 1u : 0u);
          al[f] = gt ? nb + lane : al[f];
          aw[f] = gt ? v[f] : aw[f];
        }
      }
    }
    uint32_t lo = is_all ? (uint32_t)live_mask : 0u;
    uint32_t hi = is_all ? (uint32_t)(live_mask >> 32) : 0u;
    npart += (uint32_t)__builtin_popcountll(part_b);  // (STATS trace; wts)
    // One-model PART nodes: a record of the node's facts in LDS -- {CardNumber lo, hi,
    // clock, meta, max free + 1, hfs[need - 1], bandwidth, core, power, total} -- read by
    // the per-pod pass with broadcast loads, four nodes per trip, branch-free.
    const uint64_t rec_b = part_b & ballot(one_model);
    if (rec_b != 0ull && ((rec_b >> lane) & 1ull)) {
      uint32_t* r = lds + RECS + lane * REC;
      *reinterpret_cast<uint2*>(r + 0) = make_uint2(w0.x, w0.y);
      *reinterpret_cast<uint2*>(r + 2) = make_uint2(ck, meta);
      *reinterpret_cast<uint2*>(r + 4) = make_uint2(mrf1, hfs_all_ok ? t_all : 0u);
      *reinterpret_cast<uint2*>(r + 6) = make_uint2(bw, core);
      *reinterpret_cast<uint2*>(r + 8) = make_uint2(pw, tot);
    }
    // the pod lane's hfs slot of its need (slot K: no such card, 0) for the LDS rows
    const uint32_t hk = need_mem == 0u ? (uint32_t)K : min(need_mem, (uint32_t)K + 1u) - 1u;
    uint64_t rb = rec_b;
    while (rb) {
#ifndef YODA_K1_R
#define YODA_K1_R 2
#endif
      constexpr int R = YODA_K1_R;
      uint32_t jj[R];
      bool vv[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        vv[k] = rb != 0ull;
        jj[k] = vv[k] ? (uint32_t)__builtin_ctzll(rb) : 0u;
        rb &= rb - 1;
      }
      uint2 r0[R], r1[R], r2[R], r3[R], r4[R];
      uint32_t th[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint32_t* r = lds + RECS + jj[k] * REC;
        r0[k] = *reinterpret_cast<const uint2*>(r + 0);
        r1[k] = *reinterpret_cast<const uint2*>(r + 2);
        r2[k] = *reinterpret_cast<const uint2*>(r + 4);
        r3[k] = *reinterpret_cast<const uint2*>(r + 6);
        r4[k] = *reinterpret_cast<const uint2*>(r + 8);
        // hfs[need-1] of node j: its lane's (uniform need), or the pod's slot of the row
        th[k] = need_uni ? r2[k].y : lds[jj[k] * HW + hk];
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint64_t cnj = (uint64_t)r0[k].x | ((uint64_t)r0[k].y << 32);
        const uint32_t ckj = r1[k].x, mj = r1[k].y, mrfj = r2[k].x;
        // PodFitsNumber / Memory (CardFitsMemory count >= need <=> hfs[need-1] > m) / Clock
        // (bitwise, not short-circuit: selects, no exec-mask branches)
        const bool fn = number <= cnj;
        const bool fm = (need_mem == 0u) | (th[k] > m);
        const bool fc = (need_clk == 0u) | ((ckj == c) & (((mj >> 8) & 0xffu) >= need_clk));
        const bool f = vv[k] & live & fn & fm & fc;
        nf += f ? 1u : 0u;
        nz += (f & ((mj & kSumZeroTotal) != 0u)) ? 1u : 0u;
        const bool q = f & (ckj >= c) & (mrfj > m);  // collection.go:46, one-model node
        if constexpr (WIT) {  // the node's values against the lane's maxima and witnesses
          const uint32_t v[6] = {r3[k].x, ckj, r3[k].y, mrfj - 1u, r4[k].x, r4[k].y};
#pragma unroll
          for (int g = 0; g < 6; ++g) {
            const bool gt = q & (v[g] > mx[g]), eq = q & (v[g] == mx[g]);
            wc[g] = gt ? 1u : wc[g] + (eq ? 1u : 0u);
            wn[g] = gt ? nb + jj[k] : wn[g];
            mx[g] = gt ? v[g] : mx[g];
          }
        } else {
          mx[kMaxBw] = max(mx[kMaxBw], q ? r3[k].x : 0u);
          mx[kMaxClock] = max(mx[kMaxClock], q ? ckj : 0u);
          mx[kMaxCore] = max(mx[kMaxCore], q ? r3[k].y : 0u);
          mx[kMaxFree] = max(mx[kMaxFree], q ? mrfj - 1u : 0u);
          mx[kMaxPower] = max(mx[kMaxPower], q ? r4[k].x : 0u);
          mx[kMaxTotal] = max(mx[kMaxTotal], q ? r4[k].y : 0u);
        }
        const uint64_t b = ballot(f);
        if (vv[k]) set_lane(lo, hi, b, jj[k]);
      }
    }
    part_b &= ~rec_b;
#ifndef YODA_K1_LEAN_GLOBAL
    // Other PART nodes (several GPU models, or several TotalMemory values): their cards staged
    // in LDS, lane = node, from the block's tiles (K2 summary frees / totals in free order,
    // K1MixWord cards, the health bits) -- one memory round trip per batch of nodes -- then
    // read by the per-pod pass with broadcast ds_read_b128s.  (Before: k1_node_lean's per-card
    // loop over the node record, ~2K dependent scalar loads per node: mixed50 K1 0.88 ms.)
    // The area is the rows / records above, free again here.  Per node: {CardNumber lo, hi,
    // health bits | zero-total << 31, 0}, then per card {free, clock | bw << 16, total,
    // core | power << 16} (16-bit halves: such snapshots keep those fields <= 55738).
    if constexpr (MIX) {
      constexpr uint32_t XN = 4u * (uint32_t)K + 4u;
      constexpr uint32_t NBAT = (RECS + kWave * REC) / XN;
      static_assert(NBAT >= 1u, "LDS area");
      while (part_b) {
        uint64_t bat = part_b;
        if ((uint32_t)__builtin_popcountll(bat) > NBAT) {  // the lowest NBAT nodes
          uint64_t t = bat;
          for (uint32_t k = 0; k < NBAT; ++k) t &= t - 1;
          bat &= ~t;
        }
        part_b &= ~bat;
        if ((bat >> lane) & 1ull) {
          const uint32_t slot = (uint32_t)__builtin_popcountll(bat & ((1ull << lane) - 1ull));
          uint32_t* r = lds + slot * XN;
          const uint32_t* s2 = sum2w + sum_index(nb, 0, S2) + lane;
          const uint32_t hm = mixw[sum_index(nb, 0, MS) + lane + 64u * mix_hm(K)];
          *reinterpret_cast<uint4*>(r) =
              make_uint4(w0.x, w0.y, hm | ((meta & kSumZeroTotal) ? 0x80000000u : 0u), 0u);
          // (two cards' words in flight per step: more would spill -- the kernel runs at its
          // VGPR budget)
#pragma unroll 2
          for (int t = 0; t < K; ++t)
            *reinterpret_cast<uint4*>(r + 4 + 4 * t) =
                make_uint4(s2[64 * (kS2Fs + t)], xw[64 * x1_cd(t, 0, K)],
                           s2[64 * (kS2Fs + K + t)], xw[64 * x1_cd(t, 1, K)]);
        }
        uint32_t slot = 0;
        while (bat) {
          const uint32_t j = (uint32_t)__builtin_ctzll(bat);
          bat &= bat - 1;
          const uint32_t* r = lds + (slot++) * XN;
          const uint4 h = *reinterpret_cast<const uint4*>(r);
          // PodFitsMemory / PodFitsClock counts (filter.go:52-58) from {free, clock | bw}
          uint32_t cm = 0, cc = 0;
#pragma unroll 4
          for (int t = 0; t < K; ++t) {
            const uint2 fa = *reinterpret_cast<const uint2*>(r + 4 + 4 * t);
            const uint32_t ht = (h.z >> t) & 1u;
            cm += (uint32_t)(fa.x >= m) & ht;
            cc += (uint32_t)((fa.y & 0xffffu) == c) & ht;
          }
          const uint64_t cnj = (uint64_t)h.x | ((uint64_t)h.y << 32);
          const bool f = live & (number <= cnj) & (cm >= need_mem) & (cc >= need_clk);
          nf += f ? 1u : 0u;
          nz += (f & ((h.z >> 31) != 0u)) ? 1u : 0u;
          const uint64_t b = ballot(f);
          if (b != 0ull) {  // the maxima over the qualifying cards (collection.go:46: no health
                            // check, clock >= the pod's), feasible lanes only
#pragma unroll 2
            for (int t = 0; t < K; ++t) {
              const uint4 cd = *reinterpret_cast<const uint4*>(r + 4 + 4 * t);
              const bool q = f & (cd.x >= m) & ((cd.y & 0xffffu) >= c);
              mx[kMaxBw] = max(mx[kMaxBw], q ? cd.y >> 16 : 0u);
              mx[kMaxClock] = max(mx[kMaxClock], q ? cd.y & 0xffffu : 0u);
              mx[kMaxCore] = max(mx[kMaxCore], q ? cd.w & 0xffffu : 0u);
              mx[kMaxPower] = max(mx[kMaxPower], q ? cd.w >> 16 : 0u);
              mx[kMaxFree] = max(mx[kMaxFree], q ? cd.x : 0u);
              mx[kMaxTotal] = max(mx[kMaxTotal], q ? cd.z : 0u);
            }
          }
          set_lane(lo, hi, b, j);
        }
      }
    }
#else
    while (MIX && part_b) {  // mixed-model nodes: the exact per-card predicates from the record
      const int j = __builtin_ctzll(part_b);
      part_b &= part_b - 1;
      // (the record by the node's local id: a block-grouped run reads positions, ids)
      const uint32_t rid = ids ? ids[nb + (uint32_t)j] : nb + (uint32_t)j;
      const bool f = k1_node_lean<K>(nodes + (size_t)rid * NS, m, c, number,
                                     need_mem, need_clk, mx, nf, nz) && live;
      const uint64_t b = ballot(f);
      set_lane(lo, hi, b, (uint32_t)j);
    }
#endif
    // sparse masks: the block's (nz, full) words always, a node's own mask only when it is
    // neither empty nor the wave's live mask (the ALL / NONE nodes cost no mask traffic)
    const uint64_t mine = ((uint64_t)hi << 32) | lo;
    const bool nzl = valid && mine != 0ull, fulll = nzl && mine == live_mask;
    const uint64_t nz_b = ballot(nzl), full_b = ballot(fulll);
#ifndef YODA_ABL_K1_NOBM  // (write-traffic ablations: timing/counter builds only, wrong masks)
    if (nzl && !fulll) bmw[nb + lane] = mine;
#endif
#ifndef YODA_ABL_K1_NOBS
    // (a block with no feasible pod stays out of the block list and its BlockMask unwritten:
    // every reader checks the list first)
    if (lane == 0 && nz_b != 0ull) bsw[nb >> 6] = BlockMask{nz_b, full_b};
#endif
    if (nz_b != 0) {
      const uint32_t bi = nb >> 6;
      if ((bi >> 6) != blk_wi) {
        blk_flush();
        blk_wi = bi >> 6;
        blk_bits = 0;
      }
      blk_bits |= 1ull << (bi & 63u);
    }
  };
  // ALL blocks' counts, lane = block (summed across the wave at the end); g_nu: their nodes
  // the K2 will likely score per pod (the K2 cost hint, wts)
  uint32_t g_nf = 0, g_nz = 0, g_nu = 0;
  if (bsm != nullptr) {
    // Whole-block decisions from the block summaries (BlockSumWord), 64 blocks at a time,
    // lane = block: the bounds of a block's nodes against the wave's bounds prove every node
    // NONE, or every node ALL with one contribution (all qualifying: the block's maxima; none
    // qualifying: nothing).  Sufficient conditions of node_block's per-node tests, so the
    // outcome is the same; the undecided blocks then take node_block.
    const uint32_t b0 = n0 >> 6, b1 = (n1 + 63u) >> 6;
    for (uint32_t g = b0; g < b1; g += kWave) {
      const uint32_t bi = g + lane;
      const bool bv = bi < b1;
      const uint32_t* B = bsm + sum_index(bv ? bi : b0, 0, BST);  // word w at B[64 w]
      const K1BlockClass cls = k1_block_class(B, bv, kw);
      const bool bnone = cls.none, ball = cls.all, allq = cls.allq;
      const uint32_t nreal = cls.nreal;
      const uint64_t none_m = ballot(bnone), all_m = ballot(ball);
      if (ball) {
#ifndef YODA_ABL_K1_NOBS  // (NONE blocks: unlisted, unwritten)
        const uint64_t vb = nreal >= 64u ? ~0ull : ((1ull << nreal) - 1ull);
        bsw[bi] = BlockMask{vb, vb};
#endif
        // the words an ALL block folds in, issued together (one more round trip)
        const uint32_t nzt = B[64 * kBsNzt];
        uint32_t bmx[6];
#pragma unroll
        for (int f = 0; f < 6; ++f) bmx[f] = WIT ? 0u : B[64 * (kBsMx + f)];
        uint64_t lv = 0ull;  // the block's lv[l_hi]: a node every pod passes scores it
        if (seeding && kbub != nullptr) {
          const uint32_t* U = kbub + sum_index(bi, kbub_lvl(K) + 2u * l_hi, kbub_stride(K));
          lv = (uint64_t)U[0] | ((uint64_t)U[64] << 32);
        }
        // K2 cost hint (wts): a block whose q-th healthy frees straddle the wave's memory
        // range leaves the K2 counting qualifying cards per pod on its nodes
        bool nu = false;
        if (!WIT && wts != nullptr && s_m_min != s_m_max) {
#pragma unroll
          for (int q = 0; q < K; ++q)
            nu |= (B[64 * (kBsT + q)] <= s_m_max) & (B[64 * (kBsT + K + q)] > s_m_min);
        }
        g_nf += nreal;
        g_nz += nzt;
        g_nu += nu ? nreal : 0u;
        if (seeding && kbub != nullptr) {
          const double v = __longlong_as_double((long long)lv);
          if (v > 0.0) atomicMax(sdw, (unsigned long long)v);
        }
        if (allq) {
          if constexpr (WIT) {  // (the same rule as a node's: larger replaces, equal adds)
#pragma unroll
            for (int f = 0; f < 6; ++f) {
              const uint32_t v = B[64 * (kBsMx + f)], cnt = B[64 * (kBsWc + f)];
              const uint32_t low = (bi << 6) + B[64 * (kBsWl + f)];
              const bool gt = v > aw[f], eq = v == aw[f];
              ac[f] = gt ? cnt : ac[f] + (eq ? cnt : 0u);
              al[f] = gt ? low : (eq ? min(al[f], low) : al[f]);
              aw[f] = gt ? v : aw[f];
            }
          } else {
            a_bw = max(a_bw, bmx[kMaxBw]);
            a_ck = max(a_ck, bmx[kMaxClock]);
            a_core = max(a_core, bmx[kMaxCore]);
            a_free = max(a_free, bmx[kMaxFree]);
            a_pw = max(a_pw, bmx[kMaxPower]);
            a_tot = max(a_tot, bmx[kMaxTotal]);
          }
        }
      }
      if (all_m != 0ull && lane == 0) {  // blocks g .. g + 63 -> their block-list words
        const uint32_t sh = g & 63u;
        atomicOr(reinterpret_cast<unsigned long long*>(blkw + (g >> 6)),
                 (unsigned long long)(all_m << sh));
        if (sh != 0u && (all_m >> (64u - sh)) != 0ull)
          atomicOr(reinterpret_cast<unsigned long long*>(blkw + (g >> 6) + 1),
                   (unsigned long long)(all_m >> (64u - sh)));
      }
      if (STATS && !trace && lane == 0) {
        const uint64_t bvm = ballot(bv && nreal > 0u);
        atomicAdd(stats + 10, (unsigned long long)__builtin_popcountll(none_m));
        atomicAdd(stats + 11, (unsigned long long)__builtin_popcountll(all_m));
        (void)bvm;
      }
      if (STATS && !trace) {  // (wave, node) pairs of the decided blocks
        uint32_t na = ball ? nreal : 0u, nn = bnone ? nreal : 0u;
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) {
          na += (uint32_t)__shfl_xor((int)na, o, kWave);
          nn += (uint32_t)__shfl_xor((int)nn, o, kWave);
        }
        if (lane == 0) {
          atomicAdd(stats + 0, (unsigned long long)na);
          atomicAdd(stats + 1, (unsigned long long)nn);
        }
      }
      uint64_t und = ballot(bv && nreal > 0u) & ~(none_m | all_m);
      if (YODA_K1_PF && und) load_sum((g + (uint32_t)__builtin_ctzll(und)) << 6);
      while (und) {
        const uint32_t j = (uint32_t)__builtin_ctzll(und);
        und &= und - 1;
        node_block((g + j) << 6, und ? (g + (uint32_t)__builtin_ctzll(und)) << 6 : ~0u);
      }
    }
  } else {
    if (YODA_K1_PF && n0 < n1) load_sum(n0);
    for (uint32_t nb = n0; nb < n1; nb += kWave) node_block(nb, nb + kWave < n1 ? nb + kWave : ~0u);
  }
  const uint64_t t_pass = STATS ? wall_clock64() : 0ull;
  g_nf = wave_sum_u32(g_nf);
  g_nz = wave_sum_u32(g_nz);
  nf_all += g_nf;
  nz_all += g_nz;
  blk_flush();
  if (seeding && lane == 0) {  // this (wave, chunk)'s seed into the wave's (every chunk's; max)
    const unsigned long long w = *sdw;
    if (w != 0ull) atomicMax(seed_out + (p >> 6), w);
  }
  // the wave's weight for the K2's heaviest-first order (k_lpt_order): its PART nodes and the
  // ALL nodes above, summed over its chunks (one add per (wave, chunk); k_lpt_order reads and
  // re-zeroes them)
  if (wts != nullptr) {
    g_nu = wave_sum_u32(g_nu);
    const uint32_t wgt = npart + g_nu;
    if (lane == 0 && wgt != 0u) atomicAdd(wts + (p >> 6), wgt);
  }
  const size_t slot1 = ((size_t)(p >> 6) * C + chunk) * SUB + sub;
  if (trace && lane == 0 && slot1 < (size_t)(stats[15] >> 8)) {
    unsigned long long* tr = stats + 16 + 4 * slot1;
    tr[0] = t_start;
    tr[1] = wall_clock64();
    tr[2] = npart | ((unsigned long long)nblk << 32);
    tr[3] = (t_setup - t_start) | ((t_pass - t_start) << 32);
  }
  if constexpr (WIT) {
    // the ALL nodes' maxima, witness counts and lowest witnesses, folded into every pod lane
    // (the same rule as a node's: a larger maximum replaces, an equal one adds)
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const uint32_t M = wave_max_u32(aw[f]);
      uint32_t cnt = aw[f] == M ? ac[f] : 0u, low = aw[f] == M ? al[f] : 0xffffffffu;
#pragma unroll
      for (int o = kWave / 2; o > 0; o >>= 1) {
        cnt += (uint32_t)__shfl_xor((int)cnt, o, kWave);
        low = min(low, (uint32_t)__shfl_xor((int)low, o, kWave));
      }
      if (M > mx[f]) {
        mx[f] = M;
        wc[f] = cnt;
        wn[f] = low;
      } else if (M == mx[f]) {
        wc[f] += cnt;
        wn[f] = min(wn[f], low);
      }
    }
    if (!live) return;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const size_t o = ((size_t)f * C + chunk) * n_pods + p;
      pmax[o] = (uint64_t)mx[f];
      pwit[o] = wc[f];
      pwit[(size_t)6 * C * n_pods + o] = wn[f];
    }
    pcnt[((size_t)0 * C + chunk) * n_pods + p] = nf + nf_all;
    pcnt[((size_t)1 * C + chunk) * n_pods + p] = nz + nz_all;
    return;
  }
  // fold the ALL nodes into every pod lane
  a_bw = wave_max_u32(a_bw);
  a_ck = wave_max_u32(a_ck);
  a_core = wave_max_u32(a_core);
  a_free = wave_max_u32(a_free);
  a_pw = wave_max_u32(a_pw);
  a_tot = wave_max_u32(a_tot);
  if (SUB == 1 && cmask != nullptr) {
    // no pod of the wave has a feasible node in the chunk: its partials are the identity
    // (maxima at the floor, counts 0) -- nothing written, and k_reduce1 skips the chunk
    if (ballot(live && nf + nf_all != 0u) == 0ull) return;
    if (lane == 0) atomicOr(cmask + (p >> 6), 1ull << chunk);
  }
  if (SUB == 1 && !live) return;  // (lane 0 is live: the live lanes are a prefix)
  mx[kMaxBw] = max(mx[kMaxBw], a_bw);
  mx[kMaxClock] = max(mx[kMaxClock], a_ck);
  mx[kMaxCore] = max(mx[kMaxCore], a_core);
  mx[kMaxFree] = max(mx[kMaxFree], a_free);
  mx[kMaxPower] = max(mx[kMaxPower], a_pw);
  mx[kMaxTotal] = max(mx[kMaxTotal], a_tot);
  nf += nf_all;
  nz += nz_all;
  // N32: u32 partials (k_reduce1<true>), [nwords][C][P]: packed (nwords = kNarrowWords:
  // bandwidth | clock << 16, core | power << 16 -- each <= 65535 -- FreeMemory, TotalMemory as
  // u32 codes), or one word per field in kMax* order (kWideWords)
  uint32_t* pmax32 = reinterpret_cast<uint32_t*>(pmax);
  uint32_t pw4[kWideWords];
  if (nwords == kNarrowWords) {
    pw4[0] = mx[kMaxBw] | (mx[kMaxClock] << 16);
    pw4[1] = mx[kMaxCore] | (mx[kMaxPower] << 16);
    pw4[2] = mx[kMaxFree];
    pw4[3] = mx[kMaxTotal];
    pw4[4] = pw4[5] = 0u;
  } else {
#pragma unroll
    for (int f = 0; f < kWideWords; ++f) pw4[f] = mx[f];
  }
  if constexpr (SUB > 1) {
    // the quarters' partials through LDS (each wave's own region, free after its loop);
    // wave 0 folds them and writes the chunk's
    static_assert(RECS + kWave * REC >= (kWideWords + 2) * kWave, "LDS merge area");
#pragma unroll
    for (int f = 0; f < kWideWords; ++f) lds[f * kWave + lane] = pw4[f];
    lds[kWideWords * kWave + lane] = nf;
    lds[(kWideWords + 1) * kWave + lane] = nz;
    __syncthreads();
    if (sub != 0u || !live) return;
#pragma unroll
    for (int w = 1; w < SUB; ++w) {
      const uint32_t* o = lds_all[w];
#pragma unroll
      for (int f = 0; f < kWideWords; ++f)
        pw4[f] = narrow_max(pw4[f], o[f * kWave + lane], f, nwords);
      nf += o[kWideWords * kWave + lane];
      nz += o[(kWideWords + 1) * kWave + lane];
    }
  }
#ifdef YODA_ABL_K1_NOPART  // (write-traffic ablation: no partial stores)
  return;
#endif
  pmax32[((size_t)0 * C + chunk) * n_pods + p] = pw4[0];
  pmax32[((size_t)1 * C + chunk) * n_pods + p] = pw4[1];
  pmax32[((size_t)2 * C + chunk) * n_pods + p] = pw4[2];
  pmax32[((size_t)3 * C + chunk) * n_pods + p] = pw4[3];
  if (nwords != kNarrowWords) {
    pmax32[((size_t)4 * C + chunk) * n_pods + p] = pw4[4];
    pmax32[((size_t)5 * C + chunk) * n_pods + p] = pw4[5];
  }
  pcnt[((size_t)0 * C + chunk) * n_pods + p] = nf;
  pcnt[((size_t)1 * C + chunk) * n_pods + p] = nz;
}


// feasibility of (pod p, node n) in the [wave][node] bitmask
__device__ __forceinline__ bool bm_bit(const uint64_t* __restrict__ bm, uint32_t bm_stride,
                                       uint32_t p, uint32_t n) {
  return (bm[(size_t)(p >> 6) * bm_stride + n] >> (p & 63u)) & 1ull;
}

// Live pods of wave w of a batch of n_pods (bit l: pod 64 w + l < n_pods).
__device__ __forceinline__ uint64_t wave_live(uint32_t w, uint32_t n_pods) {
  const uint32_t rem = n_pods - min(n_pods, 64u * w);
  return rem >= 64u ? ~0ull : ((1ull << rem) - 1ull);
}

// Where a kernel reads the feasibility masks: dense [wave][node] (bs == nullptr; the per-node
// K1s) or the block K1's sparse form (yoda_layout.h BlockMask).
struct MaskSrc {
  const uint64_t* bm;
  const BlockMask* bs;
  uint32_t bm_stride, bs_stride;
  const uint64_t* blk;  // with bs: the wave's block list (a clear bit: no feasible pod, and
  uint32_t blk_stride;  // the block's BlockMask was not written this run)
};
__device__ __forceinline__ bool blk_listed(const uint64_t* blk, uint32_t blk_stride, uint32_t w,
                                           uint32_t b) {
  return (blk[(size_t)w * blk_stride + (b >> 6)] >> (b & 63u)) & 1ull;
}

// Mask of (wave w, node n) for a thread that reads single masks (not the hot kernels).
__device__ __forceinline__ uint64_t mask_at(const MaskSrc& m, uint32_t w, uint32_t n,
                                            uint32_t n_pods) {
  if (!m.bs) return m.bm[(size_t)w * m.bm_stride + n];
  if (!blk_listed(m.blk, m.blk_stride, w, n >> 6)) return 0ull;
  const BlockMask b = m.bs[(size_t)w * m.bs_stride + (n >> 6)];
  const uint32_t j = n & 63u;
  if ((b.full >> j) & 1ull) return wave_live(w, n_pods);
  if ((b.nz >> j) & 1ull) return m.bm[(size_t)w * m.bm_stride + n];
  return 0ull;
}

// Per-pod merge of K1 chunk partials -> maxima [6][P] and counts [2][P].  One thread per
// (pod, field) (grid.y = the 6 maxima + 2 counts), chunk loads unrolled so each thread keeps
// several in flight.  NARROW: u32 maxima partials (the N32 K1).
__device__ __forceinline__ double ru_100_over(double M);

// rcp != nullptr (a single-handle run, whose maxima are final here): each maxima thread also
// writes its field's reciprocals (k_prep2's, fused).  Packed partial words: narrow_max.
__device__ __forceinline__ void narrow_store(uint32_t v, int w, uint32_t n_pods, uint32_t p,
                                            uint64_t* maxima, const MemTab& mt,
                                            uint32_t nw = kNarrowWords) {
  auto put = [&](int f, uint64_t x) {
    if (mt.vf && f == kMaxFree) x = rank_value(x, mt.vf);  // memory ranks -> values
    if (mt.vf && f == kMaxTotal) x = rank_value(x, mt.vt);
    maxima[(size_t)f * n_pods + p] = x;
  };
  if (nw != kNarrowWords) {
    put(w, v);
  } else if (w == 0) {
    put(kMaxBw, v & 0xffffu);
    put(kMaxClock, v >> 16);
  } else if (w == 1) {
    put(kMaxCore, v & 0xffffu);
    put(kMaxPower, v >> 16);
  } else {
    put(w == 2 ? kMaxFree : kMaxTotal, v);
  }
}

// rcp rows: bw, core, power, free, total (k_prep2's order); the clock has none
__device__ __forceinline__ void store_rcp(int f, uint64_t mx, uint32_t n_pods, uint32_t p,
                                          double* rcp) {
  const int k = f == kMaxBw ? 0 : f == kMaxCore ? 1 : f == kMaxPower ? 2 : f == kMaxFree ? 3
              : f == kMaxTotal ? 4 : -1;
  if (rcp && k >= 0) rcp[(size_t)k * n_pods + p] = ru_100_over((double)mx);
}

// The block K2's pod-block order, heaviest first (longest processing time first: a heavy
// pod block that starts late sets the kernel's tail).  Weight = the pod block's PART nodes in
// K1 (wts [n_waves], summed over the chunks by k1_block_n32; zeroed here for the next run).
// One workgroup: each pod block's rank = the blocks heavier than it (ties: lower index
// first), counted over an LDS copy of the weights; n_pb <= kLptMax.
constexpr uint32_t kLptMax = 4096;
__device__ void lpt_order_body(uint32_t* __restrict__ wts, uint32_t n_waves, uint32_t n_pb,
                               uint32_t* __restrict__ order, uint32_t* __restrict__ w) {
  for (uint32_t i = threadIdx.x; i < n_pb; i += blockDim.x) {
    uint32_t s = 0;
    if (4 * i + 4 <= n_waves) {  // the block's four waves in one 16-byte load
      const uint4 q = reinterpret_cast<const uint4*>(wts)[i];
      reinterpret_cast<uint4*>(wts)[i] = make_uint4(0u, 0u, 0u, 0u);
      s = q.x + q.y + q.z + q.w;
    } else {
      for (uint32_t v = 4 * i; v < n_waves; ++v) {
        s += wts[v];
        wts[v] = 0u;
      }
    }
    w[i] = s;
  }
  const uint32_t n4 = (n_pb + 15u) & ~15u;  // zero padding (counts for no block)
  for (uint32_t i = n_pb + threadIdx.x; i < n4; i += blockDim.x) w[i] = 0u;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n_pb; i += blockDim.x) {
    const uint32_t wi = w[i];
    uint32_t r = 0;
    const uint4* w4 = reinterpret_cast<const uint4*>(w);
    for (uint32_t j = 0; j < n4; j += 16) {  // four 16-byte LDS reads in flight per trip
      uint4 q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = w4[(j >> 2) + (uint32_t)k];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = j + 4u * (uint32_t)k;
        r += (q[k].x > wi || (q[k].x == wi && b < i)) ? 1u : 0u;
        r += (q[k].y > wi || (q[k].y == wi && b + 1u < i)) ? 1u : 0u;
        r += (q[k].z > wi || (q[k].z == wi && b + 2u < i)) ? 1u : 0u;
        r += (q[k].w > wi || (q[k].w == wi && b + 3u < i)) ? 1u : 0u;
      }
    }
    order[r] = i;
  }
}
// Cost probe of the block K1, for its heaviest-first pod-block order (k1_order): per pod wave,
// how many of 64 blocks sampled evenly across the snapshot the wave's whole-block decisions
// (k1_block_class, the block K1's) leave to the per-node pass.  The node order deals every free
// level into any run of blocks, so the sample stands for the wave's chunks, and a
// wave's per-node work sets its tasks' length: in a K1 trace the wave explains 91 % of the task-
// time variance, and list scheduling the pod blocks heaviest first shortens the launch by a
// fifth (the tail of late long tasks).  wts[wave] = 1 + that count (k_lpt_order ranks them).
// Grid: one 256-pod block of the sorted batch per workgroup, one pod wave per wave.
__global__ __launch_bounds__(kBlock) void k1_probe(
    const uint32_t* __restrict__ m_in, const uint32_t* __restrict__ c_in,
    const uint64_t* __restrict__ number_in, const uint32_t* __restrict__ need_mem_in,
    const uint32_t* __restrict__ need_clk_in, uint32_t n_pods, uint32_t n_nodes,
    const uint32_t* __restrict__ bsm, uint32_t bst, uint32_t K, uint32_t* __restrict__ wts) {
  const uint32_t lane = lane_id();
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const bool live = p < n_pods;
  const uint64_t live_mask = ballot(live);
  if (live_mask == 0ull) return;
  uint32_t m = 0, c = 0, need_mem = 0, need_clk = 0;
  uint64_t number = ~0ull;
  if (live) {
    m = m_in[p];
    c = c_in[p];
    number = number_in[p];
    need_mem = need_mem_in[p];
    need_clk = need_clk_in[p];
  }
  // the block K1's wave bounds (k1_block_n32's set-up)
  const bool pm = live && need_mem > 0, pc = live && need_clk > 0;
  const uint64_t pm_mask = ballot(pm), pc_mask = ballot(pc);
  K1Wave w;
  w.any_pm = pm_mask != 0ull;
  w.all_pm = pm_mask == live_mask;
  w.any_pc = pc_mask != 0ull;
  w.all_pc = pc_mask == live_mask;
  w.num_max = wave_max_u64(live ? number : 0ull);
  w.num_min = wave_min_u64(live ? number : ~0ull);
  const uint32_t nm_max = wave_max_u32(pm ? need_mem : 0u);
  const uint32_t nm_min = wave_min_u32(pm ? need_mem : ~0u);
  w.mpm_max = wave_max_u32(pm ? m : 0u);
  w.mpm_min = wave_min_u32(pm ? m : ~0u);
  w.nc_max = wave_max_u32(pc ? need_clk : 0u);
  w.nc_min = wave_min_u32(pc ? need_clk : ~0u);
  w.cpc_max = wave_max_u32(pc ? c : 0u);
  const uint32_t cpc_min = wave_min_u32(pc ? c : ~0u);
  w.m_max = wave_max_u32(live ? m : 0u);
  w.m_min = wave_min_u32(live ? m : ~0u);
  w.c_max = wave_max_u32(live ? c : 0u);
  w.c_min = wave_min_u32(live ? c : ~0u);
  w.c_uni = cpc_min == w.cpc_max;
  w.hfs_all_ok = nm_max <= K;
  w.hfs_none_ok = nm_min <= K;
  w.bs_tn = kBsT + K + (w.hfs_none_ok && nm_min > 0u ? nm_min - 1u : 0u);
  w.bs_ta = kBsT + (w.any_pm && w.hfs_all_ok && nm_max > 0u ? nm_max - 1u : 0u);
  // 64 blocks spread over the snapshot, lane = block
  const uint32_t nb = (n_nodes + kWave - 1) / kWave;
  const uint32_t bi = nb >= kWave ? (uint32_t)(((uint64_t)lane * nb) / kWave) : lane;
  const bool bv = bi < nb;
  const K1BlockClass cls = k1_block_class(bsm + sum_index(bv ? bi : 0u, 0, bst), bv, w, false);
  const uint64_t und = ballot(bv && cls.nreal > 0u && !cls.none && !cls.all);
  if (lane == 0) wts[p >> 6] = 1u + (uint32_t)__builtin_popcountll(und);
}

__global__ __launch_bounds__(1024) void k_lpt_order(uint32_t* __restrict__ wts,
                                                    uint32_t n_waves, uint32_t n_pb,
                                                    uint32_t* __restrict__ order) {
  __shared__ __attribute__((aligned(16))) uint32_t w[kLptMax];
  lpt_order_body(wts, n_waves, n_pb, order, w);
}

template <bool NARROW>
__global__ __launch_bounds__(kBlock) void k_reduce1(const uint64_t* __restrict__ pmax,
                                                    const uint32_t* __restrict__ pcnt, uint32_t C,
                                                    uint32_t n_pods,
                                                    uint64_t* __restrict__ maxima,
                                                    uint32_t* __restrict__ counts,
                                                    double* __restrict__ rcp,
                                                    MemTab mt, uint32_t nw,
                                                    uint32_t* __restrict__ lpt_w = nullptr,
                                                    uint32_t* __restrict__ lpt_order = nullptr,
                                                    const unsigned long long* __restrict__ cmask = nullptr) {
  if (lpt_w != nullptr && blockIdx.x == gridDim.x - 1) {  // the extra block: the K2's order
    __shared__ __attribute__((aligned(16))) uint32_t w[kLptMax];
    if (blockIdx.y == 0)
      lpt_order_body(lpt_w, (n_pods + kWave - 1) / kWave, (n_pods + kBlock - 1) / kBlock,
                     lpt_order, w);
    return;
  }
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t f = blockIdx.y;  // NARROW: the nw partial words, then the 2 counts
  const uint32_t NF = NARROW ? nw : 6u;
  if (p >= n_pods) return;
  if (f < NF) {
    if constexpr (NARROW) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(pmax) + (size_t)f * C * n_pods + p;
      uint32_t m32 = narrow_floor((int)f, nw);  // floor 1 (collection.go:31-38)
      if (cmask != nullptr) {  // only the chunks that wrote (the wave's bits; uniform loop)
        for (uint64_t bits = cmask[p >> 6]; bits != 0ull; bits &= bits - 1ull)
          m32 = narrow_max(m32, src[(size_t)__builtin_ctzll(bits) * n_pods], (int)f, nw);
      } else {
#pragma unroll 8
        for (uint32_t c = 0; c < C; ++c)
          m32 = narrow_max(m32, src[(size_t)c * n_pods], (int)f, nw);
      }
      narrow_store(m32, (int)f, n_pods, p, maxima, mt, nw);
      if (rcp && nw != kNarrowWords) {
        store_rcp((int)f, maxima[(size_t)f * n_pods + p], n_pods, p, rcp);
      } else if (rcp) {
        const int fa = f == 0 ? kMaxBw : f == 1 ? kMaxCore : f == 2 ? kMaxFree : kMaxTotal;
        store_rcp(fa, maxima[(size_t)fa * n_pods + p], n_pods, p, rcp);
        if (f == 1) store_rcp(kMaxPower, maxima[(size_t)kMaxPower * n_pods + p], n_pods, p, rcp);
      }
    } else {
      uint64_t mx = 1;
      const uint64_t* src = pmax + (size_t)f * C * n_pods + p;
#pragma unroll 8
      for (uint32_t c = 0; c < C; ++c) mx = umax64(mx, src[(size_t)c * n_pods]);
      if (mt.vf && f == kMaxFree) mx = rank_value(mx, mt.vf);  // memory ranks -> values
      if (mt.vf && f == kMaxTotal) mx = rank_value(mx, mt.vt);
      maxima[(size_t)f * n_pods + p] = mx;
      store_rcp((int)f, mx, n_pods, p, rcp);
    }
  } else {
    const uint32_t* src = pcnt + (size_t)(f - NF) * C * n_pods + p;
    uint32_t s = 0;
    if (cmask != nullptr) {
      for (uint64_t bits = cmask[p >> 6]; bits != 0ull; bits &= bits - 1ull)
        s += src[(size_t)__builtin_ctzll(bits) * n_pods];
    } else {
#pragma unroll 8
      for (uint32_t c = 0; c < C; ++c) s += src[(size_t)c * n_pods];
    }
    counts[(size_t)(f - NF) * n_pods + p] = s;
  }
}

// Wave-per-pod variant of k_reduce1 for many chunks (small pod batches, e.g. the greedy
// single-pod fallback): the 64 lanes stride over the chunks, then a shuffle reduction.
template <bool NARROW>
__global__ __launch_bounds__(kWave) void k_reduce1_wave(const uint64_t* __restrict__ pmax,
                                                         const uint32_t* __restrict__ pcnt,
                                                         uint32_t C, uint32_t n_pods,
                                                         uint64_t* __restrict__ maxima,
                                                         uint32_t* __restrict__ counts,
                                                         MemTab mt, uint32_t nw) {
  const uint32_t p = blockIdx.x, lane = threadIdx.x;
  if constexpr (NARROW) {
    for (int w = 0; w < (int)nw; ++w) {
      uint32_t m = narrow_floor(w, nw);
      for (uint32_t c = lane; c < C; c += kWave)
        m = narrow_max(m, reinterpret_cast<const uint32_t*>(pmax)[((size_t)w * C + c) * n_pods + p],
                       w, nw);
      for (int o = kWave / 2; o > 0; o >>= 1)
        m = narrow_max(m, (uint32_t)__shfl_xor((int)m, o, kWave), w, nw);
      if (lane == 0) narrow_store(m, w, n_pods, p, maxima, mt, nw);
    }
  } else {
    for (int f = 0; f < 6; ++f) {
      uint64_t mx = 1;
      for (uint32_t c = lane; c < C; c += kWave) mx = umax64(mx, pmax[((size_t)f * C + c) * n_pods + p]);
      for (int o = kWave / 2; o > 0; o >>= 1) mx = umax64(mx, __shfl_xor(mx, o, kWave));
      if (mt.vf && f == kMaxFree) mx = rank_value(mx, mt.vf);  // memory ranks -> values
      if (mt.vf && f == kMaxTotal) mx = rank_value(mx, mt.vt);
      if (lane == 0) maxima[(size_t)f * n_pods + p] = mx;
    }
  }
  for (int f = 0; f < 2; ++f) {
    uint32_t sum = 0;
    for (uint32_t c = lane; c < C; c += kWave) sum += pcnt[((size_t)f * C + c) * n_pods + p];
    for (int o = kWave / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o, kWave);
    if (lane == 0) counts[(size_t)f * n_pods + p] = sum;
  }
}

// Split variant of k_reduce1 for many chunks (small pod batches: greedy windows): thread =
// (pod, field) as in k_reduce1 (coalesced over pods), grid.z splits the chunks, and each
// split folds its share into the outputs with one atomic (maxima and counts zeroed before;
// every chunk's maxima partial is >= 1, the CollectMaxValues floor).
template <bool NARROW>
__global__ __launch_bounds__(kBlock) void k_reduce1_split(const uint64_t* __restrict__ pmax,
                                                          const uint32_t* __restrict__ pcnt,
                                                          uint32_t C, uint32_t n_pods,
                                                          uint64_t* __restrict__ maxima,
                                                          uint32_t* __restrict__ counts,
                                                          uint32_t nw) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x, f = blockIdx.y;
  const uint32_t NF = NARROW ? nw : 6u;
  if (p >= n_pods || f >= NF + 2u) return;
  const uint32_t S = gridDim.z, per = (C + S - 1) / S;
  const uint32_t c0 = blockIdx.z * per, c1 = min(C, c0 + per);
  if (c0 >= c1) return;
  auto amax = [&](int fo, uint64_t v) {
    atomicMax(reinterpret_cast<unsigned long long*>(maxima + (size_t)fo * n_pods + p),
              (unsigned long long)v);
  };
  if (f < NF) {
    if constexpr (NARROW) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(pmax) + (size_t)f * C * n_pods + p;
      uint32_t m32 = 0;
#pragma unroll 8
      for (uint32_t c = c0; c < c1; ++c)
        m32 = narrow_max(m32, src[(size_t)c * n_pods], (int)f, nw);
      if (nw != kNarrowWords) {
        amax((int)f, m32);
      } else if (f == 0) {
        amax(kMaxBw, m32 & 0xffffu);
        amax(kMaxClock, m32 >> 16);
      } else if (f == 1) {
        amax(kMaxCore, m32 & 0xffffu);
        amax(kMaxPower, m32 >> 16);
      } else {
        amax(f == 2 ? kMaxFree : kMaxTotal, m32);
      }
    } else {
      const uint64_t* src = pmax + (size_t)f * C * n_pods + p;
      uint64_t mx = 0;
#pragma unroll 8
      for (uint32_t c = c0; c < c1; ++c) mx = umax64(mx, src[(size_t)c * n_pods]);
      amax((int)f, mx);
    }
  } else {
    const uint32_t* src = pcnt + (size_t)(f - NF) * C * n_pods + p;
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t c = c0; c < c1; ++c) sum += src[(size_t)c * n_pods];
    atomicAdd(counts + (size_t)(f - NF) * n_pods + p, sum);
  }
}

// Memory ranks: scv/memory -> its rank threshold 2 + #{distinct card frees < m} (binary search
// in mt.vf[2 .. nf + 1], ascending; the frees are <= 2^44, so the f64 compares are exact), or,
// without ranks (mt.vf == nullptr), the plain N32 clamp min(m, 2^32 - 1).
__global__ __launch_bounds__(kBlock) void k_mem_rank(const uint64_t* __restrict__ m_u,
                                                     uint32_t n_pods, MemTab mt,
                                                     uint32_t* __restrict__ m32) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const uint64_t m = m_u[p];
  if (!mt.vf) {
    m32[p] = m > 0xffffffffull ? 0xffffffffu : (uint32_t)m;
    return;
  }
  const double md = (double)(m < (1ull << 53) ? m : (1ull << 53));
  uint32_t lo = 0, hi = mt.nf;  // first index with value >= m
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (mt.vf[2u + mid] < md) lo = mid + 1u; else hi = mid;
  }
  m32[p] = 2u + lo;
}

hipError_t launch_mem_rank(const uint64_t* m_u, uint32_t n_pods, const MemTab& mt, uint32_t* m32,
                           hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  hipLaunchKernelGGL(k_mem_rank, pod_grid(n_pods), dim3(kBlock), 0, s, m_u, n_pods, mt, m32);
  return hipGetLastError();
}

// Memory ranks: the free / total rows of maxima [6][P] reduced in rank space (the split
// reductions' atomics) -> values.
__global__ __launch_bounds__(kBlock) void k_rank_maxima(uint64_t* __restrict__ maxima,
                                                        uint32_t n_pods, MemTab mt) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  uint64_t* f = maxima + (size_t)kMaxFree * n_pods + p;
  uint64_t* t = maxima + (size_t)kMaxTotal * n_pods + p;
  *f = rank_value(*f, mt.vf);
  *t = rank_value(*t, mt.vt);
}

// RU(100 / M): the smallest double >= 100/M.  With every card field <= 2^44,
// floor(x * RU(100/M)) == floor(100 x / M) exactly.
__device__ __forceinline__ double ru_100_over(double M) {
  double r = 100.0 / M;  // IEEE round-to-nearest
  const double e = __builtin_fma(r, M, -100.0);  // exact sign of r*M - 100
  if (e < 0.0) r = __longlong_as_double(__double_as_longlong(r) + 1);
  return r;
}

// Per-pod reciprocals of the (all-reduced) maxima, f64 for all five divisors (every record
// path).
__global__ __launch_bounds__(kBlock) void k_prep2(const uint64_t* __restrict__ maxima,
                                                  uint32_t n_pods, double* __restrict__ rcp) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const int src[5] = {kMaxBw, kMaxCore, kMaxPower, kMaxFree, kMaxTotal};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const double M = (double)maxima[(size_t)src[k] * n_pods + p];
    rcp[(size_t)k * n_pods + p] = ru_100_over(M);
  }
}

// A capacity greedy window's outputs, from the batch's sorted order into window order, written
// straight into the host's mapped staging pages in one launch (instead of five copies and a
// host-side permutation): out = counts [2][wn] u32 | maxima [6][wn] u64 | witnesses [12][wn]
// u32 | top scores [kt][wn] f64 | top nodes [kt][wn] u32.  perm[q] = window index of sorted
// position q (nullptr: unsorted); each workgroup inverts it for its own 256 window slots, so the
// writes to host memory are coalesced and the gathers stay on the device.
__global__ __launch_bounds__(kBlock) void k_window_out(
    const uint32_t* __restrict__ counts, const uint64_t* __restrict__ maxima,
    const uint32_t* __restrict__ wit, const double* __restrict__ tk_s,
    const uint32_t* __restrict__ tk_i, const uint32_t* __restrict__ perm, uint32_t wn,
    uint32_t kt, int row_major, unsigned char* __restrict__ out, uint32_t* __restrict__ inv_out) {
  __shared__ uint32_t inv[kBlock];
  const uint32_t w0 = blockIdx.x * kBlock, w = w0 + threadIdx.x;
  if (perm) {
    for (uint32_t q = threadIdx.x; q < wn; q += kBlock) {
      const uint32_t x = perm[q];
      if (x >= w0 && x < w0 + kBlock) inv[x - w0] = q;
    }
    __syncthreads();
  }
  if (w >= wn) return;
  const uint32_t q = perm ? inv[threadIdx.x] : w;
  uint32_t* o_cnt = reinterpret_cast<uint32_t*>(out);
  uint64_t* o_mx = reinterpret_cast<uint64_t*>(out + 8 * (size_t)wn);
  uint32_t* o_wit = reinterpret_cast<uint32_t*>(out + 56 * (size_t)wn);
  double* o_ts = reinterpret_cast<double*>(out + 104 * (size_t)wn);
  uint32_t* o_ti = reinterpret_cast<uint32_t*>(out + (104 + 8 * (size_t)kt) * wn);
  for (uint32_t f = 0; f < 2; ++f) o_cnt[(size_t)f * wn + w] = counts[(size_t)f * wn + q];
  for (uint32_t f = 0; f < 6; ++f) o_mx[(size_t)f * wn + w] = maxima[(size_t)f * wn + q];
  for (uint32_t f = 0; f < 12; ++f) o_wit[(size_t)f * wn + w] = wit[(size_t)f * wn + q];
  if (inv_out) {  // the lists: k_window_lists, one thread per (pod, entry)
    inv_out[w] = q;
    return;
  }
  // the lists [k][wn], or [wn][k] (row_major: each pod's list contiguous for the host's scan)
  for (uint32_t k = 0; k < kt; ++k) {
    const size_t o = row_major ? (size_t)w * kt + k : (size_t)k * wn + w;
    o_ts[o] = tk_s[(size_t)k * wn + q];
    o_ti[o] = tk_i[(size_t)k * wn + q];
  }
}

// The window's candidate lists into the staging layout of k_window_out, one thread per (pod,
// entry) -- consecutive threads write consecutive entries (row_major: one pod's list) -- from
// the sorted positions inv[w] that k_window_out found.  (One thread per pod looping over a
// 64-deep list took 36-49 us per capacity window: 3 workgroups on the device.)
__global__ __launch_bounds__(kBlock) void k_window_lists(
    const double* __restrict__ tk_s, const uint32_t* __restrict__ tk_i,
    const uint32_t* __restrict__ inv, uint32_t wn, uint32_t kt, int row_major,
    unsigned char* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (size_t)wn * kt) return;
  double* o_ts = reinterpret_cast<double*>(out + 104 * (size_t)wn);
  uint32_t* o_ti = reinterpret_cast<uint32_t*>(out + (104 + 8 * (size_t)kt) * wn);
  const uint32_t w = row_major ? (uint32_t)(t / kt) : (uint32_t)(t % wn);
  const uint32_t k = row_major ? (uint32_t)(t - (size_t)w * kt) : (uint32_t)(t / wn);
  const uint32_t q = inv[w];
  o_ts[t] = tk_s[(size_t)k * wn + q];
  o_ti[t] = tk_i[(size_t)k * wn + q];
}

// CalculateCardScore's bandwidth, clock / MaxBandwidth (algorithm.go:283), 2 core and power
// terms of a card (or of a one-model node's model) under the reciprocals r, as products of
// the u32 fields in RS: f64 always exact (x, M < 2^32: 300 x + M < 2^53), f32 when every
// small field is <= kF32SmallMax (300 x + M < 2^24) -- the quotient lemma, DESIGN.md §5.
template <typename RS>
__device__ __forceinline__ uint32_t card_shared_terms(uint32_t bw, uint32_t ck, uint32_t core,
                                                      uint32_t pw, RS r_bw, RS r_core, RS r_pow) {
  return (uint32_t)((RS)bw * r_bw) + (uint32_t)((RS)ck * r_bw) +
         2u * (uint32_t)((RS)core * r_core) + (uint32_t)((RS)pw * r_pow);
}
// RU32(100 / M) from r = RU(100 / M) in f64: the smallest float >= r, which is the smallest
// float >= 100 / M (a float in [100 / M, r) would be a double below r).
__device__ __forceinline__ float ru32_of(double r) {
  float f = (float)r;
  if ((double)f < r) f = __int_as_float(__float_as_int(f) + 1);
  return f;
}
template <typename RS>
__device__ __forceinline__ RS rcp_as(double r) {
  if constexpr (sizeof(RS) == 4) return ru32_of(r);
  else return r;
}

// The "G table" (N32 block K2): for the snapshot-wide maxima G (per CalculateCardScore field,
// the max over every real card, floor 1 -- the PreScore maxima of any pod whose feasible
// nodes include the maximal cards, which is most pods of a large cluster) the per-node terms
// the block K2 otherwise recomputes in every (wave, block): shared = the node's bandwidth,
// clock/MaxBandwidth, 2 core and power quotients, and the prefix sums of 3 q_free + q_total
// over its free-sorted cards, stored as the basic scores B[q] = q shared + prefix[q] of the
// q = 1..K qualifying-card counts (tile layout, sum_index with gtab_stride).  A wave whose
// reciprocals equal G's (compared bit for bit) reads them instead.
// (struct GTab, gtab_stride: yoda_layout.h)

__device__ __forceinline__ uint32_t card_mem_term(uint32_t f, uint32_t t, double r_free,
                                                  double r_tot) {
  return 3u * (uint32_t)((double)f * r_free) + (uint32_t)((double)t * r_tot);
}
// With memory ranks (RK, yoda_layout.h MemTab) f and t are ranks: their values from the tables.
// The block K2 takes RK as a template parameter (a kernel of its own for rank snapshots: the
// gathers' registers never reach the plain kernel).
template <bool RK>
__device__ __forceinline__ uint32_t mem_term(uint32_t f, uint32_t t, double r_free, double r_tot,
                                             const MemTab& mt) {
  if constexpr (RK) return 3u * (uint32_t)(mt.vf[f] * r_free) + (uint32_t)(mt.vt[t] * r_tot);
  return 3u * (uint32_t)((double)f * r_free) + (uint32_t)((double)t * r_tot);
}
// the same with a run-time test (mt.vf: wave-uniform) for the sites outside the block kernels
__device__ __forceinline__ uint32_t card_mem_term(uint32_t f, uint32_t t, double r_free,
                                                  double r_tot, const MemTab& mt) {
  const double fv = mt.vf ? mt.vf[f] : (double)f, tv = mt.vf ? mt.vt[t] : (double)t;
  return 3u * (uint32_t)(fv * r_free) + (uint32_t)(tv * r_tot);
}

// Build the G table (GTab above) of the N32 snapshot: g_max = G per maxima field (kMax*
// order); rcp_out <- G's reciprocals (f64 bw, core, power, free, total: 10 words) for the host
// to hand to K2.  One thread per node, tile layout.
template <int K>
__global__ __launch_bounds__(kBlock) void k_gtable(const uint32_t* __restrict__ sum2,
                                                   const uint32_t* __restrict__ mix,
                                                   uint32_t n_nodes, const uint64_t* __restrict__ g_max,
                                                   uint32_t* __restrict__ tab,
                                                   uint32_t* __restrict__ rcp_out, MemTab mt) {
  const uint32_t n = blockIdx.x * kBlock + threadIdx.x;
  const double r_bw = ru_100_over((double)g_max[kMaxBw]);
  const double r_core = ru_100_over((double)g_max[kMaxCore]);
  const double r_pow = ru_100_over((double)g_max[kMaxPower]);
  const double r_free = ru_100_over((double)g_max[kMaxFree]);
  const double r_tot = ru_100_over((double)g_max[kMaxTotal]);
  if (n == 0) {
    const double r[5] = {r_bw, r_core, r_pow, r_free, r_tot};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint64_t b = (uint64_t)__double_as_longlong(r[k]);
      rcp_out[2 * k] = (uint32_t)b;
      rcp_out[2 * k + 1] = (uint32_t)(b >> 32);
    }
  }
  if (n >= ((n_nodes + 63u) & ~63u)) return;  // padded tail lanes: zero summaries
  constexpr uint32_t S2 = k2sum_stride(K), GS = gtab_stride(K), MS = mix_stride(K);
  auto w = [&](uint32_t word) { return sum2[sum_index(n, word, S2)]; };
  auto x = [&](uint32_t word) { return mix[sum_index(n, word, MS)]; };
  const bool uni = (w(kS2Meta) & kSumUni4) != 0u;
  const uint32_t shared =
      card_shared_terms(w(kS2Bw), w(kS2Clock), w(kS2Core), w(kS2Power), r_bw, r_core, r_pow);
  uint32_t acc = 0;
#pragma unroll
  for (int t = 0; t < K; ++t) {
    // a mixed-model node: each card's own model terms (every card counted: the row a wave
    // uses when the node's lowest clock passes every pod's scv/clock)
    const uint32_t sh = uni ? shared
                            : card_shared_terms(x(mix_word(kMixBw, t, K)), x(mix_word(kMixCk, t, K)),
                                                x(mix_word(kMixCo, t, K)), x(mix_word(kMixPw, t, K)),
                                                r_bw, r_core, r_pow);
    acc += card_mem_term(w(kS2Fs + t), w(kS2Fs + K + t), r_free, r_tot, mt) + (uni ? 0u : sh);
    tab[sum_index(n, t, GS)] = (uni ? (uint32_t)(t + 1) * shared : 0u) + acc;  // B[t + 1]
  }
}

hipError_t launch_lpt_order(uint32_t* wts, uint32_t n_pods, uint32_t* order, hipStream_t s) {
  const uint32_t n_waves = (n_pods + kWave - 1) / kWave, n_pb = (n_pods + kBlock - 1) / kBlock;
  if (n_pb == 0 || n_pb > kLptMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_lpt_order, dim3(1), dim3(1024), 0, s, wts, n_waves, n_pb, order);
  return hipGetLastError();
}

// The block K1's heaviest-first pod-block order: k1_probe's per-wave weights into wts, ranked by
// k_lpt_order into order (n_pb entries).
hipError_t launch_k1_order(int K, const PodParams& pp, uint32_t n_pods, uint32_t n_nodes,
                           uint32_t* wts, uint32_t* order, hipStream_t s) {
  const uint32_t n_pb = (n_pods + kBlock - 1) / kBlock;
  if (n_pb == 0 || n_pb > kLptMax || pp.bsum == nullptr || K < 1 || K > 16)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k1_probe, dim3(n_pb), dim3(kBlock), 0, s, pp.m_32, pp.c_32, pp.number,
                     pp.need_mem, pp.need_clk, n_pods, n_nodes, pp.bsum, bsum_stride(K),
                     (uint32_t)K, wts);
  const hipError_t e = hipGetLastError();
  return e != hipSuccess ? e : launch_lpt_order(wts, n_pods, order, s);
}

// K2 block bounds (yoda_layout.h kbub_*): one wave per 64-node block, lane = node.
template <int K>
__global__ __launch_bounds__(kWave) void k_block_ub(const uint32_t* __restrict__ sum2,
                                                    const uint32_t* __restrict__ tab,
                                                    uint32_t n_nodes, uint32_t* __restrict__ out,
                                                    const uint32_t* __restrict__ levels) {
  constexpr uint32_t S2 = k2sum_stride(K), GS = gtab_stride(K), BW = kbub_stride(K) / 4u;
  const uint32_t b = blockIdx.x, n = b * 64u + threadIdx.x;
  const bool v = n < n_nodes;
  auto o_at = [&](uint32_t w) -> uint32_t& { return out[sum_index(b, w, 4u * BW)]; };
  double stat = -1.0;
  uint32_t cnt = 0;
  if (v) {
    stat = __longlong_as_double((long long)((uint64_t)sum2[sum_index(n, kS2Static, S2)] |
                                            ((uint64_t)sum2[sum_index(n, kS2Static + 1, S2)] << 32)));
    cnt = (sum2[sum_index(n, kS2Meta, S2)] >> 8) & 0xffu;
  }
  uint32_t bq = 0;  // B_G[min(j, cnt)], j ascending
#pragma unroll
  for (int j = 0; j <= K; ++j) {
    if (j > 0 && v && (uint32_t)j <= cnt) bq = tab[sum_index(n, (uint32_t)j - 1u, GS)];
    double u = v ? stat + (double)bq : -1.0;  // exact: integers below 2^53
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) u = fmax(u, __shfl_xor(u, off, kWave));
    if (threadIdx.x == 0) {
      const uint64_t ub = (uint64_t)__double_as_longlong(u);
      o_at(2 * j) = (uint32_t)ub;
      o_at(2 * j + 1) = (uint32_t)(ub >> 32);
    }
  }
  uint32_t fs[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    fs[k] = v ? sum2[sum_index(n, kS2Fs + (uint32_t)k, S2)] : 0u;
    const uint32_t fm = wave_max_u32(fs[k]);
    if (threadIdx.x == 0) o_at(kbub_fmax(K) + k) = fm;
  }
  // the level bounds lv[l]: static + B_G[nq(t_l)] maximised over the block's real nodes
  for (uint32_t l = 0; l < kKbLevels; ++l) {
    const uint32_t t = levels[l];
    uint32_t q = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) q += fs[k] >= t ? 1u : 0u;
    q = min(q, cnt);
    const uint32_t bq2 = (v && q > 0u) ? tab[sum_index(n, q - 1u, GS)] : 0u;
    double u = v ? stat + (double)bq2 : -1.0;  // exact: integers below 2^53
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) u = fmax(u, __shfl_xor(u, off, kWave));
    if (threadIdx.x == 0) {
      const uint64_t ub = (uint64_t)__double_as_longlong(u);
      o_at(kbub_lvl(K) + 2u * l) = (uint32_t)ub;
      o_at(kbub_lvl(K) + 2u * l + 1u) = (uint32_t)(ub >> 32);
    }
  }
}

// The non-G block bounds (yoda_layout.h kbdec_*): one wave per 64-node block, lane = node.
// Memory ranks (mt.vf): the summaries' free / total words are ranks, compared with the levels
// as they are (the same order) and summed as their VALUES (the tables), which is what the
// bound's reciprocals multiply.
template <int K>
__global__ __launch_bounds__(kWave) void k_block_dec(const uint32_t* __restrict__ sum2,
                                                     const uint32_t* __restrict__ mix,
                                                     uint32_t n_nodes, uint32_t* __restrict__ out,
                                                     const uint32_t* __restrict__ levels,
                                                     MemTab mt) {
  constexpr uint32_t S2 = k2sum_stride(K), DS = kbdec_stride();
  const uint32_t b = blockIdx.x, n = b * 64u + threadIdx.x;
  const bool v = n < n_nodes;
  auto o_at = [&](uint32_t w) -> uint32_t& { return out[sum_index(b, w, DS)]; };
  auto put_d = [&](uint32_t w, double d) {
    const uint64_t u = (uint64_t)__double_as_longlong(d);
    o_at(w) = (uint32_t)u;
    o_at(w + 1u) = (uint32_t)(u >> 32);
  };
  auto w2 = [&](uint32_t word) { return sum2[sum_index(n, word, S2)]; };
  double stat = -1.0;
  uint32_t cnt = 0, meta = 0, bw = 0, ck = 0, co = 0, pw = 0;
  uint32_t fs[K], ts[K];
  if (v) {
    stat = __longlong_as_double((long long)((uint64_t)w2(kS2Static) |
                                            ((uint64_t)w2(kS2Static + 1) << 32)));
    meta = w2(kS2Meta);
    cnt = (meta >> 8) & 0xffu;
    bw = w2(kS2Bw);
    ck = w2(kS2Clock);
    co = w2(kS2Core);
    pw = w2(kS2Power);
  }
  // A node of several GPU models (no kSumUni4): each card's model terms are at most those of
  // the node's largest card values (shared_M is non-decreasing in each), so the bound holds
  // with them; its qualifying cards for a pod are a subset of the cards with free >= the pod's
  // scv/memory (collection.go:46 adds the clock test), so ql / fl / tl bound them as well.
  const bool mixed = v && (meta & kSumUni4) == 0u;
  if (mixed && mix != nullptr) {
    const uint32_t MS = mix_stride(K);
    auto x = [&](uint32_t word) { return mix[sum_index(n, word, MS)]; };
    bw = ck = co = pw = 0u;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const bool real = (uint32_t)t < cnt;
      bw = max(bw, real ? x(mix_word(kMixBw, t, K)) : 0u);
      ck = max(ck, real ? x(mix_word(kMixCk, t, K)) : 0u);
      co = max(co, real ? x(mix_word(kMixCo, t, K)) : 0u);
      pw = max(pw, real ? x(mix_word(kMixPw, t, K)) : 0u);
    }
  }
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const bool real = v && (uint32_t)t < cnt;
    fs[t] = real ? w2(kS2Fs + (uint32_t)t) : 0u;
    ts[t] = real ? w2(kS2Fs + (uint32_t)K + (uint32_t)t) : 0u;
  }
  const bool ok = ballot(mixed && mix == nullptr) == 0ull;
  const double st = wave_max_f64(stat);
  const uint32_t mbw = wave_max_u32(bw), mck = wave_max_u32(ck), mco = wave_max_u32(co),
                 mpw = wave_max_u32(pw);
  if (threadIdx.x == 0) {
    o_at(kDecOk) = ok ? 1u : 0u;
    o_at(kDecBw) = mbw;
    o_at(kDecCk) = mck;
    o_at(kDecCo) = mco;
    o_at(kDecPw) = mpw;
    put_d(kDecStat, st);
  }
  for (uint32_t l = 0; l < kKbLevels; ++l) {
    const uint32_t t = levels[l];
    uint32_t q = 0;
    double f = 0.0, tt = 0.0;  // exact: sums of at most 16 values below 2^44
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool in = fs[k] >= t && (uint32_t)k < cnt;
      q += in ? 1u : 0u;
      f += in ? (mt.vf ? mt.vf[fs[k]] : (double)fs[k]) : 0.0;
      tt += in ? (mt.vt ? mt.vt[ts[k]] : (double)ts[k]) : 0.0;
    }
    const uint32_t mq = wave_max_u32(q);
    const double mf = wave_max_f64(f), mt = wave_max_f64(tt);
    if (threadIdx.x == 0) {
      o_at(kDecQl + l) = mq;
      put_d(kbdec_fl(l), mf);
      put_d(kbdec_tl(l), mt);
    }
  }
}

hipError_t launch_block_dec(int K, const uint32_t* sum2, const uint32_t* mix, uint32_t n_nodes,
                            uint32_t* out, const uint32_t* levels, MemTab mt, hipStream_t s) {
  if (n_nodes == 0) return hipSuccess;
  const dim3 grid((n_nodes + 63) / 64);
  switch (K) {
    case 1: hipLaunchKernelGGL(k_block_dec<1>, grid, dim3(kWave), 0, s, sum2, mix, n_nodes, out, levels, mt); break;
    case 2: hipLaunchKernelGGL(k_block_dec<2>, grid, dim3(kWave), 0, s, sum2, mix, n_nodes, out, levels, mt); break;
    case 4: hipLaunchKernelGGL(k_block_dec<4>, grid, dim3(kWave), 0, s, sum2, mix, n_nodes, out, levels, mt); break;
    case 8: hipLaunchKernelGGL(k_block_dec<8>, grid, dim3(kWave), 0, s, sum2, mix, n_nodes, out, levels, mt); break;
    case 16: hipLaunchKernelGGL(k_block_dec<16>, grid, dim3(kWave), 0, s, sum2, mix, n_nodes, out, levels, mt); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_block_ub(int K, const uint32_t* sum2, const uint32_t* tab, uint32_t n_nodes,
                           uint32_t* out, const uint32_t* levels, hipStream_t s) {
  if (n_nodes == 0) return hipSuccess;
  const dim3 grid((n_nodes + 63) / 64);
  switch (K) {
    case 1: hipLaunchKernelGGL(k_block_ub<1>, grid, dim3(kWave), 0, s, sum2, tab, n_nodes, out, levels); break;
    case 2: hipLaunchKernelGGL(k_block_ub<2>, grid, dim3(kWave), 0, s, sum2, tab, n_nodes, out, levels); break;
    case 4: hipLaunchKernelGGL(k_block_ub<4>, grid, dim3(kWave), 0, s, sum2, tab, n_nodes, out, levels); break;
    case 8: hipLaunchKernelGGL(k_block_ub<8>, grid, dim3(kWave), 0, s, sum2, tab, n_nodes, out, levels); break;
    case 16: hipLaunchKernelGGL(k_block_ub<16>, grid, dim3(kWave), 0, s, sum2, tab, n_nodes, out, levels); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_gtable(int K, const uint32_t* sum2, const uint32_t* mix, uint32_t n_nodes,
                         const uint64_t* g_max, uint32_t* tab, uint32_t* rcp_out, MemTab mt,
                         hipStream_t s) {
  const dim3 grid(((n_nodes + 63u) & ~63u) / kBlock + 1);
  switch (K) {
    case 1: hipLaunchKernelGGL(k_gtable<1>, grid, dim3(kBlock), 0, s, sum2, mix, n_nodes, g_max, tab, rcp_out, mt); break;
    case 2: hipLaunchKernelGGL(k_gtable<2>, grid, dim3(kBlock), 0, s, sum2, mix, n_nodes, g_max, tab, rcp_out, mt); break;
    case 4: hipLaunchKernelGGL(k_gtable<4>, grid, dim3(kBlock), 0, s, sum2, mix, n_nodes, g_max, tab, rcp_out, mt); break;
    case 8: hipLaunchKernelGGL(k_gtable<8>, grid, dim3(kBlock), 0, s, sum2, mix, n_nodes, g_max, tab, rcp_out, mt); break;
    case 16: hipLaunchKernelGGL(k_gtable<16>, grid, dim3(kBlock), 0, s, sum2, mix, n_nodes, g_max, tab, rcp_out, mt); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// K2 on the fast paths: CalculateBasicScore + Allocate + Actual (algorithm.go:96,264-310),
// exact.  A Scorer holds one pod's thresholds and reciprocals in VGPRs and
// scores one node record (read through the scalar path).
struct ScoreArgs {
  const double* m_f;
  const double* c_f;
  const uint32_t* m_32;
  const uint32_t* c_32;
  const double* rcp;    // [5][P] f64: bw, core, power, free, total
  const uint32_t* cnt = nullptr;  // [P] feasible-node counts (phase 1), or none
  GTab g = {};                    // the snapshot-wide maxima's per-node terms (tab: none)
  const uint32_t* mix = nullptr;  // per-card models in free order (yoda_layout.h MixWord)
  MemTab mt = {};                 // memory ranks (yoda_layout.h MemTab)
  const uint32_t* ids = nullptr;  // block-grouped node order: the local id of each position
  const uint32_t* kbub = nullptr; // K2 block bounds (yoda_layout.h kbub_*): argmax pruning
  const uint64_t* hot = nullptr;  // blocks of the highest bounds (bit b % 64 of word b / 64):
                                  // visited first, so that the best so far rises early
  const uint32_t* pb_order = nullptr;  // the block K2's pod-block visiting order (or none)
  // argmax pruning: the block K1's per-wave seeds (a lower bound on every live pod's best,
  // PodParams::seed) and the free levels of kbub's lv[] bounds (nullptr: none)
  const unsigned long long* seed = nullptr;
  const uint32_t* levels = nullptr;
  // the non-G block bounds (kbdec_*) and the per-pod best shared across the chunks (PodParams)
  const uint32_t* kbdec = nullptr;
  unsigned long long* gbest = nullptr;
  // the argmax block K2's chunk mask (PodParams::cmask2; nullptr: every chunk writes)
  unsigned long long* cmask = nullptr;
};

template <Path P>
struct Scorer;


// F64: every quotient in f64; each term is an exact integer < 2^52, so the sum is exact in
// any order and the weights fold into FMAs.
template <>
struct Scorer<Path::F64> {
  using R = Rec<Path::F64>;
  double m = 0, c = 0, r_bw = 0, r_core = 0, r_pow = 0, r_free = 0, r_tot = 0;
  __device__ void load(const ScoreArgs& a, uint32_t p, uint32_t n_pods) {
    m = a.m_f[p];
    c = a.c_f[p];
    r_bw = a.rcp[0 * (size_t)n_pods + p];
    r_core = a.rcp[1 * (size_t)n_pods + p];
    r_pow = a.rcp[2 * (size_t)n_pods + p];
    r_free = a.rcp[3 * (size_t)n_pods + p];
    r_tot = a.rcp[4 * (size_t)n_pods + p];
  }
  template <int K>
  __device__ __forceinline__ double raw(const unsigned char* rec) const {
    const double stat = reinterpret_cast<const NodeHdrF*>(rec)->static_score;
    const Group<double, K> fr = load_group<double, K>(rec + R::off(kFree, K));
    const Group<double, K> ck = load_group<double, K>(rec + R::off(kClock, K));
    const Group<double, K> bw = load_group<double, K>(rec + R::off(kBandwidth, K));
    const Group<double, K> co = load_group<double, K>(rec + R::off(kCore, K));
    const Group<double, K> pw = load_group<double, K>(rec + R::off(kPower, K));
    const Group<double, K> to = load_group<double, K>(rec + R::off(kTotal, K));
    double basic = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      // CalculateCardScore (algorithm.go:280-291): each quotient truncates before its
      // weight; clock is divided by MaxBandwidth (:283).
      double sc = __builtin_trunc(bw.v[j] * r_bw);
      sc += __builtin_trunc(ck.v[j] * r_bw);
      sc = __builtin_fma(__builtin_trunc(co.v[j] * r_core), 2.0, sc);
      sc += __builtin_trunc(pw.v[j] * r_pow);
      sc = __builtin_fma(__builtin_trunc(fr.v[j] * r_free), 3.0, sc);
      sc += __builtin_trunc(to.v[j] * r_tot);
      basic += ((fr.v[j] >= m) & (ck.v[j] >= c)) ? sc : 0.0;  // algorithm.go:271
    }
    return basic + stat;
  }
};

// N32: u32 card fields, the small-field quotients in RS (card_shared_terms: f64, or f32 where
// its lemma holds -- the block K2's WQ = false), the memory quotients in f64, the card score
// summed in u32 (the host bounds it: yoda_capi.cpp n32_ok).
template <typename RS>
struct ScorerN32 {
  uint32_t m = 0, c = 0;
  RS r_bw = 0, r_core = 0, r_pow = 0;
  double r_free = 0, r_tot = 0;
  __device__ void load(const ScoreArgs& a, uint32_t p, uint32_t n_pods) {
    m = a.m_32[p];
    c = a.c_32[p];
    r_bw = rcp_as<RS>(a.rcp[0 * (size_t)n_pods + p]);
    r_core = rcp_as<RS>(a.rcp[1 * (size_t)n_pods + p]);
    r_pow = rcp_as<RS>(a.rcp[2 * (size_t)n_pods + p]);
    r_free = a.rcp[3 * (size_t)n_pods + p];
    r_tot = a.rcp[4 * (size_t)n_pods + p];
  }
  template <int K>
  __device__ __forceinline__ double raw(const unsigned char* rec) const {
    const NodeHdrF* hd = reinterpret_cast<const NodeHdrF*>(rec);
    const double stat = hd->static_score;
    if (hd->flags & kNodeUniform4) {
      // One GPU model: the bandwidth, clock, core and power quotients are the same for every
      // real card, so the card-score sum factors into  nq * shared + sum(3 q_free + q_tot)
      // over the nq qualifying real cards — the same integers, added in another order.
      const Group<uint32_t, K> fr = load_group<uint32_t, K>(rec + n32_u32_off(kFree, K));
      auto u0 = [&](int f) { return reinterpret_cast<const uint32_t*>(rec + n32_u32_off(f, K))[0]; };
      const uint32_t ck0 = u0(kClock);
      const Group<double, K> frd = load_group<double, K>(rec + n32_f64_off(kF64Free, K));
      const Group<double, K> tod = load_group<double, K>(rec + n32_f64_off(kF64Total, K));
      uint32_t shared = card_shared_terms(u0(kBandwidth), ck0, u0(kCore), u0(kPower), r_bw,
                                          r_core, r_pow);
      uint32_t nq = 0, mem = 0;
      if (hd->flags & kNodeUniformTotal) {
        shared += (uint32_t)(tod.v[0] * r_tot);
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const uint32_t q = ((hd->real_mask >> j) & 1u) & (uint32_t)(fr.v[j] >= m);
          mem += q ? 3u * (uint32_t)(frd.v[j] * r_free) : 0u;
          nq += q;
        }
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const uint32_t q = ((hd->real_mask >> j) & 1u) & (uint32_t)(fr.v[j] >= m);
          const uint32_t t = 3u * (uint32_t)(frd.v[j] * r_free) + (uint32_t)(tod.v[j] * r_tot);
          mem += q ? t : 0u;
          nq += q;
        }
      }
      const uint32_t basic = (ck0 >= c) ? nq * shared + mem : 0u;  // algorithm.go:271
      return (double)basic + stat;
    }
    const Group<uint32_t, K> fr = load_group<uint32_t, K>(rec + n32_u32_off(kFree, K));
    const Group<uint32_t, K> ck = load_group<uint32_t, K>(rec + n32_u32_off(kClock, K));
    const Group<uint32_t, K> bwu = load_group<uint32_t, K>(rec + n32_u32_off(kBandwidth, K));
    const Group<uint32_t, K> cou = load_group<uint32_t, K>(rec + n32_u32_off(kCore, K));
    const Group<uint32_t, K> pwu = load_group<uint32_t, K>(rec + n32_u32_off(kPower, K));
    const Group<double, K> frd = load_group<double, K>(rec + n32_f64_off(kF64Free, K));
    const Group<double, K> tod = load_group<double, K>(rec + n32_f64_off(kF64Total, K));
    uint32_t basic = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      // CalculateCardScore (algorithm.go:280-291); clock / MaxBandwidth (:283)
      uint32_t sc = card_shared_terms(bwu.v[j], ck.v[j], cou.v[j], pwu.v[j], r_bw, r_core, r_pow) +
                    (uint32_t)(tod.v[j] * r_tot) + 3u * (uint32_t)(frd.v[j] * r_free);
      basic += ((fr.v[j] >= m) & (ck.v[j] >= c)) ? sc : 0u;  // algorithm.go:271
    }
    return (double)basic + stat;  // algorithm.go:96
  }
};
template <>
struct Scorer<Path::N32> : ScorerN32<double> {};

__device__ __forceinline__ uint32_t rec_stride(Path p, int K) {
  return p == Path::N32 ? n32_stride(K) : node_stride(K);
}

// Output flavours of the fast K2: running argmax (OUT_ARGMAX), argmax + every feasible raw
// score to rows[n][p] (OUT_ROWS, the plugin row mode), or the TOPK best (score, node) per pod
// sorted by (score desc, node asc) into tk_s/tk_i [C][TOPK][P] (greedy candidates).
enum K2Out { OUT_ARGMAX = 0, OUT_ROWS = 1, OUT_TOPK = 2 };
// Candidates per pod: 8 for the reference-faithful greedy, 16 for the capacity mode (whose
// lists go stale faster: picks also remove nodes).  kTopK is the default.
constexpr int kTopK = 8;
constexpr int kTopKCap = 16;

template <int K, Path PATH, int OUT, int TK = kTopK>
__global__ __launch_bounds__(kBlock) void k2_score(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    ScoreArgs args, uint32_t n_pods, const MaskSrc ms,
    double* __restrict__ pbest, uint32_t* __restrict__ pidx, uint32_t* __restrict__ pties,
    double* __restrict__ plow, int64_t* __restrict__ rows, double* __restrict__ tk_s,
    uint32_t* __restrict__ tk_i) {
  const Tile tl = tile();
  const uint32_t p = tl.pb * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  const uint64_t live_mask = ballot(live);
  if (live_mask == 0) return;  // a wave past the batch
  const uint32_t w = uniform_u32(p >> 6);
  const uint64_t* bmw = ms.bm + (size_t)w * ms.bm_stride;
  const uint32_t lane = lane_id();
  Scorer<PATH> sc;
  if (live) sc.load(args, p, n_pods);
  constexpr uint32_t stride = PATH == Path::N32 ? n32_stride(K) : node_stride(K);
  double best = -1.0, low = 1.0e300;
  uint32_t idx = 0xffffffffu, ties = 0;
  double ts[OUT == OUT_TOPK ? TK : 1];
  uint32_t ti[OUT == OUT_TOPK ? TK : 1];
  if constexpr (OUT == OUT_TOPK) {
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      ts[k] = -1.0;
      ti[k] = 0xffffffffu;
    }
  }
  // score node n for this lane's pod (the caller checked the lane's feasibility bit)
  auto visit = [&](uint32_t n) {
    const double raw = sc.template raw<K>(nodes + (size_t)n * stride);
    if constexpr (OUT == OUT_ROWS) rows[(size_t)n * n_pods + p] = (int64_t)raw;
    if constexpr (OUT == OUT_TOPK) {
      // strict '>' keeps the earlier (lower) node first among equal scores
      if (raw > ts[TK - 1]) {
        double cs = raw;
        uint32_t ci = n;
#pragma unroll
        for (int k = 0; k < TK; ++k) {
          // (score desc, node asc): a carried entry that ties a slot must still shift
          const bool gt = cs > ts[k] || (cs == ts[k] && ci < ti[k]);
          const double os = ts[k];
          const uint32_t oi = ti[k];
          ts[k] = gt ? cs : os;
          ti[k] = gt ? ci : oi;
          cs = gt ? os : cs;
          ci = gt ? oi : ci;
        }
      }
    } else {
      if (raw > best) {
        best = raw;
        idx = n;
        ties = 1;
      } else if (raw == best) {
        ++ties;
      }
      low = fmin(low, raw);
    }
  };
  if (ms.bs) {
    // sparse masks: one (nz, full) pair per 64 nodes through the scalar path; a partial
    // node's own mask is one more scalar load
    const BlockMask* bsw = ms.bs + (size_t)w * ms.bs_stride;
    for (uint32_t nb = n0; nb < n1; nb += kWave) {
      if (!blk_listed(ms.blk, ms.blk_stride, w, nb >> 6)) continue;
      const BlockMask bk = bsw[nb >> 6];
      uint64_t bits = bk.nz;
      while (bits) {
        const uint32_t j = (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1;
        const uint32_t n = nb + j;
        const uint64_t mj = ((bk.full >> j) & 1ull) ? live_mask : bmw[n];
        if ((mj >> lane) & 1ull) visit(n);
      }
    }
  } else {
    // The wave's feasibility masks of 8 nodes come in with one scalar load; a node no pod of
    // the wave can use costs a scalar compare, a group of 8 such nodes one more.
    for (uint32_t g = n0; g < n1; g += 8) {
      const Group<uint64_t, 8> mk = load_group<uint64_t, 8>(
          reinterpret_cast<const unsigned char*>(bmw + g));
      if ((mk.v[0] | mk.v[1] | mk.v[2] | mk.v[3] | mk.v[4] | mk.v[5] | mk.v[6] | mk.v[7]) == 0)
        continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t n = g + (uint32_t)j;
        if (mk.v[j] == 0 || n >= n1) continue;
        if ((mk.v[j] >> lane) & 1ull) visit(n);
      }
    }
  }
  if (!live) return;
  if constexpr (OUT == OUT_TOPK) {
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      const size_t o = ((size_t)chunk * TK + k) * n_pods + p;
      tk_s[o] = ts[k];
      tk_i[o] = ti[k];
    }
  } else {
    const size_t o = (size_t)chunk * n_pods + p;
    pbest[o] = best;
    pidx[o] = idx;
    pties[o] = ties;
    plow[o] = low;
  }
}

// K2, block-classified (N32 path, argmax output).  After K1 the pods of a wave usually share
// their PreScore maxima (same feasible set), so the reciprocals RU(100/M) are the same on
// every lane ("uniform maxima", checked once per wave).  The wave then walks its chunk in
// blocks of 64 nodes with LANE = NODE and, for every one-model node, computes with those
// uniform reciprocals the node's shared quotient sum and the prefix sums of its free-sorted
// card terms (3 q_free + q_total) into LDS.  A node is
//   U     if every pod of the wave is feasible on it and has the same qualifying cards
//         (no real card's free memory between the wave's min and max scv/memory, clock not
//         between its min and max scv/clock): its score is one number for the whole wave,
//         folded into node-lane argmax/ties/min state that is reduced once per chunk;
//   FAST  a one-model node that is not U: each pod lane counts its qualifying cards nq and
//         reads  nq * shared + prefix[nq]  from LDS (the same integers as Scorer<N32>);
//   EXACT anything else (mixed-model node, or non-uniform maxima): Scorer<N32>::raw.
// Every term is an exact integer < 2^52 in each form, so all three give the same raw score.
//
// TKO > 0 (greedy candidate lists): instead of the argmax, each pod's TKO best (score, node)
// pairs as packed keys  score << ib | (2^ib - 1 - node)  (a larger key is a higher score, or
// the same score on a lower node: the (score desc, node asc) order of the per-pair top-k; the
// host guarantees score < 2^(64 - ib) and n_nodes < 2^ib), sorted descending into
// tk_keys[chunk][pod][TKO] (0 = no entry).  U nodes go into one wave-uniform list (their score
// is the same on every active lane), the per-pod nodes into a per-lane list; the two are merged
// at the end of the chunk.
#ifndef YODA_K2_WAVES
#define YODA_K2_WAVES 5
#endif
// MIX = false: a snapshot whose every node is one GPU model (kSumUni4): no mixed-model rows
// and no exact per-pod Scorer in the kernel.
// Q32: the small-field quotients in f32 (host: every bandwidth / clock / core / power <=
// kF32SmallMax, where the f32 quotient lemma holds; fewer registers than f64), else f64.
template <int K, bool STATS, int TKO = 0, bool RK = false, bool MIX = true, bool Q32 = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(K <= 8 ? (TKO == 0 ? YODA_K2_WAVES : (TKO <= 8 ? 4 : 3)) : 1))) void k2_block_n32(
    const unsigned char* __restrict__ nodes, const unsigned char* __restrict__ sum2,
    uint32_t n_nodes, uint32_t chunk_nodes, ScoreArgs args, uint32_t n_pods,
    const uint64_t* __restrict__ bm, uint32_t bm_stride, const BlockMask* __restrict__ bs,
    uint32_t bs_stride, const uint64_t* __restrict__ blk,
    uint32_t blk_stride, double* __restrict__ pbest,
    uint32_t* __restrict__ pidx, uint32_t* __restrict__ pties, double* __restrict__ plow,
    unsigned long long* __restrict__ stats, uint64_t* __restrict__ tk_keys, uint32_t ib) {
  constexpr uint32_t S2 = k2sum_stride(K), NS = n32_stride(K), MS = mix_stride(K);
  constexpr bool TOPK = TKO > 0;
  constexpr int TL = TOPK ? TKO : 1;
  constexpr uint32_t PSW = K + 2;  // LDS words per node: B[0..K] (B[q] = q shared + prefix[q]), pad
  constexpr uint32_t TAB = kWave * PSW;  // the prefix table: 64 nodes
  // node records (below): 16 words -- 8 of header, then 4 basic scores (uniform maxima) or
  // the (basic at nq_lo, at nq_lo + 1) pair of each reciprocal set
  constexpr uint32_t kSets = 4, REC = 16;
  // LDS per wave: prefix table | 64 node records | the sets' reciprocals (5 f64, 16 words each).
  // No lowest score: on this path NormalizeScore cannot overflow, so the
  // lowest raw score is never read (the chunk merge reports the best in its place).
  // + the nodes' local ids of a block-grouped run (args.ids)
  // TT > 1 (top-k lists, whose small diverse windows have several reciprocal sets per wave):
  // prefix rows B_q[0..K] of every one-model node for each of the first TT sets (row 0 in the
  // table above, the others after the ids), so the per-pod pass reads a lane's basic score as
  // in a uniform wave instead of computing its card terms per node
  constexpr uint32_t TT = (TOPK && !RK) ? (TKO > 8 ? 3u : 2u) : 1u;
  // (RCPS: the sets' reciprocals, then one more slot: the decoupled bound's, below)
  constexpr uint32_t RECS = TAB, RCPS = TAB + kWave * REC, IDW = RCPS + 16 * (kSets + 1),
                     XTAB = IDW + kWave, LDSW = XTAB + (TT - 1) * TAB;
  auto row_base = [&](uint32_t q) -> uint32_t { return q == 0 ? 0u : XTAB + (q - 1u) * TAB; };
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[kBlock / kWave][LDSW];
  const uint32_t lane = lane_id();
  uint32_t* lds = lds_all[threadIdx.x >> 6];
  const Tile tl = tile();
  // args.pb_order: the pod blocks heaviest first (k_lpt_order), so the long ones do not start last
  const uint32_t pbk = args.pb_order ? args.pb_order[tl.pb] : tl.pb;
  const uint32_t p = pbk * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  const uint64_t live_mask = ballot(live);
  if (live_mask == 0) return;  // a wave past the batch
  // STATS with stats[15] set: the timing trace only (no per-block counter atomics)
  const bool trace = STATS && (stats[15] & 0xffull) == 1ull;
  const uint64_t t_start = STATS ? wall_clock64() : 0ull;
  const uint64_t* bmw = bm + (size_t)uniform_u32(p >> 6) * bm_stride;
  const BlockMask* bsw = bs ? bs + (size_t)uniform_u32(p >> 6) * bs_stride : nullptr;
  using RS = std::conditional_t<Q32, float, double>;  // small-field reciprocal type
  ScorerN32<RS> sc;
  if (live) sc.load(args, p, n_pods);
  // A pod feasible on no node has no bit in any mask: it takes no part in the wave's bounds
  // and reciprocal sets, and its outputs stay "no node".
  const bool act = live && (args.cnt == nullptr || args.cnt[p] != 0u);
  const uint64_t act_mask = ballot(act);
  // every active lane's maxima are at most G's (its reciprocals at least G's): the K1 seed, a
  // score under G, is then a lower bound of the wave's scores (thr below)
  bool seed_le_g = false;
  if constexpr (!TOPK) {
    if (args.seed != nullptr && args.g.tab != nullptr) {
      bool le;
      if constexpr (Q32)
        le = sc.r_bw >= args.g.f_bw && sc.r_core >= args.g.f_core && sc.r_pow >= args.g.f_pow;
      else
        le = sc.r_bw >= args.g.r_bw && sc.r_core >= args.g.r_core && sc.r_pow >= args.g.r_pow;
      le = le && sc.r_free >= args.g.r_free && sc.r_tot >= args.g.r_tot;
      seed_le_g = (ballot(act && !le) == 0ull);
    }
  }
  // Reciprocal sets: active lanes with the same (bw, core, power, free, total) reciprocals,
  // numbered in order of their first lane; up to kSets, any further lanes "overflow".
  auto rl_d = [&](double x, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return __longlong_as_double((long long)((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
        (int)(uint32_t)b, l) | ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(
        (int)(uint32_t)(b >> 32), l) << 32)));
  };
  uint32_t set = 0, nsets = 0;
  bool has_set = false;  // this lane is in one of the sets (else it overflowed them)
  uint64_t rem = act_mask;
  auto rl_s = [&](RS x, int l) -> RS {
    if constexpr (Q32) return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
    else return rl_d(x, l);
  };
  RS u_bw = 0, u_core = 0, u_pow = 0;  // set 0's reciprocals (wave-uniform)
  double u_free = 0.0, u_tot = 0.0;
  for (; rem != 0ull && nsets < kSets; ++nsets) {
    const int l = __builtin_ctzll(rem);
    const RS b_bw = rl_s(sc.r_bw, l), b_core = rl_s(sc.r_core, l), b_pow = rl_s(sc.r_pow, l);
    const double b_free = rl_d(sc.r_free, l), b_tot = rl_d(sc.r_tot, l);
    const bool in = act && sc.r_bw == b_bw && sc.r_core == b_core && sc.r_pow == b_pow &&
                    sc.r_free == b_free && sc.r_tot == b_tot;
    const uint64_t in_b = ballot(in) & rem;
    if ((in_b >> lane) & 1ull) {
      set = nsets;
      has_set = true;
    }
    rem &= ~in_b;
    if (nsets == 0) {
      u_bw = b_bw;
      u_core = b_core;
      u_pow = b_pow;
      u_free = b_free;
      u_tot = b_tot;
    }
    if (lane == (uint32_t)l) {  // (bw, core, power in RS at word 0; free, total at word 8)
      RS* r = reinterpret_cast<RS*>(lds + RCPS + 16 * nsets);
      r[0] = b_bw;
      r[1] = b_core;
      r[2] = b_pow;
      double* d = reinterpret_cast<double*>(lds + RCPS + 16 * nsets + 8);
      d[0] = b_free;
      d[1] = b_tot;
    }
  }
  const bool uni_max = nsets <= 1u && rem == 0ull;  // "uniform maxima"
  const bool rec_ok = rem == 0ull;  // every active lane has a set: node records serve it
  // the wave's reciprocals are the snapshot-wide maxima's: the G table serves its terms
  RS g_bw, g_core, g_pow;
  if constexpr (Q32) {
    g_bw = args.g.f_bw;
    g_core = args.g.f_core;
    g_pow = args.g.f_pow;
  } else {
    g_bw = args.g.r_bw;
    g_core = args.g.r_core;
    g_pow = args.g.r_pow;
  }
  const bool use_g = uni_max && args.g.tab != nullptr && u_bw == g_bw && u_core == g_core &&
                     u_pow == g_pow && u_free == args.g.r_free && u_tot == args.g.r_tot;
  const uint32_t m_max = wave_max_u32(act ? sc.m : 0u), m_min = wave_min_u32(act ? sc.m : ~0u);
  const uint32_t c_max = wave_max_u32(act ? sc.c : 0u), c_min = wave_min_u32(act ? sc.c : ~0u);
  // Block pruning (argmax, G waves): a block whose bound -- the most any node of it can score
  // for a pod with at most J qualifying cards, J from the block's largest frees and the wave's
  // smallest scv/memory (kbub_*) -- is below every active lane's best so far cannot hold a
  // pick or a tie of any of them.  thr: the min over active lanes of that best, refreshed
  // after each block the wave works on (it only grows, so a stale value stays a lower bound).
  // TOPK (greedy windows): a block whose best possible key cannot beat any active lane's
  // k-th key (thrk: the min over active lanes of their own and the U list's k-th) is skipped.
  // Non-G uniform waves (one reciprocal set, not G's -- e.g. clock-labelled pods, whose feasible
  // nodes are one GPU model): the decoupled bounds kbdec_* (argmax, no memory ranks).
  // Several reciprocal sets: the largest reciprocal of each field over the active lanes (the
  // smallest maxima) gives the highest score any of them can make, so the bound holds for all.
  const bool dec = args.kbdec != nullptr && !use_g && act_mask != 0ull;
  const bool prune = args.kbub != nullptr && (use_g || dec);
  if (dec) {  // the bound's reciprocals into the extra RCPS slot (RS at word 0, f64 at word 8)
    RS d_bw = act ? sc.r_bw : (RS)0, d_core = act ? sc.r_core : (RS)0, d_pow = act ? sc.r_pow : (RS)0;
    double d_free = act ? sc.r_free : 0.0, d_tot = act ? sc.r_tot : 0.0;
    if constexpr (Q32) {
      d_bw = wave_allreduce(d_bw, OpMaxF32{});
      d_core = wave_allreduce(d_core, OpMaxF32{});
      d_pow = wave_allreduce(d_pow, OpMaxF32{});
    } else {
      d_bw = wave_allreduce(d_bw, OpMaxF64{});
      d_core = wave_allreduce(d_core, OpMaxF64{});
      d_pow = wave_allreduce(d_pow, OpMaxF64{});
    }
    d_free = wave_allreduce(d_free, OpMaxF64{});
    d_tot = wave_allreduce(d_tot, OpMaxF64{});
    if (lane == 0) {
      RS* r = reinterpret_cast<RS*>(lds + RCPS + 16 * kSets);
      r[0] = d_bw;
      r[1] = d_core;
      r[2] = d_pow;
      double* d = reinterpret_cast<double*>(lds + RCPS + 16 * kSets + 8);
      d[0] = d_free;
      d[1] = d_tot;
    }
  }
  constexpr uint32_t KBST = kbub_stride(K);
  // The block K1's seed: a score every live pod of the wave reaches on some node it passes,
  // under the G maxima.  A pod whose maxima are at most G's field by field (reciprocals at
  // least G's) scores at least as much under its own, so no pod's best -- nor a tie of it --
  // lies below, and thr starts there instead of at -1.  On one handle that always holds (a
  // max over fewer cards); on a node shard the exchanged maxima can exceed this shard's G
  // (another shard holds a faster model), so the wave checks it (tests/test_gpu_shard_seeds.py).
  double thr = -1.0;
  if (prune && !TOPK && args.seed != nullptr) {
    const uint64_t sv = args.seed[uniform_u32(p >> 6)];
    if (sv != 0ull && (use_g || seed_le_g)) thr = (double)sv;  // (an integer below 2^53)
  }
  // the largest free level <= the wave's smallest scv/memory: every active pod qualifies at
  // most nq(t) cards on every node, so kbub's lv[l_lo] bounds the block too (its word: lvw)
  uint32_t lvw = 0, l_lo = 0;
  if (prune && args.levels != nullptr) {
    for (uint32_t l = 1; l < kKbLevels; ++l) l_lo = args.levels[l] <= m_min ? l : l_lo;
    l_lo = uniform_u32(l_lo);
    lvw = kbub_lvl(K) + 2u * l_lo;
  }
  uint64_t thrk = 0ull;

  double ubest = -1.0;                      // node lane (U nodes)
  uint32_t uidx = 0xffffffffu, uties = 0;
  // pod lane, every per-pod node: integer scores (static part + basic, exact below 2^53);
  // (0, 0 ties) is the empty state -- a first score of 0 counts as a tie of it
  uint64_t rbest = 0;
  uint32_t ridx = 0xffffffffu, rties = 0;
  auto to_u = [](double x) {  // an integer-valued double in [0, 2^52) -> its value
    return (uint64_t)__double_as_longlong(x + 4503599627370496.0) - 0x4330000000000000ull;
  };
  uint32_t npart = 0;  // STATS: per-pod-pass nodes of this (wave, chunk)
  // TOPK: the lane's list (per-pod nodes) and the wave-uniform list (U nodes), descending
  uint64_t pl[TL], ul[TL];
#pragma unroll
  for (int k = 0; k < TL; ++k) pl[k] = ul[k] = 0ull;
  const uint32_t imax = TOPK ? (1u << ib) - 1u : 0u;
  // insert key x into the lane's sorted list (x > pl[TL - 1])
  auto pl_insert = [&](uint64_t x) {
#pragma unroll
    for (int k = 0; k < TL; ++k) {
      const uint64_t o = pl[k];
      const bool gt = x > o;
      pl[k] = gt ? x : o;
      x = gt ? o : x;
    }
  };
  // One block: the wave's mask of node nb + lane and its summary (kept for the per-pod pass,
  // read back with v_readlane), loaded together: one memory latency per block.
  bool worked = false;  // the last block() call did the block's work (not pruned / empty)
  // a block's bound for this wave (kbub_*): J = the most cards any pod of the wave can
  // qualify on any node of it (from the block's largest frees and the wave's smallest
  // scv/memory), ub = static + B_G[J] maximised over the block's nodes
  auto block_ub = [&](uint32_t b) -> double {
    if (dec) {  // static + nq shared + 3 r_free F + r_total T, each maximised over the block
      constexpr uint32_t DS = kbdec_stride();
      const uint32_t* D = args.kbdec;
      if (args.levels == nullptr) return HUGE_VAL;
      // every word loaded before the first test (one round trip; the ok flag gated them before)
      const uint32_t ok = D[sum_index(b, kDecOk, DS)];
      const uint32_t wbw = D[sum_index(b, kDecBw, DS)], wck = D[sum_index(b, kDecCk, DS)];
      const uint32_t wco = D[sum_index(b, kDecCo, DS)], wpw = D[sum_index(b, kDecPw, DS)];
      const uint32_t wq = D[sum_index(b, kDecQl + l_lo, DS)];
      uint32_t w2[6];
      const uint32_t wsrc[3] = {kDecStat, kbdec_fl(l_lo), kbdec_tl(l_lo)};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        w2[2 * i] = D[sum_index(b, wsrc[i], DS)];
        w2[2 * i + 1] = D[sum_index(b, wsrc[i] + 1u, DS)];
      }
      __builtin_amdgcn_sched_group_barrier(0x0020, 12, 0);  // (the VMEM reads above, grouped)
      auto d64 = [&](int i) {
        return __longlong_as_double((long long)((uint64_t)w2[2 * i] | ((uint64_t)w2[2 * i + 1] << 32)));
      };
      const RS* r = reinterpret_cast<const RS*>(lds + RCPS + 16 * kSets);
      const double* rd = reinterpret_cast<const double*>(lds + RCPS + 16 * kSets + 8);
      const uint32_t sh = card_shared_terms(wbw, wck, wco, wpw, r[0], r[1], r[2]);
      const double q = (double)wq;
      // (+1: the f64 rounding of the products; the scores are integers)
      const double ub = d64(0) + q * (double)sh + 3.0 * rd[0] * d64(1) + rd[1] * d64(2) + 1.0;
      return ok == 0u ? HUGE_VAL : ub;
    }
    const uint32_t* U = args.kbub;
    // the block's K largest frees and its level bound, all in flight together (the level
    // words do not depend on J); then the J-indexed bound: two round trips
    uint32_t fm[K];
#pragma unroll
    for (int k = 0; k < K; ++k) fm[k] = U[sum_index(b, kbub_fmax(K) + (uint32_t)k, KBST)];
    // (lvw == 0: no level bound -- words 0 and 1 read and ignored, so no branch splits the group)
    const uint32_t lv_lo = U[sum_index(b, lvw, KBST)], lv_hi = U[sum_index(b, lvw + 1u, KBST)];
    __builtin_amdgcn_sched_group_barrier(0x0020, K + 2, 0);  // (the VMEM reads above, grouped)
    uint32_t J = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) J += fm[k] >= m_min ? 1u : 0u;
    double ub = __longlong_as_double((long long)((uint64_t)U[sum_index(b, 2 * J, KBST)] |
                                                 ((uint64_t)U[sum_index(b, 2 * J + 1, KBST)] << 32)));
    if (lvw != 0u)
      ub = fmin(ub, __longlong_as_double((long long)((uint64_t)lv_lo | ((uint64_t)lv_hi << 32))));
    return ub;
  };
  auto pruned = [&](double ub) -> bool {
    if constexpr (TOPK) {  // (ub >= 0; a score is an integer <= floor(ub); beyond 2^52: none)
      if (!(ub < 4503599627370496.0)) return false;
      return ((((uint64_t)ub) << ib) | (uint64_t)imax) <= thrk;
    } else {
      return ub < thr;
    }
  };
  auto block = [&](uint32_t nb) {
    worked = false;
    const uint32_t n = nb + lane;
    const bool valid0 = n < n1;
    const uint32_t nid = (args.ids && valid0) ? args.ids[n] : n;
    if (args.ids) lds[IDW + lane] = nid;
    const bool valid = n < n1;
    // the block's (nz, full) mask words and its summaries, loaded together (before the branch
    // to a partial node's own mask: one round trip for both, not two)
    BlockMask bk{0ull, 0ull};
    if (bsw) bk = bsw[nb >> 6];
    // this block's tile of summaries (nb is a multiple of 64): word w at s[64 w]
    const uint32_t* s = reinterpret_cast<const uint32_t*>(sum2) + sum_index(nb, 0, S2) + lane;
    const uint4 h0 = make_uint4(s[64 * kS2Static], s[64 * (kS2Static + 1)], s[64 * kS2Clock],
                                s[64 * kS2Meta]);
    // (bandwidth, core, power: only waves that compute their own card terms read them, i.e.
    // not the G waves of a one-model snapshot; minclk: the mixed-model rows)
    uint4 h1 = make_uint4(0u, 0u, 0u, 0u);
    if (MIX || !use_g)
      h1 = make_uint4(s[64 * kS2Bw], s[64 * kS2Core], s[64 * kS2Power], s[64 * kS2MinClk]);
    Group<uint32_t, K> fs, ts;  // ts: TotalMemory in free order, or (use_g) B[1..K]
#pragma unroll
    for (int t = 0; t < K; ++t) fs.v[t] = s[64 * (kS2Fs + t)];
    if (use_g) {  // a G wave needs no TotalMemory: the table has the basic scores
      const uint32_t* gs = args.g.tab + sum_index(nb, 0, gtab_stride(K)) + lane;
#pragma unroll
      for (int t = 0; t < K; ++t) ts.v[t] = gs[64 * t];
    } else {
#pragma unroll
      for (int t = 0; t < K; ++t) ts.v[t] = s[64 * (kS2Fs + K + t)];
    }
    // the wave's mask of node n: from the block's (nz, full) words, and a load of its own
    // only for a partial node (sparse form); or the dense [wave][node] array
    uint64_t mask, feas_b;
    if (bsw) {
      mask = ((bk.full >> lane) & 1ull) ? live_mask : 0ull;
      if (((bk.nz & ~bk.full) >> lane) & 1ull) mask = bmw[n];
      feas_b = bk.nz;
    } else {
      mask = valid ? bmw[n] : 0ull;
      feas_b = ballot(mask != 0ull);
    }
    if (feas_b == 0) return;  // no pod of the wave can use any node of the block
    worked = true;
    if (STATS && !trace && lane == 0) atomicAdd(stats + 14, 1ull);
    uint64_t fast_b = 0, u_b = 0, rec_b = 0;
    // the clock the per-pod passes compare with the pods' scv/clock (algorithm.go:271): the
    // node's one model, or ~0 for a mixed-model node whose clock test is folded into its row
    uint32_t ck = h0.z;
    bool fast = mask != 0ull && (!MIX || (h0.w & kSumUni4) != 0u);
    // TOPK: an upper bound on node n's key for every pod of the wave (uniform maxima, one-model
    // node: every pod qualifies at most the nq_hi cards the smallest scv/memory does); ~0:
    // no bound
    uint64_t ub_key = ~0ull;
    {
      const uint32_t meta = h0.w, bw = h1.x, core = h1.y, pw = h1.z;
      const uint32_t cnt = (meta >> 8) & 0xffu;
      uint32_t nq_lo = 0, nq_hi = 0;  // qualifying cards for the largest / smallest m
#pragma unroll
      for (int t = 0; t < K; ++t) {
        nq_lo += (uint32_t)(fs.v[t] >= m_max);
        nq_hi += (uint32_t)(fs.v[t] >= m_min);
      }
      nq_lo = min(nq_lo, cnt);
      nq_hi = min(nq_hi, cnt);
      // fs[nq_lo + i]: a pod with m <= thr_i qualifies card nq_lo + i too (the free order
      // is descending); 0 past the node's range (only m == 0 meets it, and then every
      // lower threshold as well).  Read back by index from the lane's record slot, where
      // the frees are staged (the slot is overwritten by a record further down).
      const uint32_t range = nq_hi - nq_lo;
      uint32_t* rec = lds + RECS + lane * REC;
      if constexpr (K >= 4) {
#pragma unroll
        for (int t = 0; t < K; t += 4)
          *reinterpret_cast<uint4*>(rec + t) =
              make_uint4(fs.v[t], fs.v[t + 1], fs.v[t + 2], fs.v[t + 3]);
      } else {
#pragma unroll
        for (int t = 0; t < K; ++t) rec[t] = fs.v[t];
      }
      const uint32_t thr = nq_lo < (uint32_t)K ? rec[nq_lo] : 0u;
      const uint32_t thr1 = range > 1u && nq_lo + 1u < (uint32_t)K ? rec[nq_lo + 1u] : 0u;
      const uint32_t thr2 = range > 2u && nq_lo + 2u < (uint32_t)K ? rec[nq_lo + 2u] : 0u;
      // the static part as an integer (< 2^52: its f64 bits above 2^52's)
      const double stat_d =
          __longlong_as_double((long long)((uint64_t)h0.x | ((uint64_t)h0.y << 32)));
      const uint64_t stat_u = (uint64_t)__double_as_longlong(stat_d + 4503599627370496.0) -
                              0x4330000000000000ull;
      // A one-model node whose qualifying-card count takes at most four values over the
      // wave (two with several reciprocal sets) gets a record: its clock, the wave's mask,
      // the thresholds, the static part and the basic scores -- the per-pod pass reads it
      // with three broadcast LDS loads.
      if (uni_max) {
        // CalculateCardScore terms (algorithm.go:280-291) with the wave's reciprocals: from
        // the G table when they are G's (the same integers), else computed
        // B[q] = q shared + prefix[q]: the basic score with q qualifying cards (prefix: the
        // sums of 3 q_free + q_total in free order); sel = B[nq_lo], sel_hi = B[nq_hi]
        uint32_t sel = 0, sel_hi = 0;
        lds[lane * PSW + 0] = 0u;
        if (use_g) {  // (wave-uniform branch)
#pragma unroll
          for (int t = 0; t < K; ++t) {
            const uint32_t b = ts.v[t];
            lds[lane * PSW + t + 1] = b;
            if constexpr (TOPK) sel_hi = (uint32_t)(t + 1) == nq_hi ? b : sel_hi;
          }
          sel = lds[lane * PSW + nq_lo];  // B[nq_lo], read back
        } else {
          const uint32_t shared = card_shared_terms(bw, ck, core, pw, u_bw, u_core, u_pow);
          auto row = [&](auto rk) {
            uint32_t acc = 0;
#pragma unroll
            for (int t = 0; t < K; ++t) {
              acc += mem_term<decltype(rk)::value>(fs.v[t], ts.v[t], u_free, u_tot, args.mt);
              const uint32_t b = (uint32_t)(t + 1) * shared + acc;
              lds[lane * PSW + t + 1] = b;
              if constexpr (TOPK) sel_hi = (uint32_t)(t + 1) == nq_hi ? b : sel_hi;
            }
          };
          row(std::integral_constant<bool, RK>{});
          sel = lds[lane * PSW + nq_lo];  // B[nq_lo], read back
        }
        // Mixed-model nodes (cards of several GPU models): when every card's clock test
        // (clock >= c, algorithm.go:271) comes out the same for every pod of the wave, the
        // basic score with the first q free-ordered cards qualifying on memory is
        // B'[q] = the sum of CalculateCardScore over those of them whose clock passes --
        // a row like the one-model B[q], with the clock test folded in (ck := ~0).  The G
        // row is B' when every card passes (the node's lowest clock >= the wave's
        // largest scv/clock).  Otherwise the node stays on the exact per-pod path.
        const bool mixn = MIX && mask != 0ull && (meta & kSumUni4) == 0u;
        if (ballot(mixn) != 0ull) {
          if (mixn) {
            bool ok = use_g && h1.w >= c_max;
            if (!ok) {
              const uint32_t* mxw = args.mix + sum_index(nb, 0, MS) + lane;
              bool cu = true;
              sel = 0u;
              sel_hi = 0u;
              auto row = [&](auto rk) {
                uint32_t acc = 0;
#pragma unroll
                for (int t = 0; t < K; ++t) {
                  const uint32_t cj = mxw[64 * mix_word(kMixCk, t, K)];
                  const uint32_t to = use_g ? s[64 * (kS2Fs + K + t)] : ts.v[t];
                  cu = cu && ((cj >= c_max) || (cj < c_min));
                  const uint32_t term =
                      card_shared_terms(mxw[64 * mix_word(kMixBw, t, K)], cj,
                                        mxw[64 * mix_word(kMixCo, t, K)],
                                        mxw[64 * mix_word(kMixPw, t, K)], u_bw, u_core, u_pow) +
                      mem_term<decltype(rk)::value>(fs.v[t], to, u_free, u_tot, args.mt);
                  acc += cj >= c_max ? term : 0u;
                  lds[lane * PSW + t + 1] = acc;
                  sel = (uint32_t)(t + 1) == nq_lo ? acc : sel;
                  if constexpr (TOPK) sel_hi = (uint32_t)(t + 1) == nq_hi ? acc : sel_hi;
                }
              };
              row(std::integral_constant<bool, RK>{});
              ok = cu;
            }
            fast = ok;
            ck = ~0u;
          }
        }
        if constexpr (TOPK) {
          // basic = B[nq] grows with nq <= nq_hi (0 when the clock fails)
          const uint64_t ub = stat_u + (ck >= c_min ? sel_hi : 0u);
          if (fast) ub_key = (ub << ib) | (uint64_t)(imax - n);
        }
        const double stat = stat_d;
        const bool q_all = ck >= c_max, q_none = ck < c_min;
        const bool is_u = fast && mask == act_mask && nq_lo == nq_hi && (q_all || q_none);
        u_b = ballot(is_u);
        if constexpr (TOPK) {
          // the wave's U keys above the uniform list's last one enter it, best first
          const uint32_t basic = q_all ? sel : 0u;  // algorithm.go:271
          const uint64_t key =
              is_u ? ((stat_u + basic) << ib) | (uint64_t)(imax - n) : 0ull;
          bool cand = key > ul[TL - 1];
          while (ballot(cand) != 0ull) {
            uint64_t x = wave_max_u64(cand ? key : 0ull);
            cand = cand && key != x;
#pragma unroll
            for (int k = 0; k < TL; ++k) {
              const uint64_t o = ul[k];
              const bool gt = x > o;
              ul[k] = gt ? x : o;
              x = gt ? o : x;
            }
            cand = cand && key > ul[TL - 1];
          }
        } else {
          // (branch-free: selects instead of exec-mask branches around the update)
          const uint32_t basic = q_all ? sel : 0u;  // algorithm.go:271
          const double raw = (double)basic + stat;                   // algorithm.go:96
          const bool gt = is_u && raw > ubest, eq = is_u && raw == ubest;
          uidx = gt ? nid : (eq ? min(uidx, nid) : uidx);
          uties = gt ? 1u : uties + (eq ? 1u : 0u);
          ubest = gt ? raw : ubest;
        }
        const bool is_rec = fast && range <= 3u && !is_u;
        rec_b = ballot(is_rec);
        if (is_rec) {
          // basic at nq_lo + i (i <= range; repeated past it), from the prefix row
          const uint32_t* row = lds + lane * PSW;
          const uint32_t q1 = nq_lo + min(range, 1u), q2 = nq_lo + min(range, 2u);
          const uint32_t q3 = nq_lo + min(range, 3u);
          *reinterpret_cast<uint4*>(rec) = make_uint4(ck, (uint32_t)mask, (uint32_t)(mask >> 32),
                                                      thr);
          *reinterpret_cast<uint4*>(rec + 4) = make_uint4((uint32_t)stat_u,
                                                          (uint32_t)(stat_u >> 32), thr1, thr2);
          *reinterpret_cast<uint4*>(rec + 8) =
              make_uint4(sel, row[q1], row[q2], row[q3]);
        }
      } else {
        // several reciprocal sets: no U nodes (scores differ across the wave), a record per
        // two-valued one-model node with the basic scores of every set (not with memory ranks,
        // RK: the per-set loop's table gathers would spill the kernel; those nodes take the
        // per-pod pass)
        const bool is_rec = !RK && rec_ok && fast && range <= 1u;
        rec_b = ballot(is_rec);
        if (!RK && (rec_b != 0ull || (TT > 1u && ballot(fast && !is_rec) != 0ull))) {
          if (is_rec) {
            *reinterpret_cast<uint4*>(rec) = make_uint4(ck, (uint32_t)mask,
                                                        (uint32_t)(mask >> 32), thr);
            *reinterpret_cast<uint4*>(rec + 4) = make_uint4((uint32_t)stat_u,
                                                            (uint32_t)(stat_u >> 32), 0u, 0u);
          }
          for (uint32_t q = 0; q < nsets; ++q) {
            // the set's reciprocals (broadcast)
            const RS* r = reinterpret_cast<const RS*>(lds + RCPS + 16 * q);
            const double* d = reinterpret_cast<const double*>(lds + RCPS + 16 * q + 8);
            const double v_free = d[0], v_tot = d[1];
            const uint32_t shared = card_shared_terms(bw, ck, core, pw, r[0], r[1], r[2]);
            uint32_t sel = 0, sel_hi = 0;
            // the set's prefix row of this node lane (TT > 1, the first TT sets)
            uint32_t* trow = lds + row_base(q < TT ? q : 0u) + lane * PSW;
            const bool wrow = TT > 1u && q < TT;
            if (wrow) trow[0] = 0u;
            auto row = [&](auto rk) {
              uint32_t acc = 0;
#pragma unroll
              for (int t = 0; t < K; ++t) {
                acc += mem_term<decltype(rk)::value>(fs.v[t], ts.v[t], v_free, v_tot, args.mt);
                sel = (uint32_t)(t + 1) == nq_lo ? acc : sel;
                sel_hi = (uint32_t)(t + 1) == nq_hi ? acc : sel_hi;
                if (wrow) trow[t + 1] = (uint32_t)(t + 1) * shared + acc;
              }
            };
            row(std::integral_constant<bool, RK>{});
            if (is_rec)
              *reinterpret_cast<uint2*>(rec + 8 + 2 * q) =
                  make_uint2(nq_lo * shared + sel, nq_hi * shared + sel_hi);
          }
        }
      }
    }
    fast_b = ballot(fast);
    uint64_t part_b = feas_b & ~u_b;
    if constexpr (TOPK) {
      // a node whose bound is below every active lane's k-th key cannot enter any list: no
      // per-pod pass for it (lists fill within the first blocks of a chunk)
      const uint64_t thr = wave_min_u64(act ? pl[TL - 1] : ~0ull);
      const uint64_t keep_b = ballot(ub_key > thr);
      part_b &= keep_b;
      rec_b &= keep_b;
    }
    if (STATS && !trace && lane == 0) {  // (wave, node) pairs: U, FAST, EXACT (skipped: rest)
      atomicAdd(stats + 2, (unsigned long long)__builtin_popcountll(u_b));
      atomicAdd(stats + 3, (unsigned long long)__builtin_popcountll(part_b & fast_b));
      atomicAdd(stats + 4, (unsigned long long)__builtin_popcountll(part_b & ~fast_b));
      atomicAdd(stats + 7, (unsigned long long)__builtin_popcountll(rec_b));
      if (!uni_max) atomicAdd(stats + 8, (unsigned long long)__builtin_popcountll(part_b));
    }
    if (STATS) npart += (uint32_t)__builtin_popcountll(part_b);
    // node order is not kept across the loops: the tie rule keeps the lowest index.
    // Branch-free (selects, no exec-mask branches): f = this pod lane is feasible on nn.
    uint64_t rb = rec_b;
    part_b &= ~rec_b;
    auto take_r = [&](bool f, uint64_t raw, uint32_t nn) {
      if constexpr (TOPK) {
        const uint64_t key = f ? (raw << ib) | (uint64_t)(imax - nn) : 0ull;
        if (key > pl[TL - 1]) pl_insert(key);
        return;
      }
      const bool gt = f & (raw > rbest), eq = f & (raw == rbest);
      ridx = gt ? nn : (eq ? min(ridx, nn) : ridx);
      rties = gt ? 1u : rties + (eq ? 1u : 0u);
      rbest = gt ? raw : rbest;
    };
    while (rb) {  // R records per trip: all their LDS loads in flight before the first use
#ifndef YODA_K2_R
#define YODA_K2_R 2
#endif
      constexpr int R = YODA_K2_R;
      uint32_t jj[R];
      bool vv[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        vv[k] = rb != 0ull;
        jj[k] = vv[k] ? (uint32_t)__builtin_ctzll(rb) : 0u;
        rb &= rb - 1;
      }
      uint4 ra[R], rs[R], rp[R];
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const uint32_t* r = lds + RECS + jj[k] * REC;
        ra[k] = *reinterpret_cast<const uint4*>(r);
        rs[k] = *reinterpret_cast<const uint4*>(r + 4);
        if (uni_max) {
          rp[k] = *reinterpret_cast<const uint4*>(r + 8);
        } else {
          const uint2 pr = *reinterpret_cast<const uint2*>(r + 8 + 2 * set);
          rp[k] = make_uint4(pr.x, pr.y, pr.y, pr.y);
        }
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        // nq = nq_lo + #{thresholds >= m}; basic = nq * shared + prefix[nq] if the clock
        // qualifies (algorithm.go:271-291)
        const bool c0 = sc.m <= ra[k].w, c1 = sc.m <= rs[k].z, c2 = sc.m <= rs[k].w;
        const uint32_t bsel = c2 ? rp[k].w : (c1 ? rp[k].z : (c0 ? rp[k].y : rp[k].x));
        const uint32_t basic = ra[k].x >= sc.c ? bsel : 0u;
        const uint64_t raw = ((uint64_t)rs[k].x | ((uint64_t)rs[k].y << 32)) + basic;
        const uint32_t mw = lane < 32u ? ra[k].y : ra[k].z;  // the wave's mask of the node
        take_r(vv[k] && ((mw >> (lane & 31u)) & 1u) != 0u, raw,
               args.ids ? lds[IDW + jj[k]] : nb + jj[k]);
      }
    }
    while (part_b) {  // wave-uniform loop over the remaining feasible nodes
      const int j = __builtin_ctzll(part_b);
      part_b &= part_b - 1;
      // the node's local id (its position, unless the run is block-grouped)
      const uint32_t nn =
          args.ids ? (uint32_t)__builtin_amdgcn_readlane((int)nid, j) : nb + (uint32_t)j;
      const uint64_t mj =
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mask >> 32), j) << 32) |
          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mask, j);
      if constexpr (TOPK) {
        // per lane: a node whose bound cannot beat the lane's k-th key is skipped by it;
        // the node is skipped when no feasible lane can take it
        const uint64_t ubj =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ub_key >> 32), j)
             << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ub_key, j);
        if (ballot(((mj >> lane) & 1ull) != 0ull && ubj > pl[TL - 1]) == 0ull) continue;
      }
      double raw;
      if (!MIX || ((fast_b >> j) & 1ull)) {
        // one-model node: nq qualifying cards (a prefix of the free order), then
        // nq * shared + prefix[nq] from LDS -- the node's facts come from its lane
        const uint32_t cnt = ((uint32_t)__builtin_amdgcn_readlane((int)h0.w, j) >> 8) & 0xffu;
        uint32_t nq = 0;
#pragma unroll
        for (int t = 0; t < K; ++t)
          nq += (uint32_t)((uint32_t)__builtin_amdgcn_readlane((int)fs.v[t], j) >= sc.m);
        nq = min(nq, cnt);
        const uint32_t ckj = (uint32_t)__builtin_amdgcn_readlane((int)ck, j);
        const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)h0.x, j) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)h0.y, j) << 32);
        uint32_t basic;
        if (uni_max) {
          const uint32_t* tab = lds + (uint32_t)j * PSW;
          basic = ckj >= sc.c ? tab[nq] : 0u;  // B[nq]
        } else if (TT > 1u &&
                   ballot(((mj >> lane) & 1ull) != 0ull && !(has_set && set < TT)) == 0ull) {
          // several reciprocal sets, every lane in a tabled one: its set's row of the node
          const uint32_t* tab = lds + row_base(set) + (uint32_t)j * PSW;
          basic = ckj >= sc.c ? tab[nq] : 0u;
        } else {
          // several reciprocal sets: Scorer<N32>'s one-model branch on the node lane's data,
          // with its own reciprocals
          const auto& own = sc;
          const uint32_t shared = card_shared_terms(
              (uint32_t)__builtin_amdgcn_readlane((int)h1.x, j), ckj,
              (uint32_t)__builtin_amdgcn_readlane((int)h1.y, j),
              (uint32_t)__builtin_amdgcn_readlane((int)h1.z, j), own.r_bw, own.r_core, own.r_pow);
          uint32_t mem = 0;
          auto terms = [&](auto rk) {
#pragma unroll
            for (int t = 0; t < K; ++t) {
              const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)fs.v[t], j);
              const uint32_t to = (uint32_t)__builtin_amdgcn_readlane((int)ts.v[t], j);
              const uint32_t term =
                  mem_term<decltype(rk)::value>(f, to, own.r_free, own.r_tot, args.mt);
              mem += (uint32_t)t < nq ? term : 0u;  // the qualifying cards are a prefix
            }
          };
          terms(std::integral_constant<bool, RK>{});
          basic = ckj >= sc.c ? nq * shared + mem : 0u;  // algorithm.go:271
        }
        raw = (double)basic + __longlong_as_double((long long)sb);
      } else {
        raw = sc.template raw<K>(nodes + (size_t)nn * NS);  // a mixed-model node
      }
      take_r(((mj >> lane) & 1ull) != 0ull, to_u(raw), nn);
    }
  };
  // thr := max(thr, the min over active lanes of their best so far -- this chunk's nodes', the
  // U nodes', and (gbest) every other chunk's, which this one publishes its own to); each
  // value is a score the lane reaches on a feasible node, so thr stays below every lane's best
  unsigned long long gpub = 0ull;  // the largest value this lane published to gbest
  auto refresh_thr = [&]() {
    const double wu = wave_allreduce(ubest, OpMaxF64{});
    double lb = act ? fmax(rties > 0u ? (double)rbest : -1.0, wu) : HUGE_VAL;
    if (args.gbest != nullptr && act) {  // (score + 1; 0: none yet)
      const unsigned long long g = args.gbest[p];
      const unsigned long long mine = lb >= 0.0 ? (unsigned long long)lb + 1ull : 0ull;
      // (published once per value: the load may see a stale line, not this lane's own atomic)
#ifndef YODA_GBEST_REPUB
      if (mine > g && mine > gpub) {
        atomicMax(args.gbest + p, mine);
        gpub = mine;
      }
#else
      if (mine > g) atomicMax(args.gbest + p, mine);
#endif
      lb = fmax(lb, (double)g - 1.0);
    }
    lb = wave_allreduce(lb, OpMinF64{});
    thr = fmax(thr, __longlong_as_double(
                        (long long)uniform_u64((uint64_t)__double_as_longlong(lb))));
  };
  // TOPK: thrk := the min over active lanes of their k-th key so far (own list or the U list:
  // the merged list's k-th is at least either) -- and (gbest) the largest k-th key any chunk
  // has published for the lane: a chunk whose own list has k keys >= x proves the lane's global
  // k-th key >= x, so a block that cannot beat it holds none of the lane's top k
  auto refresh_thrk = [&]() {
    uint64_t kth = act ? (pl[TL - 1] > ul[TL - 1] ? pl[TL - 1] : ul[TL - 1]) : ~0ull;
    if (args.gbest != nullptr && act) {
      const unsigned long long g = args.gbest[p];
      if (kth > g) atomicMax(args.gbest + p, (unsigned long long)kth);
      kth = kth > g ? kth : g;
    }
    thrk = wave_min_u64(kth);
  };
  const uint64_t t_setup = STATS ? wall_clock64() : 0ull;
  if (blk) {
    // only the blocks K1 found a feasible pod of this wave in (bit b of word b/64)
    const uint64_t* bw = blk + (size_t)uniform_u32(p >> 6) * blk_stride;
    const uint32_t b0 = n0 >> 6, b1 = (n1 + 63) >> 6;
    // pruning: the chunk's high-bound blocks first (pass 0), then the rest (pass 1)
    const int passes = prune && args.hot ? 2 : 1;
    for (int pass = 0; pass < passes; ++pass)
    for (uint32_t wi = b0 >> 6; b0 < b1 && wi <= (b1 - 1) >> 6; ++wi) {
      uint64_t bits = bw[wi];
      const uint32_t base = wi << 6;
      if (b0 > base) bits &= ~0ull << (b0 - base);
      if (b1 < base + 64) bits &= (1ull << (b1 - base)) - 1ull;
      if (passes == 2) bits &= pass == 0 ? args.hot[wi] : ~args.hot[wi];
      // the bounds of the word's 64 blocks, lane = block (one coalesced pass; a block is
      // then skipped on a v_readlane and a compare against the current threshold)
      double ub_l = 0.0;
      if (prune && bits != 0ull) {
        ub_l = block_ub(min(base + lane, b1 - 1u));
        if (args.gbest != nullptr) {  // (the other chunks' progress)
          if constexpr (TOPK) refresh_thrk(); else refresh_thr();
        }
        // every listed block of the word below the threshold: skipped at once
#ifdef YODA_K2_WORDSKIP  // (A/B: off -- K2 0.218 vs 0.205 ms without, profiles/r05/g)
        const double wmax = wave_max_f64(((bits >> lane) & 1ull) ? ub_l : -1.0);
        if (pruned(wmax)) {
#else
        if (false) {
#endif
          if (STATS && !trace && lane == 0)
            atomicAdd(stats + 13, (unsigned long long)__builtin_popcountll(bits));
          bits = 0ull;
        }
      }
      while (bits) {
        const uint32_t j = (uint32_t)__builtin_ctzll(bits);
        bits &= bits - 1;
        if (prune) {
          const uint64_t ubb = (uint64_t)__double_as_longlong(ub_l);
          const double ub = __longlong_as_double(
              (long long)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ubb >> 32), (int)j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ubb, (int)j)));
          if (pruned(ub)) {
            if (STATS && !trace && lane == 0) atomicAdd(stats + 13, 1ull);
            continue;
          }
        }
        block((base + j) << 6);
        if (prune && worked && TOPK) {
          refresh_thrk();
        } else if (prune && worked) {
          refresh_thr();
        }
      }
    }
  } else {
    for (uint32_t nb = n0; nb < n1; nb += kWave) block(nb);
  }
  const uint64_t t_pass = STATS ? wall_clock64() : 0ull;
  if (STATS && !trace && lane == 0) {  // (wave, chunk)s with uniform maxima / all
    atomicAdd(stats + 5, uni_max ? 1ull : 0ull);
    atomicAdd(stats + 6, 1ull);
    atomicMax(stats + 9, (unsigned long long)npart);
  }
  const size_t slot2 = (size_t)(p >> 6) * gridDim.y + chunk;
  if (trace && lane == 0 && slot2 < (size_t)(stats[15] >> 8)) {
    {  // per-(wave, chunk) trace: start, end (100 MHz clock), per-pod nodes
      unsigned long long* tr = stats + 16 + 4 * slot2;
      tr[0] = t_start;
      tr[1] = wall_clock64();
      tr[2] = npart;
      // uniform maxima | G's << 1 | decoupled bounds << 2 | reciprocal sets << 4
      // | set-up end << 16 | block-list walk end << 40 (ticks after the start)
      tr[3] = (uni_max ? 1ull : 0ull) | (use_g ? 2ull : 0ull) | (dec ? 4ull : 0ull) |
              ((unsigned long long)nsets << 4) |
              ((unsigned long long)min((unsigned long long)(t_setup - t_start), 0xffffffull) << 16) |
              ((unsigned long long)min((unsigned long long)(t_pass - t_start), 0xffffffull) << 40);
    }
  }
  if constexpr (TOPK) {
    // the U list (descending, the same for every active lane) into each active lane's list:
    // once no lane takes entry k, none takes a later (smaller) one
#pragma unroll
    for (int k = 0; k < TL; ++k) {
      const uint64_t x = act ? ul[k] : 0ull;
      const bool take = x > pl[TL - 1];
      if (ballot(take) == 0ull) break;
      if (take) pl_insert(x);
    }
    if (!live) return;
    uint64_t* o = tk_keys + ((size_t)chunk * n_pods + p) * TL;
#pragma unroll
    for (int k = 0; k < TL; k += 2)
      *reinterpret_cast<ulonglong2*>(o + k) = make_ulonglong2(pl[k], pl[k + 1]);
    return;
  }
  // merge the U nodes (the same for every pod lane) into each pod lane
  double wb = ubest;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) wb = fmax(wb, __shfl_xor(wb, o, kWave));
  const bool top = ubest == wb && uties > 0;
  uint32_t wi = top ? uidx : 0xffffffffu, wt = top ? uties : 0u;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    wi = min(wi, (uint32_t)__shfl_xor((int)wi, o, kWave));
    wt += (uint32_t)__shfl_xor((int)wt, o, kWave);
  }
  // the per-pod nodes' state (exact: every score < 2^53), then the U nodes
  double best = rties > 0 ? (double)rbest : -1.0;
  uint32_t idx = ridx, ties = rties;
  if (act && wt > 0) {
    if (wb > best) {
      best = wb;
      idx = wi;
      ties = wt;
    } else if (wb == best) {
      idx = min(idx, wi);
      ties += wt;
    }
  }
  if (args.cmask != nullptr) {
    // no pod of the wave has a node here that can be its pick or a tie (none at all, or below
    // a score another chunk already reached: gbest): nothing written, k_reduce2 skips the chunk
    bool useful = live && act && best >= 0.0;
    if (useful && args.gbest != nullptr)
      useful = (unsigned long long)best + 1ull >= args.gbest[p];
    if (ballot(useful) == 0ull) return;
    if (lane == 0) atomicOr(args.cmask + (p >> 6), 1ull << chunk);
  }
  if (!live) return;
  const size_t o = (size_t)chunk * n_pods + p;
  pbest[o] = best;
  pidx[o] = idx;
  pties[o] = ties;
}

// Merge the per-chunk top-k lists of each pod (chunks in node order, so the strict '>'
// insertion keeps lower node indices first among equal scores) -> [TOPK][P], global ids.
template <int TK>
__global__ __launch_bounds__(kBlock) void k_topk_merge(const double* __restrict__ tk_s,
                                                       const uint32_t* __restrict__ tk_i,
                                                       uint32_t C, uint32_t n_pods,
                                                       uint32_t node_offset,
                                                       double* __restrict__ out_s,
                                                       uint32_t* __restrict__ out_i) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  double ts[TK];
  uint32_t ti[TK];
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    ts[k] = -1.0;
    ti[k] = 0xffffffffu;
  }
  for (uint32_t c = 0; c < C; ++c) {
    for (int e = 0; e < TK; ++e) {
      const size_t o = ((size_t)c * TK + e) * n_pods + p;
      double cs = tk_s[o];
      uint32_t ci = tk_i[o];
      // lists are sorted and later chunks hold higher node ids: the rest cannot enter
      if (!(cs > ts[TK - 1])) break;
#pragma unroll
      for (int k = 0; k < TK; ++k) {
        const bool gt = cs > ts[k] || (cs == ts[k] && ci < ti[k]);
        const double os = ts[k];
        const uint32_t oi = ti[k];
        ts[k] = gt ? cs : os;
        ti[k] = gt ? ci : oi;
        cs = gt ? os : cs;
        ci = gt ? oi : ci;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    out_s[(size_t)k * n_pods + p] = ts[k];
    out_i[(size_t)k * n_pods + p] = ti[k] == 0xffffffffu ? ti[k] : ti[k] + node_offset;
  }
}

// Wave-per-pod top-k merge: each lane folds a strided subset of chunk lists into its own
// top-k, then the 64 lists are folded pairwise through shuffles.  The (score desc, node asc)
// comparison is a total order, so the result does not depend on the folding order.
template <int TK>
__device__ __forceinline__ void topk_insert(double (&ts)[TK], uint32_t (&ti)[TK],
                                            double cs, uint32_t ci) {
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    const bool gt = cs > ts[k] || (cs == ts[k] && ci < ti[k]);
    const double os = ts[k];
    const uint32_t oi = ti[k];
    ts[k] = gt ? cs : os;
    ti[k] = gt ? ci : oi;
    cs = gt ? os : cs;
    ci = gt ? oi : ci;
  }
}

template <int TK>
__global__ __launch_bounds__(kWave) void k_topk_merge_wave(const double* __restrict__ tk_s,
                                                            const uint32_t* __restrict__ tk_i,
                                                            uint32_t C, uint32_t n_pods,
                                                            uint32_t node_offset,
                                                            double* __restrict__ out_s,
                                                            uint32_t* __restrict__ out_i) {
  const uint32_t p = blockIdx.x, lane = threadIdx.x;
  double ts[TK];
  uint32_t ti[TK];
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    ts[k] = -1.0;
    ti[k] = 0xffffffffu;
  }
  for (uint32_t c = lane; c < C; c += kWave) {
    for (int e = 0; e < TK; ++e) {
      const size_t o = ((size_t)c * TK + e) * n_pods + p;
      const double cs = tk_s[o];
      const uint32_t ci = tk_i[o];
      if (!(cs > ts[TK - 1] || (cs == ts[TK - 1] && ci < ti[TK - 1]))) break;
      topk_insert(ts, ti, cs, ci);
    }
  }
  for (int o = kWave / 2; o > 0; o >>= 1) {
    double ps[TK];
    uint32_t pi[TK];
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      ps[k] = __shfl_xor(ts[k], o, kWave);
      pi[k] = __shfl_xor(ti[k], o, kWave);
    }
#pragma unroll
    for (int k = 0; k < TK; ++k) topk_insert(ts, ti, ps[k], pi[k]);
  }
  if (lane != 0) return;
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    out_s[(size_t)k * n_pods + p] = ts[k];
    out_i[(size_t)k * n_pods + p] = ti[k] == 0xffffffffu ? ti[k] : ti[k] + node_offset;
  }
}

// Merge of the block K2's packed top-k lists keys[C][P][TK] (descending, 0 = none): one
// workgroup per pod.  Thread t folds chunks t, t + 256, ... into its own sorted list (the
// first list copied, then insertions until a key falls below the list's tail; each list one
// contiguous read); each wave then extracts its top TK by TK rounds of wave max over the lane
// heads (the winning lane shifts its list), and wave 0 the pod's top TK from the four wave
// lists the same way.  Keys are unique (one node each), so the result is the global top TK
// whatever the folding order.  Out: [TK][P] scores (-1: no entry) and global node ids
// (0xFFFFFFFF).  (One workgroup per pod: the capacity windows' 256-1024 pods still fill the
// chip, and no thread walks more than a few of the C <= 1568 chunks.)
template <int TK>
__global__ __launch_bounds__(kBlock) void k_topk_merge_keys(const uint64_t* __restrict__ keys,
                                                            uint32_t C, uint32_t n_pods,
                                                            uint32_t ib, uint32_t node_offset,
                                                            double* __restrict__ out_s,
                                                            uint32_t* __restrict__ out_i) {
  constexpr uint32_t NW = kBlock / kWave;
  static_assert(NW * TK <= kWave, "wave 0 holds every wave's list, one key a lane");
  __shared__ uint64_t lst[NW * TK];
  const uint32_t p = blockIdx.x, lane = lane_id(), wv = threadIdx.x >> 6;
  if (p >= n_pods) return;  // workgroup-uniform
  uint64_t pl[TK];
#pragma unroll
  for (int k = 0; k < TK; ++k) pl[k] = 0ull;
  auto insert = [&](uint64_t x) {
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      const uint64_t o = pl[k];
      const bool gt = x > o;
      pl[k] = gt ? x : o;
      x = gt ? o : x;
    }
  };
  bool empty = true;
  for (uint32_t c = threadIdx.x; c < C; c += kBlock) {
    const ulonglong2* l = reinterpret_cast<const ulonglong2*>(keys + ((size_t)c * n_pods + p) * TK);
    uint64_t v[TK];
#pragma unroll
    for (int k = 0; k < TK / 2; ++k) {
      const ulonglong2 t = l[k];
      v[2 * k] = t.x;
      v[2 * k + 1] = t.y;
    }
    if (empty) {  // the thread's first list: already sorted
#pragma unroll
      for (int k = 0; k < TK; ++k) pl[k] = v[k];
      empty = false;
      continue;
    }
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      if (!(v[k] > pl[TK - 1])) break;  // the list is sorted: nothing further enters
      insert(v[k]);
    }
  }
  // the wave's top TK: round k takes the largest lane head (one lane holds it) and that lane
  // moves on to its next key
  uint64_t mine = 0ull;
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    const uint64_t m = wave_max_u64v(pl[0]);
    mine = lane == (uint32_t)k ? m : mine;
    if (pl[0] == m) {
#pragma unroll
      for (int j = 0; j + 1 < TK; ++j) pl[j] = pl[j + 1];
      pl[TK - 1] = 0ull;
    }
  }
  if (lane < (uint32_t)TK) lst[wv * TK + lane] = mine;
  __syncthreads();
  if (wv != 0) return;
  uint64_t x = lane < NW * TK ? lst[lane] : 0ull;
  mine = 0ull;
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    const uint64_t m = wave_max_u64v(x);
    mine = lane == (uint32_t)k ? m : mine;
    x = x == m ? 0ull : x;
  }
  if (lane >= (uint32_t)TK) return;
  const uint64_t imask = (1ull << ib) - 1ull;
  out_s[(size_t)lane * n_pods + p] = mine ? (double)(mine >> ib) : -1.0;
  out_i[(size_t)lane * n_pods + p] =
      mine ? (uint32_t)(imask - (mine & imask)) + node_offset : 0xffffffffu;
}

// Deeper lists from the same chunk lists (the capacity windows' certificates):
// the merged top KO of every chunk's top TK, kept as far as it is exact.  A node missing from
// its chunk's list (or from the list a thread folds its chunks into) is at most that list's
// TK-th key, so with M = the largest such key over the full lists, every candidate above M is
// in place; the global top TK always is (each of them is within its chunk's and its thread's
// top TK).  Output entries 0..L-1, L = max(TK, #candidates > M) capped at KO; the rest empty
// (-1, 0xffffffff): every node left out is at most entry L-1 in (score desc, node asc).
template <int TK, int KO>
__global__ __launch_bounds__(kWave) void k_topk_merge_deep(const uint64_t* __restrict__ keys,
                                                           uint32_t C, uint32_t n_pods,
                                                           uint32_t ib, uint32_t node_offset,
                                                           double* __restrict__ out_s,
                                                           uint32_t* __restrict__ out_i) {
  // one wave per pod: each lane folds every 64th chunk's list into its own top TK, then KO
  // rounds take the largest lane head (the lane holding it moves on)
  static_assert(KO % kWave == 0 || KO < kWave, "whole output rows per lane");
  constexpr uint32_t PER = KO >= kWave ? KO / kWave : 1;  // output keys a lane holds
  const uint32_t p = blockIdx.x, lane = threadIdx.x;
  if (p >= n_pods) return;  // workgroup-uniform
  uint64_t pl[TK];
#pragma unroll
  for (int k = 0; k < TK; ++k) pl[k] = 0ull;
  uint64_t mbound = 0ull;  // the largest TK-th key of a full chunk list or of this lane's
  for (uint32_t c = lane; c < C; c += kWave) {
    const ulonglong2* l = reinterpret_cast<const ulonglong2*>(keys + ((size_t)c * n_pods + p) * TK);
    uint64_t v[TK];
#pragma unroll
    for (int k = 0; k < TK / 2; ++k) {
      const ulonglong2 t = l[k];
      v[2 * k] = t.x;
      v[2 * k + 1] = t.y;
    }
    mbound = max(mbound, v[TK - 1]);  // (0 unless the chunk's list is full)
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      if (!(v[k] > pl[TK - 1])) break;  // the list is sorted: nothing further enters
      uint64_t x = v[k];
#pragma unroll
      for (int j = 0; j < TK; ++j) {
        const uint64_t o = pl[j];
        const bool gt = x > o;
        pl[j] = gt ? x : o;
        x = gt ? o : x;
      }
    }
  }
  mbound = max(mbound, pl[TK - 1]);  // (what this lane's folding dropped is below it)
  const uint64_t M = wave_max_u64v(mbound);
  uint64_t out[PER];
#pragma unroll
  for (uint32_t r = 0; r < PER; ++r) out[r] = 0ull;
  uint32_t L = 0;
  for (int k = 0; k < KO; ++k) {
    const uint64_t m = wave_max_u64v(pl[0]);
    if (m == 0ull) break;                // (uniform)
    if (k >= TK && !(m > M)) break;      // no longer certain to be in place
#pragma unroll
    for (uint32_t r = 0; r < PER; ++r) out[r] = (uint32_t)k == r * kWave + lane ? m : out[r];
    if (pl[0] == m) {
#pragma unroll
      for (int j = 0; j + 1 < TK; ++j) pl[j] = pl[j + 1];
      pl[TK - 1] = 0ull;
    }
    ++L;
  }
  const uint64_t imask = (1ull << ib) - 1ull;
#pragma unroll
  for (uint32_t r = 0; r < PER; ++r) {
    const uint32_t k = r * kWave + lane;
    if (k >= (uint32_t)KO) continue;
    const uint64_t x = k < L ? out[r] : 0ull;
    out_s[(size_t)k * n_pods + p] = x ? (double)(x >> ib) : -1.0;
    out_i[(size_t)k * n_pods + p] = x ? (uint32_t)(imask - (x & imask)) + node_offset : 0xffffffffu;
  }
}

// Greedy: overwrite the static score (record header offset 0) of a few nodes.
__global__ __launch_bounds__(kBlock) void k_set_static(unsigned char* __restrict__ nodes,
                                                       uint32_t stride,
                                                       const uint32_t* __restrict__ node,
                                                       const uint64_t* __restrict__ value,
                                                       const uint64_t* __restrict__ card_number,
                                                       uint32_t count,
                                                       unsigned char* __restrict__ sum,
                                                       uint32_t sum_stride,
                                                       unsigned char* __restrict__ sum2,
                                                       uint32_t sum2_stride, PermCopy pc) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= count) return;
  if (pc.inv) {  // the block-grouped copies (private runs) at the node's internal position
    const uint32_t q = pc.inv[node[t]];
    uint32_t* s1 = reinterpret_cast<uint32_t*>(pc.sum);
    s1[sum_index(q, kSumCnLo, sum_stride)] = (uint32_t)card_number[t];
    s1[sum_index(q, kSumCnHi, sum_stride)] = (uint32_t)(card_number[t] >> 32);
    uint32_t* s2 = reinterpret_cast<uint32_t*>(pc.sum2);
    s2[sum_index(q, kS2Static, sum2_stride)] = (uint32_t)value[t];
    s2[sum_index(q, kS2Static + 1, sum2_stride)] = (uint32_t)(value[t] >> 32);
  }
  if (pc.bsum || pc.bsum_p) {  // widen the blocks' CardNumber bounds to the new value
    const uint32_t bst = 4u * pc.bsum_words;
    const uint32_t cn = (uint32_t)min(card_number[t], (uint64_t)0xffffffffu);
    if (pc.bsum) {
      const uint32_t b = node[t] >> 6;
      atomicMin(pc.bsum + sum_index(b, kBsCnMin, bst), cn);
      atomicMax(pc.bsum + sum_index(b, kBsCnMax, bst), cn);
    }
    if (pc.bsum_p) {
      const uint32_t b = pc.inv[node[t]] >> 6;
      atomicMin(pc.bsum_p + sum_index(b, kBsCnMin, bst), cn);
      atomicMax(pc.bsum_p + sum_index(b, kBsCnMax, bst), cn);
    }
  }
  uint64_t* hdr = reinterpret_cast<uint64_t*>(nodes + (size_t)node[t] * stride);
  hdr[0] = value[t];        // static_score bits (f64 on the fast paths, u64 on U64)
  hdr[1] = card_number[t];  // CardNumber
  if (sum) {                // the K1 summary's copy of CardNumber (words cn_lo, cn_hi)
    uint32_t* s = reinterpret_cast<uint32_t*>(sum);
    s[sum_index(node[t], kSumCnLo, sum_stride)] = (uint32_t)card_number[t];
    s[sum_index(node[t], kSumCnHi, sum_stride)] = (uint32_t)(card_number[t] >> 32);
  }
  if (sum2) {  // the K2 summary's copy of the static score (words 0-1)
    uint32_t* s = reinterpret_cast<uint32_t*>(sum2);
    s[sum_index(node[t], kS2Static, sum2_stride)] = (uint32_t)value[t];
    s[sum_index(node[t], kS2Static + 1, sum2_stride)] = (uint32_t)(value[t] >> 32);
  }
}

// Greedy fallback: ONE pod of the current window (sorted position `s`) scored exactly against
// the CURRENT node state, lane = node.  In the reference-faithful greedy only the nodes'
// static scores (Allocate) change inside a window: the pod's feasibility bits (bm, written by
// the window's K1) and its PreScore maxima / reciprocals stay valid, and k_set_static keeps
// the records' static scores current.  Result: argmax raw score, lowest node index among
// equal scores (the same pick as a full evaluation); out[0] = node (local),
// out[1..2] = its raw score as f64 (-1: no feasible node).  One launch: every block
// writes its (best, index) partial and the last block to finish merges them (the counter is
// reset for the next call).
// N32 with the K2 summary (sum2): a one-model node is scored from its summary tile (static
// part, clock, free-sorted cards; the basic score B[nq] from the G table when the pod's
// reciprocals are G's, else the k2_block_n32 terms) -- ~50 coalesced bytes instead of the
// ~250-byte record; other nodes read the record.  The same integers either way (K2's U/FAST
// classes rely on it).
template <int K, Path PATH>
__global__ __launch_bounds__(kBlock) void k_greedy_one(
    const unsigned char* __restrict__ nodes, const uint32_t* __restrict__ sum2,
    uint32_t n_nodes, ScoreArgs args, uint32_t n_pods,
    uint32_t s, const MaskSrc ms, double* __restrict__ part_s,
    uint32_t* __restrict__ part_i, uint32_t* __restrict__ done, uint32_t* __restrict__ out) {
  constexpr uint32_t stride = PATH == Path::N32 ? n32_stride(K) : node_stride(K);
  __shared__ double red_s[kBlock / kWave];
  __shared__ uint32_t red_i[kBlock / kWave];
  __shared__ bool last;
  Scorer<PATH> sc;
  sc.load(args, s, n_pods);  // the same pod on every lane
  bool use_g = false;
  if constexpr (PATH == Path::N32)
    use_g = args.g.tab != nullptr && sc.r_bw == args.g.r_bw && sc.r_core == args.g.r_core &&
            sc.r_pow == args.g.r_pow && sc.r_free == args.g.r_free && sc.r_tot == args.g.r_tot;
  const uint32_t bit = s & 63u;
  double best = -1.0;
  uint32_t idx = 0xffffffffu;
  for (uint32_t n = blockIdx.x * kBlock + threadIdx.x; n < n_nodes; n += gridDim.x * kBlock) {
    if ((mask_at(ms, s >> 6, n, n_pods) >> bit) & 1ull) {
      double raw = -1.0;
      bool done_raw = false;
      if constexpr (PATH == Path::N32) {
        if (sum2) {
          constexpr uint32_t S2 = k2sum_stride(K);
          auto w = [&](uint32_t word) { return sum2[sum_index(n, word, S2)]; };
          const uint32_t meta = w(kS2Meta);
          if (meta & kSumUni4) {
            const uint32_t cnt = (meta >> 8) & 0xffu;
            uint32_t nq = 0;
#pragma unroll
            for (int t = 0; t < K; ++t) nq += (uint32_t)(w(kS2Fs + t) >= sc.m);
            nq = min(nq, cnt);
            uint32_t basic = 0;
            if (nq) {
              if (use_g) {
                basic = args.g.tab[sum_index(n, nq - 1u, gtab_stride(K))];  // B[nq]
              } else {
                uint32_t acc = 0;
#pragma unroll
                for (int t = 0; t < K; ++t)
                  acc += (uint32_t)t < nq
                             ? card_mem_term(w(kS2Fs + t), w(kS2Fs + K + t), sc.r_free, sc.r_tot,
                                             args.mt)
                             : 0u;
                basic = nq * card_shared_terms(w(kS2Bw), w(kS2Clock), w(kS2Core), w(kS2Power),
                                               sc.r_bw, sc.r_core, sc.r_pow) +
                        acc;
              }
            }
            basic = w(kS2Clock) >= sc.c ? basic : 0u;  // algorithm.go:271
            const double stat = __longlong_as_double(
                (long long)((uint64_t)w(kS2Static) | ((uint64_t)w(kS2Static + 1) << 32)));
            raw = (double)basic + stat;
            done_raw = true;
          }
        }
      }
      if (!done_raw) raw = sc.template raw<K>(nodes + (size_t)n * stride);
      if (raw > best) {  // n grows along the thread's sweep: the first maximum is the lowest
        best = raw;
        idx = n;
      }
    }
  }
  auto merge = [](double& b, uint32_t& i, double ob, uint32_t oi) {
    if (ob > b || (ob == b && oi < i)) {
      b = ob;
      i = oi;
    }
  };
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1)
    merge(best, idx, __shfl_xor(best, o, kWave), (uint32_t)__shfl_xor((int)idx, o, kWave));
  const uint32_t w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    red_s[w] = best;
    red_i[w] = idx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < kBlock / kWave; ++k) merge(best, idx, red_s[k], red_i[k]);
    part_s[blockIdx.x] = best;
    part_i[blockIdx.x] = idx;
    __threadfence();
    last = atomicAdd(done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  best = -1.0;
  idx = 0xffffffffu;
  for (uint32_t b = threadIdx.x; b < gridDim.x; b += kBlock)
    merge(best, idx, static_cast<volatile double*>(part_s)[b], static_cast<volatile uint32_t*>(part_i)[b]);
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1)
    merge(best, idx, __shfl_xor(best, o, kWave), (uint32_t)__shfl_xor((int)idx, o, kWave));
  if (lane_id() == 0) {
    red_s[w] = best;
    red_i[w] = idx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < kBlock / kWave; ++k) merge(best, idx, red_s[k], red_i[k]);
    // the score first, then the node: a host polling out[0] (mapped memory) reads a complete
    // result once the node word changes
    *reinterpret_cast<double*>(out + 1) = best;  // 8-byte aligned: out = done + 1 (sharded merge)
    __threadfence_system();
    __hip_atomic_store(out, idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *done = 0u;
  }
}

// ---------------------------------------------------------------------------------------
// One pod against the CURRENT node state, lane = node (the capacity greedy's exact fallback:
// CardNumber may have dropped since the window's K1, so its bitmask and maxima are stale).
// k_one_filter: Filter + CollectMaxValues for the pod over every node (feasibility bits
// feas[n / 64], maxima, counts) and, in the last block to finish, the reciprocals of the
// maxima.  k_one_score: Score of the feasible nodes with them, argmax / ties / lowest.  Both
// reduce in the last block (a counter reset for the next call), so a pod costs two
// launches and one small copy.
template <int K, Path PATH>
__global__ __launch_bounds__(kBlock) void k_one_filter(const unsigned char* __restrict__ nodes,
                                                       uint32_t n_nodes, OnePod pod,
                                                       uint64_t* __restrict__ feas,
                                                       uint64_t* __restrict__ part,
                                                       uint32_t* __restrict__ done,
                                                       OneOut* __restrict__ out, MemTab mt) {
  using R = Rec<PATH>;
  using T = typename R::T;
  __shared__ uint64_t red[kBlock / kWave][9];
  __shared__ bool last;
  T m, c;
  if constexpr (PATH == Path::N32) {
    m = pod.m32;
    c = pod.c32;
  } else {
    m = pod.mf;
    c = pod.cf;
  }
  uint64_t mx[6] = {1, 1, 1, 1, 1, 1};  // floor 1 (collection.go:31-38)
  uint32_t nf = 0, nz = 0, first = 0xffffffffu;
  const uint32_t stride_n = gridDim.x * kBlock;
  // every wave covers 64 consecutive nodes per step, so its ballot is one feasibility word
  for (uint32_t nb = blockIdx.x * kBlock; nb < n_nodes; nb += stride_n) {
    const uint32_t n = nb + threadIdx.x;
    bool f = false;
    if (n < n_nodes) {
      const unsigned char* rec = nodes + (size_t)n * R::stride(K);
      const NodeHdrG hd = *reinterpret_cast<const NodeHdrG*>(rec);
      const Group<T, K> fr = load_group<T, K>(rec + R::off(kFree, K));
      const Group<T, K> ck = load_group<T, K>(rec + R::off(kClock, K));
      uint32_t cm = 0, cc = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t hj = (hd.healthy_mask >> j) & 1u;
        cm += (uint32_t)(fr.v[j] >= m) & hj;  // CardFitsMemory (filter.go:52-54)
        cc += (uint32_t)(ck.v[j] == c) & hj;  // CardFitsClock (filter.go:56-58)
      }
      f = (pod.number <= hd.card_number) & (cm >= pod.need_mem) & (cc >= pod.need_clk);
      if (f) {
        ++nf;
        nz += hd.zero_total;
        first = min(first, n);
        const Group<T, K> bw = load_group<T, K>(rec + R::off(kBandwidth, K));
        const Group<T, K> co = load_group<T, K>(rec + R::off(kCore, K));
        const Group<T, K> pw = load_group<T, K>(rec + R::off(kPower, K));
        const Group<T, K> to = load_group<T, K>(rec + R::off(kTotal, K));
#pragma unroll
        for (int j = 0; j < K; ++j) {
          if ((fr.v[j] >= m) & (ck.v[j] >= c)) {  // collection.go:46
            mx[kMaxBw] = umax64(mx[kMaxBw], (uint64_t)bw.v[j]);
            mx[kMaxClock] = umax64(mx[kMaxClock], (uint64_t)ck.v[j]);
            mx[kMaxCore] = umax64(mx[kMaxCore], (uint64_t)co.v[j]);
            mx[kMaxFree] = umax64(mx[kMaxFree], (uint64_t)fr.v[j]);
            mx[kMaxPower] = umax64(mx[kMaxPower], (uint64_t)pw.v[j]);
            mx[kMaxTotal] = umax64(mx[kMaxTotal], (uint64_t)to.v[j]);
          }
        }
      }
    }
    const uint64_t b = ballot(f);
    if (lane_id() == 0 && nb + (threadIdx.x & ~63u) < n_nodes) feas[(nb + threadIdx.x) >> 6] = b;
  }
  // block reduce: waves through shuffles, then LDS
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
#pragma unroll
    for (int f = 0; f < 6; ++f) mx[f] = umax64(mx[f], __shfl_xor(mx[f], o, kWave));
    nf += __shfl_xor(nf, o, kWave);
    nz += __shfl_xor(nz, o, kWave);
    first = min(first, (uint32_t)__shfl_xor((int)first, o, kWave));
  }
  const uint32_t w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    for (int f = 0; f < 6; ++f) red[w][f] = mx[f];
    red[w][6] = nf;
    red[w][7] = nz;
    red[w][8] = first;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < kBlock / kWave; ++k) {
      for (int f = 0; f < 6; ++f) red[0][f] = umax64(red[0][f], red[k][f]);
      red[0][6] += red[k][6];
      red[0][7] += red[k][7];
      red[0][8] = red[0][8] < red[k][8] ? red[0][8] : red[k][8];
    }
    for (int f = 0; f < 9; ++f) part[(size_t)blockIdx.x * 9 + f] = red[0][f];
    __threadfence();
    last = atomicAdd(done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the last block merges every block's partial: threads stride over them, then as above
  for (int f = 0; f < 6; ++f) mx[f] = 1;
  nf = nz = 0;
  first = 0xffffffffu;
  const volatile uint64_t* vp = part;
  for (uint32_t b = threadIdx.x; b < gridDim.x; b += kBlock) {
    for (int f = 0; f < 6; ++f) mx[f] = umax64(mx[f], vp[(size_t)b * 9 + f]);
    nf += (uint32_t)vp[(size_t)b * 9 + 6];
    nz += (uint32_t)vp[(size_t)b * 9 + 7];
    first = min(first, (uint32_t)vp[(size_t)b * 9 + 8]);
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
#pragma unroll
    for (int f = 0; f < 6; ++f) mx[f] = umax64(mx[f], __shfl_xor(mx[f], o, kWave));
    nf += __shfl_xor(nf, o, kWave);
    nz += __shfl_xor(nz, o, kWave);
    first = min(first, (uint32_t)__shfl_xor((int)first, o, kWave));
  }
  __syncthreads();
  if (lane_id() == 0) {
    for (int f = 0; f < 6; ++f) red[w][f] = mx[f];
    red[w][6] = nf;
    red[w][7] = nz;
    red[w][8] = first;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint64_t acc[9];
  for (int f = 0; f < 9; ++f) acc[f] = red[0][f];
  for (uint32_t k = 1; k < kBlock / kWave; ++k) {
    for (int f = 0; f < 6; ++f) acc[f] = umax64(acc[f], red[k][f]);
    acc[6] += red[k][6];
    acc[7] += red[k][7];
    acc[8] = acc[8] < red[k][8] ? acc[8] : red[k][8];
  }
  if (mt.vf) {  // memory ranks -> values
    acc[kMaxFree] = rank_value(acc[kMaxFree], mt.vf);
    acc[kMaxTotal] = rank_value(acc[kMaxTotal], mt.vt);
  }
  for (int f = 0; f < 6; ++f) out->maxima[f] = acc[f];
  out->nf = (uint32_t)acc[6];
  out->nz = (uint32_t)acc[7];
  out->first = (uint32_t)acc[8];
  const int src[5] = {kMaxBw, kMaxCore, kMaxPower, kMaxFree, kMaxTotal};
  for (int k = 0; k < 5; ++k) {
    const double M = (double)acc[src[k]];
    out->rcp[k] = ru_100_over(M);
  }
  *done = 0u;
}

template <int K, Path PATH>
__global__ __launch_bounds__(kBlock) void k_one_score(const unsigned char* __restrict__ nodes,
                                                      uint32_t n_nodes, OnePod pod,
                                                      const uint64_t* __restrict__ feas,
                                                      double* __restrict__ part,
                                                      uint32_t* __restrict__ done,
                                                      OneOut* __restrict__ out) {
  __shared__ double red_d[kBlock / kWave][2];
  __shared__ uint32_t red_u[kBlock / kWave][2];
  __shared__ bool last;
  Scorer<PATH> sc;
  if constexpr (PATH == Path::N32) {
    sc.m = pod.m32;
    sc.c = pod.c32;
  } else {
    sc.m = pod.mf;
    sc.c = pod.cf;
  }
  sc.r_bw = out->rcp[0];
  sc.r_core = out->rcp[1];
  sc.r_pow = out->rcp[2];
  sc.r_free = out->rcp[3];
  sc.r_tot = out->rcp[4];
  constexpr uint32_t stride = PATH == Path::N32 ? n32_stride(K) : node_stride(K);
  double best = -1.0, low = 1.0e300;
  uint32_t idx = 0xffffffffu, ties = 0;
  for (uint32_t n = blockIdx.x * kBlock + threadIdx.x; n < n_nodes; n += gridDim.x * kBlock) {
    if ((feas[n >> 6] >> (n & 63u)) & 1ull) {
      const double raw = sc.template raw<K>(nodes + (size_t)n * stride);
      if (raw > best) {  // n grows along the thread's sweep: the first maximum is the lowest
        best = raw;
        idx = n;
        ties = 1;
      } else if (raw == best) {
        ++ties;
      }
      low = fmin(low, raw);
    }
  }
  auto merge = [](double& b, uint32_t& i, uint32_t& t, double ob, uint32_t oi, uint32_t ot) {
    if (ob > b) {
      b = ob;
      i = oi;
      t = ot;
    } else if (ob == b && ot) {
      i = min(i, oi);
      t += ot;
    }
  };
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    merge(best, idx, ties, __shfl_xor(best, o, kWave), (uint32_t)__shfl_xor((int)idx, o, kWave),
          (uint32_t)__shfl_xor((int)ties, o, kWave));
    low = fmin(low, __shfl_xor(low, o, kWave));
  }
  const uint32_t w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    red_d[w][0] = best;
    red_d[w][1] = low;
    red_u[w][0] = idx;
    red_u[w][1] = ties;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t k = 1; k < kBlock / kWave; ++k) {
      merge(best, idx, ties, red_d[k][0], red_u[k][0], red_u[k][1]);
      low = fmin(low, red_d[k][1]);
    }
    part[(size_t)blockIdx.x * 4 + 0] = best;
    part[(size_t)blockIdx.x * 4 + 1] = low;
    part[(size_t)blockIdx.x * 4 + 2] = (double)idx;
    part[(size_t)blockIdx.x * 4 + 3] = (double)ties;
    __threadfence();
    last = atomicAdd(done, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  best = -1.0;
  low = 1.0e300;
  idx = 0xffffffffu;
  ties = 0;
  const volatile double* vp = part;
  for (uint32_t b = threadIdx.x; b < gridDim.x; b += kBlock) {  // blocks in node order
    merge(best, idx, ties, vp[(size_t)b * 4], (uint32_t)vp[(size_t)b * 4 + 2],
          (uint32_t)vp[(size_t)b * 4 + 3]);
    low = fmin(low, vp[(size_t)b * 4 + 1]);
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    merge(best, idx, ties, __shfl_xor(best, o, kWave), (uint32_t)__shfl_xor((int)idx, o, kWave),
          (uint32_t)__shfl_xor((int)ties, o, kWave));
    low = fmin(low, __shfl_xor(low, o, kWave));
  }
  __syncthreads();
  if (lane_id() == 0) {
    red_d[w][0] = best;
    red_d[w][1] = low;
    red_u[w][0] = idx;
    red_u[w][1] = ties;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (uint32_t k = 1; k < kBlock / kWave; ++k) {
    merge(best, idx, ties, red_d[k][0], red_u[k][0], red_u[k][1]);
    low = fmin(low, red_d[k][1]);
  }
  out->best = best;
  out->low = low;
  out->idx = idx;
  out->ties = ties;
  *done = 0u;
}

// ---------------------------------------------------------------------------------------
// Generic (exact uint64, Go wrap-around) card score — algorithm.go:280-291.
__device__ __forceinline__ uint64_t card_score_u64(uint64_t bw, uint64_t ck, uint64_t core,
                                                   uint64_t pw, uint64_t fr, uint64_t tot,
                                                   const uint64_t M[6]) {
  const uint64_t a = bw * 100u / M[kMaxBw];
  const uint64_t b = ck * 100u / M[kMaxBw];  // quirk: MaxBandwidth (:283)
  const uint64_t d = core * 100u / M[kMaxCore];
  const uint64_t e = pw * 100u / M[kMaxPower];
  const uint64_t f = fr * 100u / M[kMaxFree];
  const uint64_t g = tot * 100u / M[kMaxTotal];
  return (a + b + d * 2u + e) + f * 3u + g;
}

// raw Score of one feasible (pod, node) on the generic path, after Uint64ToInt64.
template <int K>
__device__ __forceinline__ int64_t raw_score_u64(const unsigned char* rec, uint64_t m, uint64_t c,
                                                 const uint64_t M[6]) {
  const NodeHdrG* h = reinterpret_cast<const NodeHdrG*>(rec);
  const uint64_t* fld = reinterpret_cast<const uint64_t*>(rec + sizeof(NodeHdrG));
  uint64_t basic = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t fr = fld[kFree * K + j], ck = fld[kClock * K + j];
    if (fr >= m && ck >= c)
      basic += card_score_u64(fld[kBandwidth * K + j], ck, fld[kCore * K + j],
                              fld[kPower * K + j], fr, fld[kTotal * K + j], M);
  }
  const uint64_t raw = basic + h->static_score;
  return raw > (uint64_t)kI64Max ? 0 : (int64_t)raw;  // filter.Uint64ToInt64 (filter.go:84-86)
}

template <int K, bool ROWS>
__global__ __launch_bounds__(kBlock) void k2_score_generic(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const uint64_t* __restrict__ m_u, const uint64_t* __restrict__ c_u,
    const uint64_t* __restrict__ maxima, uint32_t n_pods, const uint64_t* __restrict__ bm,
    uint32_t bm_stride, int64_t* __restrict__ pbest, uint32_t* __restrict__ pidx,
    uint32_t* __restrict__ pties, int64_t* __restrict__ plow, int64_t* __restrict__ rows) {
  const Tile tl = tile();
  const uint32_t p = tl.pb * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  uint64_t m = 0, c = 0, M[6] = {1, 1, 1, 1, 1, 1};
  if (live) {
    m = m_u[p];
    c = c_u[p];
#pragma unroll
    for (int f = 0; f < 6; ++f) M[f] = maxima[(size_t)f * n_pods + p];
  }
  int64_t best = -1, low = kI64Max;
  uint32_t idx = 0xffffffffu, ties = 0;
  if (ballot(live) == 0) return;
  const uint64_t* bmw = bm + (size_t)uniform_u32(p >> 6) * bm_stride;
  const uint32_t lane = lane_id();
  for (uint32_t n = n0; n < n1; ++n) {
    const uint64_t mask = bmw[n];
    if (mask == 0) continue;
    if ((mask >> lane) & 1ull) {
      const int64_t s = raw_score_u64<K>(nodes + (size_t)n * node_stride(K), m, c, M);
      if constexpr (ROWS) rows[(size_t)n * n_pods + p] = s;
      if (s > best) {
        best = s;
        idx = n;
        ties = 1;
      } else if (s == best) {
        ++ties;
      }
      low = s < low ? s : low;
    }
  }
  if (!live) return;
  const size_t o = (size_t)chunk * n_pods + p;
  pbest[o] = best;
  pidx[o] = idx;
  pties[o] = ties;
  plow[o] = low;
}

// ---------------------------------------------------------------------------------------
// K2B: BalancedCpuDiskIOPriority (algorithm.go:99-119), every node feasible
// (Yoda.Filter is a pass-through, scheduler.go:96-99).  No FMA contraction (Go on amd64).
template <bool ROWS>
__global__ __launch_bounds__(kBlock) void k2_diskio(const NodeRecB* __restrict__ nodes,
                                                    uint32_t n_nodes, uint32_t chunk_nodes,
                                                    const double* __restrict__ alpha_in,
                                                    const double* __restrict__ beta_in,
                                                    uint32_t n_pods, double* __restrict__ pbest,
                                                    uint32_t* __restrict__ pidx,
                                                    uint32_t* __restrict__ pties,
                                                    double* __restrict__ plow,
                                                    int64_t* __restrict__ rows) {
#pragma clang fp contract(off)
  const Tile tl = tile();
  const uint32_t p = tl.pb * kBlock + threadIdx.x;
  const uint32_t chunk = tl.chunk;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  const double alpha = live ? alpha_in[p] : 0.0, beta = live ? beta_in[p] : 0.0;
  double best = -1.0, low = 1.0e300;
  uint32_t idx = 0xffffffffu, ties = 0;
  for (uint32_t n = n0; n < n1; ++n) {
    const NodeRecB r = nodes[n];
    const double a = alpha * r.v;
    const double b = beta * r.u;
    const double l = fabs(a - b);             // :110
    const double t = 10.0 * l;
    const double s = 10.0 - t;                // :111
    // uint64(Si) on amd64 then Uint64ToInt64: trunc for Si >= 1, else 0 (NaN, negatives)
    const double score = (s >= 1.0) ? __builtin_trunc(s) : 0.0;
    if constexpr (ROWS) {
      if (live) rows[(size_t)n * n_pods + p] = (int64_t)score;
    }
    if (score > best) {
      best = score;
      idx = n;
      ties = 1;
    } else if (score == best) {
      ++ties;
    }
    low = fmin(low, score);
  }
  if (!live) return;
  const size_t o = (size_t)chunk * n_pods + p;
  pbest[o] = best;
  pidx[o] = idx;
  pties[o] = ties;
  plow[o] = low;
}

// K2B score rows (yoda_score_rows in Mode B, the plugin's per-cycle row): lane = node, one
// 256-node chunk per workgroup, the pods of the (small) batch in turn -- every lane busy and
// the row stores coalesced at P = 1, where the lane = pod kernel above runs one lane of 64.
// Per pod the chunk's (best, lowest node, ties, lowest score) as k2_diskio's partials.
__global__ __launch_bounds__(kBlock) void k2b_rows(const NodeRecB* __restrict__ nodes,
                                                   uint32_t n_nodes,
                                                   const double* __restrict__ alpha_in,
                                                   const double* __restrict__ beta_in,
                                                   uint32_t n_pods, double* __restrict__ pbest,
                                                   uint32_t* __restrict__ pidx,
                                                   uint32_t* __restrict__ pties,
                                                   double* __restrict__ plow,
                                                   int64_t* __restrict__ rows) {
#pragma clang fp contract(off)
  __shared__ double s_best[kBlock / kWave], s_low[kBlock / kWave];
  __shared__ uint32_t s_idx[kBlock / kWave], s_ties[kBlock / kWave];
  const uint32_t c = blockIdx.x, n = c * kBlock + threadIdx.x, w = threadIdx.x >> 6;
  const bool v = n < n_nodes;
  const NodeRecB r = v ? nodes[n] : NodeRecB{0.0, 0.0};
  for (uint32_t p = 0; p < n_pods; ++p) {
    const double alpha = alpha_in[p], beta = beta_in[p];
    const double a = alpha * r.v;
    const double b = beta * r.u;
    const double l = fabs(a - b);  // algorithm.go:110
    const double t = 10.0 * l;
    const double sc = 10.0 - t;    // :111
    // uint64(Si) on amd64 then Uint64ToInt64: trunc for Si >= 1, else 0 (NaN, negatives)
    const double score = (sc >= 1.0) ? __builtin_trunc(sc) : 0.0;
    if (v) rows[(size_t)n * n_pods + p] = (int64_t)score;
    double best = v ? score : -1.0, low = v ? score : 1.0e300;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      best = fmax(best, __shfl_xor(best, o, kWave));
      low = fmin(low, __shfl_xor(low, o, kWave));
    }
    const bool at = v && score == best;
    const uint64_t bb = ballot(at);
    if ((threadIdx.x & (kWave - 1)) == 0) {
      s_best[w] = best;
      s_low[w] = low;
      s_idx[w] = bb ? (c * kBlock + w * kWave + (uint32_t)__builtin_ctzll(bb)) : 0xffffffffu;
      s_ties[w] = (uint32_t)__builtin_popcountll(bb);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double B = -1.0, L = 1.0e300;
      uint32_t I = 0xffffffffu, T = 0;
      for (int k = 0; k < kBlock / kWave; ++k) {  // waves in node order: strict '>' keeps lowest
        if (s_best[k] > B) {
          B = s_best[k];
          I = s_idx[k];
          T = s_ties[k];
        } else if (s_best[k] == B && s_ties[k]) {
          T += s_ties[k];
        }
        L = fmin(L, s_low[k]);
      }
      const size_t o = (size_t)c * n_pods + p;
      pbest[o] = B;
      pidx[o] = I;
      pties[o] = T;
      plow[o] = L;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// K2B batch path (Mode B): the same score over pod CLASSES -- the distinct
// (alpha, beta) bit pairs of the batch (algorithm.go:105-106).  Pods of one class score every
// node alike, so their outcome is the class's.  Per pair: a = alpha*V, b = beta*U, d = a - b
// (:109), and the level of |d| against DiskLevels (score >= k <=> |d| <= t[k]): three f64
// operations, two compares.  A lane keeps, over nodes in increasing order, the best level
// seen, its node count and its first (lowest) node; level 0 counts nothing while running
// (every node is >= 0, NaN included) and is settled at the end.
struct DiskAcc {
  uint32_t lev, cnt, idx;
  double tc, tu;  // count threshold of the current level (-1 at level 0), the next level's
};

__device__ __forceinline__ void disk_init(DiskAcc& s, const double* lv) {
  s.lev = 0;
  s.cnt = 0;
  s.idx = 0xffffffffu;
  s.tc = -1.0;
  s.tu = lv[1];
}

__device__ __forceinline__ void disk_step(DiskAcc& s, double ad, uint32_t n, const double* lv) {
  s.cnt += (ad <= s.tc) ? 1u : 0u;
  if (ad <= s.tu) {  // a higher level (rare once the first nodes are seen)
    uint32_t L = 1;  // the levels are nested: |d| <= t[k] for every k up to its level
#pragma unroll
    for (int k = 2; k <= 10; ++k) L += (ad <= lv[k]) ? 1u : 0u;
    s.lev = L;
    s.cnt = 1;
    s.idx = n;
    s.tc = lv[L];
    s.tu = lv[L + 1];
  }
}

// Lane = class: each lane runs CPL classes over the chunk's nodes, one node record per
// iteration read by a scalar (wave-uniform) load.
template <int CPL>
__global__ __launch_bounds__(kBlock) void k2b_class_lanes(const NodeRecB* __restrict__ nodes,
                                                          uint32_t n_nodes, uint32_t chunk_nodes,
                                                          const double* __restrict__ cab,
                                                          uint32_t n_cls, DiskLevels lvs,
                                                          uint32_t* __restrict__ plc,
                                                          uint32_t* __restrict__ pidx) {
#pragma clang fp contract(off)
  __shared__ double lv[12];
  if (threadIdx.x < 12) lv[threadIdx.x] = lvs.t[threadIdx.x];
  __syncthreads();
  const uint32_t chunk = blockIdx.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const uint32_t c0 = blockIdx.x * (kBlock * CPL) + threadIdx.x;
  double al[CPL], be[CPL];
  DiskAcc s[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const uint32_t c = c0 + j * kBlock;
    al[j] = c < n_cls ? cab[c] : 0.0;
    be[j] = c < n_cls ? cab[(size_t)n_cls + c] : 0.0;
    disk_init(s[j], lv);
  }
  // 8 node records per trip: the scalar loads are issued together, one wait per trip
  constexpr int kTrip = 8;
  uint32_t n = n0;
  for (; n + kTrip <= n1; n += kTrip) {
    NodeRecB r[kTrip];
#pragma unroll
    for (int i = 0; i < kTrip; ++i) r[i] = nodes[n + i];
#pragma unroll
    for (int i = 0; i < kTrip; ++i) {
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const double a = al[j] * r[i].v;
        const double b = be[j] * r[i].u;
        disk_step(s[j], fabs(a - b), n + i, lv);
      }
    }
  }
  for (; n < n1; ++n) {
    const NodeRecB r = nodes[n];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const double a = al[j] * r.v;
      const double b = be[j] * r.u;
      disk_step(s[j], fabs(a - b), n, lv);
    }
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const uint32_t c = c0 + j * kBlock;
    if (c >= n_cls) continue;
    uint32_t cnt = s[j].cnt, idx = s[j].idx;
    if (s[j].lev == 0u) {
      cnt = n1 - n0;
      idx = n0;
    }
    plc[(size_t)chunk * n_cls + c] = (s[j].lev << kDiskCountBits) | cnt;
    pidx[(size_t)chunk * n_cls + c] = idx;
  }
}

// Lane = node, one class per workgroup (batches of few classes, e.g. one pod spec): each
// thread strides over the chunk's nodes, then the workgroup merges (max level; at it, count
// sum and lowest node).
__global__ __launch_bounds__(kBlock) void k2b_node_lanes(const NodeRecB* __restrict__ nodes,
                                                         uint32_t n_nodes, uint32_t chunk_nodes,
                                                         const double* __restrict__ cab,
                                                         uint32_t n_cls, DiskLevels lvs,
                                                         uint32_t* __restrict__ plc,
                                                         uint32_t* __restrict__ pidx) {
#pragma clang fp contract(off)
  __shared__ double lv[12];
  __shared__ uint32_t red[3][kBlock / kWave];
  if (threadIdx.x < 12) lv[threadIdx.x] = lvs.t[threadIdx.x];
  __syncthreads();
  const uint32_t chunk = blockIdx.x, c = blockIdx.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const double al = cab[c], be = cab[(size_t)n_cls + c];
  DiskAcc s;
  disk_init(s, lv);
  uint32_t seen = 0;
  for (uint32_t n = n0 + threadIdx.x; n < n1; n += kBlock, ++seen) {
    const NodeRecB r = nodes[n];
    const double a = al * r.v;
    const double b = be * r.u;
    disk_step(s, fabs(a - b), n, lv);
  }
  if (s.lev == 0u) {
    s.cnt = seen;
    s.idx = seen ? n0 + threadIdx.x : 0xffffffffu;
  }
  const uint32_t L = wave_max_u32(s.lev);
  uint32_t cnt = s.lev == L ? s.cnt : 0u;
  uint32_t idx = s.lev == L ? s.idx : 0xffffffffu;
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    cnt += (uint32_t)__shfl_xor((int)cnt, o, kWave);
    idx = min(idx, (uint32_t)__shfl_xor((int)idx, o, kWave));
  }
  const uint32_t w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    red[0][w] = L;
    red[1][w] = cnt;
    red[2][w] = idx;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t bl = 0, bc = 0, bi = 0xffffffffu;
  for (int i = 0; i < kBlock / kWave; ++i) {
    if (red[1][i] == 0u) continue;  // a wave with no node of this chunk
    if (red[0][i] > bl) {
      bl = red[0][i];
      bc = red[1][i];
      bi = red[2][i];
    } else if (red[0][i] == bl) {
      bc += red[1][i];
      bi = min(bi, red[2][i]);
    }
  }
  plc[(size_t)chunk * n_cls + c] = (bl << kDiskCountBits) | bc;
  pidx[(size_t)chunk * n_cls + c] = bi;
}

// Per pod: its class's chunk partials (chunks in node order: the first chunk reaching the best
// level holds the lowest node) -> best level, lowest node (+ node_offset), count.  Mode B
// scores lie in [0, 10], so NormalizeScore cannot overflow and the lowest score is not needed
// (written as 0).
__global__ __launch_bounds__(kBlock) void k_reduce2b(const uint32_t* __restrict__ plc,
                                                     const uint32_t* __restrict__ pidx,
                                                     uint32_t C, uint32_t n_cls,
                                                     const uint32_t* __restrict__ cls,
                                                     uint32_t n_pods, uint32_t node_offset,
                                                     int64_t* __restrict__ best_out,
                                                     uint32_t* __restrict__ idx_out,
                                                     uint32_t* __restrict__ ties_out,
                                                     int64_t* __restrict__ low_out) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const uint32_t c = cls[p];
  int64_t bl = -1;
  uint32_t bc = 0, bi = 0xffffffffu;
  for (uint32_t k = 0; k < C; ++k) {
    const uint32_t w = plc[(size_t)k * n_cls + c];
    const int64_t L = (int64_t)(w >> kDiskCountBits);
    if (L > bl) {
      bl = L;
      bc = w & ((1u << kDiskCountBits) - 1u);
      bi = pidx[(size_t)k * n_cls + c];
    } else if (L == bl) {
      bc += w & ((1u << kDiskCountBits) - 1u);
    }
  }
  best_out[p] = bl;
  idx_out[p] = bi == 0xffffffffu ? bi : bi + node_offset;
  ties_out[p] = bc;
  low_out[p] = 0;
}

// Per-pod merge of K2 chunk partials.  Chunks are in node order, so on equal scores the
// earlier chunk's index (lower) is kept.
__global__ __launch_bounds__(kBlock) void k_reduce2(const double* __restrict__ pbest_f,
                                                    const int64_t* __restrict__ pbest_i,
                                                    const uint32_t* __restrict__ pidx,
                                                    const uint32_t* __restrict__ pties,
                                                    const double* __restrict__ plow_f,
                                                    const int64_t* __restrict__ plow_i,
                                                    uint32_t C, uint32_t n_pods, int is_f64,
                                                    uint32_t node_offset,
                                                    int64_t* __restrict__ best_out,
                                                    uint32_t* __restrict__ idx_out,
                                                    uint32_t* __restrict__ ties_out,
                                                    int64_t* __restrict__ low_out,
                                                    const unsigned long long* __restrict__ cmask = nullptr) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  int64_t best = -1, low = kI64Max;
  uint32_t idx = 0xffffffffu, ties = 0;
  // (cmask: only the chunks whose bit is set wrote this run -- the wave's bits, a uniform loop)
  uint64_t bits = cmask != nullptr ? cmask[p >> 6] : 0ull;
  const uint32_t CN = cmask != nullptr ? (uint32_t)__builtin_popcountll(bits) : C;
  // branch-free, unrolled: every chunk's four words are loaded up front (several chunks in
  // flight), then folded with selects; equal bests keep the earlier chunk's (lower) index
#pragma unroll 4
  for (uint32_t k = 0; k < CN; ++k) {
    uint32_t c = k;
    if (cmask != nullptr) {
      c = (uint32_t)__builtin_ctzll(bits);
      bits &= bits - 1ull;
    }
    const size_t o = (size_t)c * n_pods + p;
    int64_t b, l;
    if (is_f64) {
      const double bf = pbest_f[o], lf = plow_f ? plow_f[o] : 1.0e300;
      b = bf < 0.0 ? -1 : (int64_t)bf;
      l = lf > 9.0e18 ? kI64Max : (int64_t)lf;
    } else {
      b = pbest_i[o];
      l = plow_i[o];
    }
    const uint32_t ix = pidx[o], tt = pties[o];
    const bool v = b >= 0, gt = v && b > best, eq = v && b == best;
    // (equal bests: the lower node -- chunks need not be in node order, block-grouped runs)
    idx = gt ? ix : (eq ? min(idx, ix) : idx);
    ties = gt ? tt : (eq ? ties + tt : ties);
    best = gt ? b : best;
    low = (v && l < low) ? l : low;
  }
  best_out[p] = best;
  idx_out[p] = idx == 0xffffffffu ? idx : idx + node_offset;
  ties_out[p] = ties;
  low_out[p] = (is_f64 && !plow_f) ? best : low;  // no lowest scores: the best in its place
}

// Wave-per-pod variant of k_reduce2 (many chunks).  Each lane merges a strided subset of
// chunks in increasing order; lanes then combine (best desc, idx asc), summing ties.
__global__ __launch_bounds__(kWave) void k_reduce2_wave(const double* __restrict__ pbest_f,
                                                         const int64_t* __restrict__ pbest_i,
                                                         const uint32_t* __restrict__ pidx,
                                                         const uint32_t* __restrict__ pties,
                                                         const double* __restrict__ plow_f,
                                                         const int64_t* __restrict__ plow_i,
                                                         uint32_t C, uint32_t n_pods, int is_f64,
                                                         uint32_t node_offset,
                                                         int64_t* __restrict__ best_out,
                                                         uint32_t* __restrict__ idx_out,
                                                         uint32_t* __restrict__ ties_out,
                                                         int64_t* __restrict__ low_out) {
  const uint32_t p = blockIdx.x, lane = threadIdx.x;
  int64_t best = -1, low = kI64Max;
  uint32_t idx = 0xffffffffu, ties = 0;
  for (uint32_t c = lane; c < C; c += kWave) {
    const size_t o = (size_t)c * n_pods + p;
    int64_t b, l;
    if (is_f64) {
      const double bf = pbest_f[o], lf = plow_f ? plow_f[o] : 1.0e300;
      b = bf < 0.0 ? -1 : (int64_t)bf;
      l = lf > 9.0e18 ? kI64Max : (int64_t)lf;
    } else {
      b = pbest_i[o];
      l = plow_i[o];
    }
    if (b < 0) continue;
    if (b > best) {
      best = b;
      idx = pidx[o];
      ties = pties[o];
    } else if (b == best) {
      ties += pties[o];
      idx = min(idx, pidx[o]);
    }
    low = l < low ? l : low;
  }
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const int64_t ob = __shfl_xor(best, o, kWave);
    const uint32_t oi = __shfl_xor(idx, o, kWave);
    const uint32_t ot = __shfl_xor(ties, o, kWave);
    const int64_t ol = __shfl_xor(low, o, kWave);
    if (ob > best) {
      best = ob;
      idx = oi;
      ties = ot;
    } else if (ob == best && ob >= 0) {
      ties += ot;
      idx = min(idx, oi);
    }
    low = ol < low ? ol : low;
  }
  if (lane != 0) return;
  best_out[p] = best;
  idx_out[p] = idx == 0xffffffffu ? idx : idx + node_offset;
  ties_out[p] = ties;
  low_out[p] = (is_f64 && !plow_f) ? best : low;  // no lowest scores: the best in its place
}

// Multi-GPU: after the MAX all-reduce of best, keep idx/ties only on shards that reach the
// global best (then MIN-reduce idx, SUM-reduce ties).
__global__ __launch_bounds__(kBlock) void k_merge_prepare(const int64_t* __restrict__ best_global,
                                                          const int64_t* __restrict__ best_local,
                                                          uint32_t n_pods, uint32_t* idx,
                                                          uint32_t* ties) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  if (best_local[p] != best_global[p] || best_global[p] < 0) {
    idx[p] = 0xffffffffu;
    ties[p] = 0;
  }
}

// Mode B: every node passes Filter.
__global__ __launch_bounds__(kBlock) void k_fill_diskio_state(uint32_t n_pods, uint32_t n_nodes,
                                                              uint64_t* __restrict__ maxima,
                                                              uint32_t* __restrict__ counts) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  for (int f = 0; f < 6; ++f) maxima[(size_t)f * n_pods + p] = 1;
  counts[p] = n_nodes;
  counts[(size_t)n_pods + p] = 0;
}

// Outcome of the cycle: NormalizeScore maps the raw maximum to 100
// and nothing else to 100 when (highest - lowest) * 100 cannot overflow int64, so selectHost
// picks among the raw-score maxima; ties broken by lowest node index.
__global__ __launch_bounds__(kBlock) void k_finalize(const uint32_t* __restrict__ counts,
                                                     const int64_t* __restrict__ best,
                                                     const uint32_t* __restrict__ idx,
                                                     const uint32_t* ties_io,
                                                     const int64_t* __restrict__ lowest,
                                                     uint32_t n_pods, int generic,
                                                     int32_t* __restrict__ pick,
                                                     int32_t* __restrict__ status,
                                                     uint32_t* ties_out,
                                                     uint32_t* __restrict__ flagged,
                                                     uint32_t* __restrict__ n_flagged,
                                                     FinalScatter sc) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  if (sc.perm) {
    // ordered run: every per-pod output goes straight to the caller's pod order (a padded
    // order's copies write the same values twice)
    const uint32_t q = sc.perm[p];
    sc.counts[q] = counts[p];
    sc.counts[(size_t)sc.n_out + q] = counts[(size_t)n_pods + p];
    sc.best[q] = best[p];
    if (sc.maxima) {
#pragma unroll
      for (int f = 0; f < 6; ++f)
        sc.maxima[(size_t)f * sc.n_out + q] = sc.maxima_in[(size_t)f * n_pods + p];
    }
  }
  const uint32_t o = sc.perm ? sc.perm[p] : p;  // where this pod's outputs land
  const uint32_t nf = counts[p], nz = counts[(size_t)n_pods + p];
  uint32_t t = ties_io[p];
  if (nf == 0) {
    pick[o] = -1;
    status[o] = 1;
    t = 0;
  } else if (nf == 1) {  // k8s: the only feasible node is returned without scoring
    pick[o] = (int32_t)idx[p];
    status[o] = 0;
    t = 1;
  } else if (nz > 0) {  // Score would divide by TotalMemorySum == 0: Go panics
    pick[o] = -2;
    status[o] = 2;
    t = 0;
  } else {
    const int64_t h = best[p];
    int64_t l = lowest[p];
    if (h == l) --l;  // scheduler.go:173-175
    if (generic && (uint64_t)(h - l) > (uint64_t)(kI64Max / 100)) {
      pick[o] = -3;  // pending: exact normalize (K3)
      status[o] = -1;
      flagged[atomicAdd(n_flagged, 1u)] = p;
    } else {
      pick[o] = (int32_t)idx[p];
      status[o] = 0;
    }
  }
  ties_out[o] = t;
}

// ---------------------------------------------------------------------------------------
// K3 (generic path, rare): NormalizeScore with Go's int64 wrap-around for pods whose
// (highest - lowest) * 100 can overflow, then the k8s range check and selectHost.  One lane
// per flagged pod.
template <int K>
__global__ __launch_bounds__(kBlock) void k3_exact_normalize(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const uint64_t* __restrict__ m_u, const uint64_t* __restrict__ c_u,
    const uint64_t* __restrict__ maxima, uint32_t n_pods, const uint64_t* __restrict__ bm,
    uint32_t bm_stride, const uint32_t* __restrict__ flagged,
    const uint32_t* __restrict__ n_flagged_p,
    const int64_t* __restrict__ best_in, const int64_t* __restrict__ low_in,
    int64_t* __restrict__ pbest, uint32_t* __restrict__ pidx, uint32_t* __restrict__ pties,
    uint32_t* __restrict__ perr, uint32_t max_flagged) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t nfl = min(*n_flagged_p, max_flagged);
  const uint32_t chunk = blockIdx.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  if (i >= nfl) return;
  const uint32_t p = flagged[i];
  const uint64_t m = m_u[p], c = c_u[p];
  uint64_t M[6];
  for (int f = 0; f < 6; ++f) M[f] = maxima[(size_t)f * n_pods + p];
  const int64_t h = best_in[p];
  int64_t l = low_in[p];
  if (h == l) --l;
  const int64_t d = h - l;
  int64_t best = -1;
  uint32_t idx = 0xffffffffu, ties = 0, err = 0;
  for (uint32_t n = n0; n < n1; ++n) {
    if (!bm_bit(bm, bm_stride, p, n)) continue;
    const int64_t s = raw_score_u64<K>(nodes + (size_t)n * node_stride(K), m, c, M);
    const int64_t norm = (int64_t)((uint64_t)(s - l) * 100u) / d;  // scheduler.go:178
    if (norm < 0 || norm > 100) err = 1;                            // RunScorePlugins check
    if (norm > best) {
      best = norm;
      idx = n;
      ties = 1;
    } else if (norm == best) {
      ++ties;
    }
  }
  const size_t o = (size_t)chunk * max_flagged + i;
  pbest[o] = best;
  pidx[o] = idx;
  pties[o] = ties;
  perr[o] = err;
}

__global__ __launch_bounds__(kBlock) void k_reduce3(const int64_t* __restrict__ pbest,
                                                    const uint32_t* __restrict__ pidx,
                                                    const uint32_t* __restrict__ pties,
                                                    const uint32_t* __restrict__ perr, uint32_t C,
                                                    const uint32_t* __restrict__ flagged,
                                                    const uint32_t* __restrict__ n_flagged_p,
                                                    uint32_t max_flagged, uint32_t node_offset,
                                                    int32_t* __restrict__ pick,
                                                    int32_t* __restrict__ status,
                                                    uint32_t* __restrict__ ties_out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= min(*n_flagged_p, max_flagged)) return;
  const uint32_t p = flagged[i];
  int64_t best = -1;
  uint32_t idx = 0xffffffffu, ties = 0, err = 0;
  for (uint32_t c = 0; c < C; ++c) {
    const size_t o = (size_t)c * max_flagged + i;
    err |= perr[o];
    const int64_t b = pbest[o];
    if (b < 0) continue;
    if (b > best) {
      best = b;
      idx = pidx[o];
      ties = pties[o];
    } else if (b == best) {
      ties += pties[o];
    }
  }
  if (err) {
    pick[p] = -2;
    status[p] = 3;
    ties_out[p] = 0;
  } else {
    pick[p] = (int32_t)(idx + node_offset);
    status[p] = 0;
    ties_out[p] = ties;
  }
}

// Sharded K3 (several node shards): each shard folds its chunk partials of the flagged pods
// into one record per pod -- {best normalized score, lowest GLOBAL node reaching it, ties,
// low := 1 if a score left [0, 100]} at rec[p] -- the records are all-gathered across the
// shards and k_merge3 folds them (best MAX, lowest node among the shards reaching it, ties
// summed over those, range errors OR-ed) into the picks as k_reduce3 would.
__global__ __launch_bounds__(kBlock) void k_reduce3_rec(const int64_t* __restrict__ pbest,
                                                        const uint32_t* __restrict__ pidx,
                                                        const uint32_t* __restrict__ pties,
                                                        const uint32_t* __restrict__ perr,
                                                        uint32_t C,
                                                        const uint32_t* __restrict__ flagged,
                                                        const uint32_t* __restrict__ n_flagged_p,
                                                        uint32_t max_flagged, uint32_t node_offset,
                                                        ShardRec* __restrict__ rec) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= min(*n_flagged_p, max_flagged)) return;
  const uint32_t p = flagged[i];
  int64_t best = -1;
  uint32_t idx = 0xffffffffu, ties = 0, err = 0;
  for (uint32_t c = 0; c < C; ++c) {
    const size_t o = (size_t)c * max_flagged + i;
    err |= perr[o];
    const int64_t b = pbest[o];
    if (b < 0) continue;
    if (b > best) {
      best = b;
      idx = pidx[o];
      ties = pties[o];
    } else if (b == best) {
      ties += pties[o];
    }
  }
  rec[p] = ShardRec{best, idx == 0xffffffffu ? idx : idx + node_offset, ties, (int64_t)err};
}

__global__ __launch_bounds__(kBlock) void k_merge3(const ShardRec* __restrict__ all,
                                                   uint32_t n_pods, uint32_t world,
                                                   const uint32_t* __restrict__ flagged,
                                                   const uint32_t* __restrict__ n_flagged_p,
                                                   uint32_t max_flagged,
                                                   int32_t* __restrict__ pick,
                                                   int32_t* __restrict__ status,
                                                   uint32_t* __restrict__ ties_out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= min(*n_flagged_p, max_flagged)) return;
  const uint32_t p = flagged[i];
  int64_t best = -1;
  uint32_t idx = 0xffffffffu, ties = 0, err = 0;
  for (uint32_t r = 0; r < world; ++r) {
    const ShardRec x = all[(size_t)r * n_pods + p];
    err |= x.low != 0 ? 1u : 0u;
    if (x.best < 0) continue;
    if (x.best > best) {
      best = x.best;
      idx = x.idx;
      ties = x.ties;
    } else if (x.best == best) {
      idx = min(idx, x.idx);
      ties += x.ties;
    }
  }
  if (err) {
    pick[p] = -2;
    status[p] = 3;
    ties_out[p] = 0;
  } else {
    pick[p] = (int32_t)idx;
    status[p] = 0;
    ties_out[p] = ties;
  }
}

hipError_t launch_reduce3_rec(const Partials& part, uint32_t C, const uint32_t* flagged,
                              const uint32_t* n_flagged, uint32_t max_flagged,
                              uint32_t node_offset, ShardRec* rec, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce3_rec, pod_grid(max_flagged), dim3(kBlock), 0, s, part.best_i,
                     part.idx, part.ties, part.err, C, flagged, n_flagged, max_flagged,
                     node_offset, rec);
  return hipGetLastError();
}

hipError_t launch_merge3(const ShardRec* all, uint32_t n_pods, uint32_t world,
                         const uint32_t* flagged, const uint32_t* n_flagged, uint32_t max_flagged,
                         int32_t* pick, int32_t* status, uint32_t* ties, hipStream_t s) {
  hipLaunchKernelGGL(k_merge3, pod_grid(max_flagged), dim3(kBlock), 0, s, all, n_pods, world,
                     flagged, n_flagged, max_flagged, pick, status, ties);
  return hipGetLastError();
}

// Bitmask [wave][node] u64 (device, yoda_layout.h) -> [P][W] u32 words (host API layout:
// word w of pod q, bit b = node 32 w + b).
__global__ __launch_bounds__(kBlock) void k_bitmask_transpose(const MaskSrc ms,
                                                              uint32_t n_nodes, uint32_t W,
                                                              uint32_t n_pods,
                                                              const uint32_t* __restrict__ perm,
                                                              uint32_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (uint64_t)W * n_pods) return;
  const uint32_t p = (uint32_t)(t / W), w = (uint32_t)(t % W);
  // row p of the output belongs to caller pod perm[p] when the run was ordered
  const uint32_t q = perm ? perm[p] : p;
  uint32_t bits = 0;
  for (uint32_t b = 0; b < 32u && 32u * w + b < n_nodes; ++b)
    bits |= (uint32_t)((mask_at(ms, p >> 6, 32u * w + b, n_pods) >> (p & 63u)) & 1ull) << b;
  out[(size_t)q * W + w] = bits;
}

// ---------------------------------------------------------------------------------------
// Launchers (host side of this translation unit).
#define YODA_K_SWITCH(K, ...)                       \
  switch (K) {                                      \
    case 1: { constexpr int KK = 1; __VA_ARGS__; } break;  \
    case 2: { constexpr int KK = 2; __VA_ARGS__; } break;  \
    case 4: { constexpr int KK = 4; __VA_ARGS__; } break;  \
    case 8: { constexpr int KK = 8; __VA_ARGS__; } break;  \
    case 16: { constexpr int KK = 16; __VA_ARGS__; } break; \
    default: return hipErrorInvalidValue;           \
  }



// sub (block K1 only): 1, or 4 = one pod wave per workgroup over four quarters of each
// chunk, chunk_nodes then being the quarter (k1_block_n32's SUB).
hipError_t launch_k1(int K, Path path, const unsigned char* nodes, const unsigned char* sum,
                     const unsigned char* sum2, const unsigned char* mix, uint32_t n_nodes, uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                     uint32_t n_pods, const Partials& part, uint64_t* bm, uint32_t bm_stride,
                     BlockMask* bs, uint32_t bs_stride, uint64_t* blk, uint32_t blk_stride,
                     unsigned long long* stats, hipStream_t s, uint32_t sub) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  switch (path) {
    case Path::N32:
      if (sum) {
        if (sub != 1u && sub != (uint32_t)(kBlock / kWave)) return hipErrorInvalidValue;
        const dim3 g1 = sub == 1u ? grid : dim3((n_pods + kWave - 1) / kWave, C);
#define YODA_K1B(...)                                                                          \
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_block_n32<__VA_ARGS__>), g1, dim3(kBlock), 0, s, nodes, \
                                      sum, reinterpret_cast<const uint32_t*>(sum2),            \
                                      reinterpret_cast<const uint32_t*>(mix), pp.x1, n_nodes,  \
                                      chunk_nodes, pp.m_32, pp.c_32, pp.number, pp.need_mem,   \
                                      pp.need_clk, n_pods, part.max_u, part.cnt, bm, bm_stride, \
                                      bs, bs_stride, blk, blk_stride, stats, nullptr, pp.bsum,   \
                                      pp.nwords, pp.lpt_w, pp.seed ? pp.g.tab : nullptr,         \
                                      pp.kbub_exact ? pp.kbub : nullptr, pp.kb_levels,           \
                                      reinterpret_cast<unsigned long long*>(pp.seed),          \
                                      reinterpret_cast<unsigned long long*>(pp.cmask1), pp.ids, \
                                      pp.k1_order))
        if (sub == 1u) {
          if (stats) YODA_K1B(KK, true)
          else if (pp.one_model) YODA_K1B(KK, false, false)
          else YODA_K1B(KK, false)
        } else {
          if (stats) YODA_K1B(KK, true, true, false, kBlock / kWave)
          else if (pp.one_model) YODA_K1B(KK, false, false, false, kBlock / kWave)
          else YODA_K1B(KK, false, true, false, kBlock / kWave)
        }
#undef YODA_K1B
      } else {
        YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_filter_maxima<KK, Path::N32>), grid, dim3(kBlock),
                                            0, s, nodes, n_nodes, chunk_nodes, pp.m_32, pp.c_32,
                                            pp.number, pp.need_mem, pp.need_clk, n_pods,
                                            part.max_u, part.cnt, bm, bm_stride));
      }
      break;
    case Path::F64:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_filter_maxima<KK, Path::F64>), grid, dim3(kBlock), 0,
                                          s, nodes, n_nodes, chunk_nodes, pp.m_f, pp.c_f,
                                          pp.number, pp.need_mem, pp.need_clk, n_pods, part.max_u,
                                          part.cnt, bm, bm_stride));
      break;
    case Path::U64:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_filter_maxima<KK, Path::U64>), grid, dim3(kBlock), 0,
                                          s, nodes, n_nodes, chunk_nodes, pp.m_u, pp.c_u,
                                          pp.number, pp.need_mem, pp.need_clk, n_pods, part.max_u,
                                          part.cnt, bm, bm_stride));
      break;
  }
  return hipGetLastError();
}

// Resident 256-thread workgroups of one K1 / K2 instantiation on the whole device (occupancy
// API x CUs), for grid sizing.  which: 1 = K1, 2 = K2.
int kernel_capacity(int K, Path path, int which, int mode_diskio) {
  int dev = 0, cus = 0, nb = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const void* fn = nullptr;
#define YODA_FN(expr) fn = reinterpret_cast<const void*>(expr)
  if (mode_diskio) {
    YODA_FN(&k2_diskio<false>);
  } else if (which == 1) {
    switch (path) {
      // (the one-model tiles' kernel: the chunk plan of config 3 as measured)
      case Path::N32: YODA_K_SWITCH(K, YODA_FN((&k1_block_n32<KK, false, false>))); break;
      case Path::F64: YODA_K_SWITCH(K, YODA_FN((&k1_filter_maxima<KK, Path::F64>))); break;
      case Path::U64: YODA_K_SWITCH(K, YODA_FN((&k1_filter_maxima<KK, Path::U64>))); break;
    }
  } else {
    switch (path) {
      case Path::N32:
        YODA_K_SWITCH(K, YODA_FN((&k2_block_n32<KK, false>)));
        break;
      case Path::F64: YODA_K_SWITCH(K, YODA_FN((&k2_score<KK, Path::F64, OUT_ARGMAX>))); break;
      case Path::U64: YODA_K_SWITCH(K, YODA_FN((&k2_score_generic<KK, false>))); break;
    }
  }
#undef YODA_FN
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kBlock, 0) != hipSuccess) return 0;
  return nb * cus;
}

// Chunk partials are merged one thread per pod (coalesced over pods) when there are few
// chunks, one wave per pod (strided over chunks) when there are many.
constexpr uint32_t kWaveReduceChunks = 48;

hipError_t launch_prep2(const uint64_t* maxima, uint32_t n_pods, double* rcp,
                        hipStream_t s);

// rcp non-null: also the reciprocals (k_prep2 fused; the wave variant runs it after)
// nw: the block K1's partial words (kNarrowWords / kWideWords), 0: u64 partials [6][C][P]
// lpt_w / lpt_order non-null: also the block K2's heaviest-first pod-block order (k_lpt_order;
// in k_reduce1's grid as one extra workgroup where that kernel runs)
hipError_t launch_lpt_order(uint32_t* wts, uint32_t n_pods, uint32_t* order, hipStream_t s);
hipError_t launch_reduce1(const Partials& part, uint32_t C, uint32_t n_pods, uint32_t nw,
                          uint64_t* maxima, uint32_t* counts, double* rcp,
                          const MemTab& mt, hipStream_t s, uint32_t* lpt_w,
                          uint32_t* lpt_order, const uint64_t* cmask) {
  if (cmask != nullptr && (C > kWaveReduceChunks || !nw)) return hipErrorInvalidValue;
  const bool lpt_apart = lpt_w != nullptr && (C > kWaveReduceChunks || !nw);
  if (lpt_apart) {
    const hipError_t e = launch_lpt_order(lpt_w, n_pods, lpt_order, s);
    if (e != hipSuccess) return e;
  }
  if (C > kWaveReduceChunks && n_pods >= 2 * kBlock) {
    // split the chunks so that ~64k threads read the partials, then atomics
    const uint32_t pb = (n_pods + kBlock - 1) / kBlock;
    const uint32_t S = std::max<uint32_t>(1, std::min<uint32_t>(C / 16, 256 / pb + 1));
    hipError_t e = hipMemsetAsync(maxima, 0, 6 * (size_t)n_pods * 8, s);
    if (e == hipSuccess) e = hipMemsetAsync(counts, 0, 2 * (size_t)n_pods * 4, s);
    if (e != hipSuccess) return e;
    const dim3 grid(pb, nw ? nw + 2u : 8u, S);
    if (nw)
      hipLaunchKernelGGL(k_reduce1_split<true>, grid, dim3(kBlock), 0, s, part.max_u, part.cnt, C,
                         n_pods, maxima, counts, nw);
    else
      hipLaunchKernelGGL(k_reduce1_split<false>, grid, dim3(kBlock), 0, s, part.max_u, part.cnt,
                         C, n_pods, maxima, counts, 0u);
    if (mt.vf)  // the atomics ran in rank space
      hipLaunchKernelGGL(k_rank_maxima, pod_grid(n_pods), dim3(kBlock), 0, s, maxima, n_pods, mt);
    if (rcp) return launch_prep2(maxima, n_pods, rcp, s);
  } else if (C > kWaveReduceChunks) {
    if (nw)
      hipLaunchKernelGGL(k_reduce1_wave<true>, dim3(n_pods), dim3(kWave), 0, s, part.max_u,
                         part.cnt, C, n_pods, maxima, counts, mt, nw);
    else
      hipLaunchKernelGGL(k_reduce1_wave<false>, dim3(n_pods), dim3(kWave), 0, s, part.max_u,
                         part.cnt, C, n_pods, maxima, counts, mt, 0u);
    if (rcp) return launch_prep2(maxima, n_pods, rcp, s);
  } else {
    const bool lpt = lpt_w != nullptr && !lpt_apart;
    const dim3 grid((n_pods + kBlock - 1) / kBlock + (lpt ? 1u : 0u), nw ? nw + 2u : 8u);
    if (nw)
      hipLaunchKernelGGL(k_reduce1<true>, grid, dim3(kBlock), 0, s, part.max_u, part.cnt, C,
                         n_pods, maxima, counts, rcp, mt, nw, lpt ? lpt_w : nullptr,
                         lpt ? lpt_order : nullptr,
                         reinterpret_cast<const unsigned long long*>(cmask));
    else
      hipLaunchKernelGGL(k_reduce1<false>, grid, dim3(kBlock), 0, s, part.max_u, part.cnt, C,
                         n_pods, maxima, counts, rcp, mt, 0u);
  }
  return hipGetLastError();
}

hipError_t launch_prep2(const uint64_t* maxima, uint32_t n_pods, double* rcp,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_prep2, pod_grid(n_pods), dim3(kBlock), 0, s, maxima, n_pods, rcp);
  return hipGetLastError();
}

hipError_t launch_window_out(const uint32_t* counts, const uint64_t* maxima, const uint32_t* wit,
                             const double* tk_s, const uint32_t* tk_i, const uint32_t* perm,
                             uint32_t wn, uint32_t kt, bool lists_row_major, unsigned char* out,
                             uint32_t* inv_scratch, hipStream_t s) {
  if (wn == 0) return hipSuccess;
  hipLaunchKernelGGL(k_window_out, pod_grid(wn), dim3(kBlock), 0, s, counts, maxima, wit, tk_s,
                     tk_i, perm, wn, kt, lists_row_major ? 1 : 0, out, inv_scratch);
  if (inv_scratch && kt > 0) {
    const size_t n = (size_t)wn * kt;
    hipLaunchKernelGGL(k_window_lists, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, s, tk_s, tk_i, inv_scratch, wn, kt, lists_row_major ? 1 : 0, out);
  }
  return hipGetLastError();
}

template <int OUT>
static hipError_t launch_k2_t(int K, Path path, const unsigned char* nodes,
                              const unsigned char* sum2, const uint64_t* blk, uint32_t blk_stride,
                              uint32_t n_nodes,
                              uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                              const uint64_t* maxima, const double* rcp,
                              uint32_t n_pods, const uint64_t* bm, uint32_t bm_stride,
                              const BlockMask* bs, uint32_t bs_stride, const Partials& part,
                              int64_t* rows, double* tk_s, uint32_t* tk_i,
                              unsigned long long* stats, const uint32_t* counts, hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  const ScoreArgs a{pp.m_f, pp.c_f, pp.m_32, pp.c_32, rcp, counts, pp.g, pp.mix, pp.mt,
                    pp.ids, OUT == OUT_ARGMAX ? pp.kbub : nullptr,
                    OUT == OUT_ARGMAX ? pp.hot : nullptr, OUT == OUT_ARGMAX ? pp.lpt_order : nullptr,
                    OUT == OUT_ARGMAX ? reinterpret_cast<const unsigned long long*>(pp.seed) : nullptr,
                    OUT == OUT_ARGMAX && pp.kbub ? pp.kb_levels : nullptr,
                    OUT == OUT_ARGMAX && pp.kbub ? pp.kbdec : nullptr,
                    OUT == OUT_ARGMAX ? reinterpret_cast<unsigned long long*>(pp.gbest) : nullptr,
                    OUT == OUT_ARGMAX && sum2 ? reinterpret_cast<unsigned long long*>(pp.cmask2)
                                              : nullptr};
  const MaskSrc ms{bm, bs, bm_stride, bs_stride, blk, blk_stride};
  if (bs && !blk) return hipErrorInvalidValue;  // sparse masks are read through their block list
  switch (path) {
    case Path::N32:
      if (OUT == OUT_ARGMAX && sum2) {
#define YODA_K2B(ST, RKV, MIXV, Q32V)                                                           \
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_block_n32<KK, ST, 0, RKV, MIXV, Q32V>), grid,          \
                                      dim3(kBlock), 0, s, nodes, sum2, n_nodes, chunk_nodes, a,   \
                                      n_pods, bm, bm_stride, bs, bs_stride, blk, blk_stride,      \
                                      part.best_f, part.idx, part.ties, part.low_f, stats,        \
                                      nullptr, 0u))
        // memory ranks: the kernel of its own (RK = true); small fields beyond kF32SmallMax
        // (one-model snapshots only, yoda_capi.cpp n32_ok): the f64-quotient kernels
        if (!pp.q32) {
          if (stats) {
            if (a.mt.vf) YODA_K2B(true, true, true, false) else YODA_K2B(true, false, true, false);
          } else if (a.mt.vf) {
            YODA_K2B(false, true, true, false);
          } else {
            if (!pp.all_uni4) return hipErrorInvalidValue;
            YODA_K2B(false, false, false, false);
          }
        } else if (stats) {
          if (a.mt.vf) YODA_K2B(true, true, true, true) else YODA_K2B(true, false, true, true);
        } else if (pp.all_uni4 && !a.mt.vf) {
          YODA_K2B(false, false, false, true);
        } else if (pp.all_uni4) {  // memory ranks on one-model nodes (e.g. memory in bytes)
          YODA_K2B(false, true, false, true);
        } else {
          if (a.mt.vf) YODA_K2B(false, true, true, true) else YODA_K2B(false, false, true, true);
        }
#undef YODA_K2B
        break;
      }
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_score<KK, Path::N32, OUT>), grid, dim3(kBlock), 0,
                                          s, nodes, n_nodes, chunk_nodes, a, n_pods, ms,
                                          part.best_f, part.idx, part.ties, part.low_f, rows,
                                          tk_s, tk_i));
      break;
    case Path::F64:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_score<KK, Path::F64, OUT>), grid, dim3(kBlock), 0,
                                          s, nodes, n_nodes, chunk_nodes, a, n_pods, ms,
                                          part.best_f, part.idx, part.ties, part.low_f, rows,
                                          tk_s, tk_i));
      break;
    case Path::U64:
      if (OUT == OUT_TOPK) return hipErrorInvalidValue;
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_score_generic<KK, OUT == OUT_ROWS>), grid,
                                          dim3(kBlock), 0, s, nodes, n_nodes, chunk_nodes,
                                          pp.m_u, pp.c_u, maxima, n_pods, bm, bm_stride, part.best_i,
                                          part.idx, part.ties, part.low_i, rows));
      break;
  }
  return hipGetLastError();
}

hipError_t launch_k2_topk(int K, Path path, const unsigned char* nodes, uint32_t n_nodes,
                          uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                          const double* rcp, uint32_t n_pods,
                          const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                          uint32_t bs_stride, const uint64_t* blk, uint32_t blk_stride,
                          const Partials& part, double* tk_s, uint32_t* tk_i, int tk,
                          hipStream_t s) {
  if (tk != kTopK && tk != kTopKCap) return hipErrorInvalidValue;
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  const ScoreArgs a{pp.m_f, pp.c_f, pp.m_32, pp.c_32, rcp};
  const MaskSrc ms{bm, bs, bm_stride, bs_stride, blk, blk_stride};
  if (bs && !blk) return hipErrorInvalidValue;  // sparse masks are read through their block list
#define YODA_TOPK(PTH, TKV)                                                                      \
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_score<KK, PTH, OUT_TOPK, TKV>), grid, dim3(kBlock), 0, \
                                      s, nodes, n_nodes, chunk_nodes, a, n_pods, ms, part.best_f, \
                                      part.idx, part.ties, part.low_f, nullptr, tk_s, tk_i))
  switch (path) {
    case Path::N32:
      if (tk == kTopK) YODA_TOPK(Path::N32, kTopK) else YODA_TOPK(Path::N32, kTopKCap);
      break;
    case Path::F64:
      if (tk == kTopK) YODA_TOPK(Path::F64, kTopK) else YODA_TOPK(Path::F64, kTopKCap);
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef YODA_TOPK
  return hipGetLastError();
}

// The block K2's packed-key top-k (N32 path with node summaries; DESIGN.md §5 greedy):
// keys [C][P][tk], merged by launch_topk_merge_keys.  counts: the pods' feasible-node counts
// (a pod with none takes no part in the wave's bounds).
hipError_t launch_k2_topk_block(int K, const unsigned char* nodes, const unsigned char* sum2,
                                const uint64_t* blk, uint32_t blk_stride, uint32_t n_nodes,
                                uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                                const double* rcp, uint32_t n_pods,
                                const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                                uint32_t bs_stride, const uint32_t* counts, uint64_t* keys,
                                uint32_t ib, int tk, hipStream_t s) {
  if ((tk != kTopK && tk != kTopKCap) || K > 8 || n_pods == 0) return hipErrorInvalidValue;
  if (bs && !blk) return hipErrorInvalidValue;  // sparse masks are read through their block list
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  const ScoreArgs a{pp.m_f, pp.c_f, pp.m_32, pp.c_32, rcp, counts, pp.g, pp.mix, pp.mt,
                    nullptr, pp.kbub, nullptr, pp.lpt_order, nullptr,
                    pp.kbub ? pp.kb_levels : nullptr, pp.kbub ? pp.kbdec : nullptr,
                    reinterpret_cast<unsigned long long*>(pp.gbest)};
#define YODA_TOPKB(TKV, RKV, MIXV, Q32V)                                                        \
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_block_n32<KK, false, TKV, RKV, MIXV, Q32V>), grid,      \
                                      dim3(kBlock), 0, s, nodes, sum2, n_nodes, chunk_nodes, a,   \
                                      n_pods, bm, bm_stride, bs, bs_stride, blk, blk_stride,      \
                                      nullptr, nullptr, nullptr, nullptr, nullptr, keys, ib))
  // one-model snapshots without memory ranks: the kernel without the mixed-model rows;
  // small fields beyond kF32SmallMax (one-model snapshots only): the f64-quotient kernels
  const bool lean = pp.all_uni4 && !a.mt.vf;
  if (!pp.q32 && !a.mt.vf && !lean) return hipErrorInvalidValue;
  if (tk == kTopK) {
    if (!pp.q32) {
      if (a.mt.vf) YODA_TOPKB(kTopK, true, true, false) else YODA_TOPKB(kTopK, false, false, false);
    } else if (a.mt.vf) YODA_TOPKB(kTopK, true, true, true)
    else if (lean) YODA_TOPKB(kTopK, false, false, true)
    else YODA_TOPKB(kTopK, false, true, true);
  } else {
    if (!pp.q32) {
      if (a.mt.vf) YODA_TOPKB(kTopKCap, true, true, false)
      else YODA_TOPKB(kTopKCap, false, false, false);
    } else if (a.mt.vf) YODA_TOPKB(kTopKCap, true, true, true)
    else if (lean) YODA_TOPKB(kTopKCap, false, false, true)
    else YODA_TOPKB(kTopKCap, false, true, true);
  }
#undef YODA_TOPKB
  return hipGetLastError();
}

// The 16-deep chunk lists merged into ko-deep exact-prefix lists (k_topk_merge_deep).
hipError_t launch_topk_merge_deep(const uint64_t* keys, uint32_t C, uint32_t n_pods, uint32_t ib,
                                  uint32_t node_offset, double* out_s, uint32_t* out_i, int tk,
                                  int ko, hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  if (tk != kTopK && tk != kTopKCap) return hipErrorInvalidValue;
  const dim3 grid(n_pods);
#define YODA_DEEP(TKV, KOV)                                                                     \
  hipLaunchKernelGGL((k_topk_merge_deep<TKV, KOV>), grid, dim3(kWave), 0, s, keys, C, n_pods, ib, \
                     node_offset, out_s, out_i)
  switch (ko) {
    case 32:
      if (tk == kTopK) YODA_DEEP(kTopK, 32); else YODA_DEEP(kTopKCap, 32);
      break;
    case 64:
      if (tk == kTopK) YODA_DEEP(kTopK, 64); else YODA_DEEP(kTopKCap, 64);
      break;
    case 128:
      if (tk == kTopK) YODA_DEEP(kTopK, 128); else YODA_DEEP(kTopKCap, 128);
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef YODA_DEEP
  return hipGetLastError();
}

hipError_t launch_topk_merge_keys(const uint64_t* keys, uint32_t C, uint32_t n_pods, uint32_t ib,
                                  uint32_t node_offset, double* out_s, uint32_t* out_i, int tk,
                                  hipStream_t s) {
  if (tk != kTopK && tk != kTopKCap) return hipErrorInvalidValue;
  const dim3 grid(n_pods);  // one workgroup per pod
  if (n_pods == 0) return hipSuccess;
  if (tk == kTopK)
    hipLaunchKernelGGL(k_topk_merge_keys<kTopK>, grid, dim3(kBlock), 0, s, keys, C, n_pods, ib,
                       node_offset, out_s, out_i);
  else
    hipLaunchKernelGGL(k_topk_merge_keys<kTopKCap>, grid, dim3(kBlock), 0, s, keys, C, n_pods, ib,
                       node_offset, out_s, out_i);
  return hipGetLastError();
}

hipError_t launch_topk_merge(const double* tk_s, const uint32_t* tk_i, uint32_t C,
                             uint32_t n_pods, uint32_t node_offset, double* out_s,
                             uint32_t* out_i, int tk, hipStream_t s) {
  if (tk != kTopK && tk != kTopKCap) return hipErrorInvalidValue;
  if (C > 8) {
    if (tk == kTopK)
      hipLaunchKernelGGL(k_topk_merge_wave<kTopK>, dim3(n_pods), dim3(kWave), 0, s, tk_s, tk_i, C,
                         n_pods, node_offset, out_s, out_i);
    else
      hipLaunchKernelGGL(k_topk_merge_wave<kTopKCap>, dim3(n_pods), dim3(kWave), 0, s, tk_s, tk_i,
                         C, n_pods, node_offset, out_s, out_i);
    return hipGetLastError();
  }
  if (tk == kTopK)
    hipLaunchKernelGGL(k_topk_merge<kTopK>, pod_grid(n_pods), dim3(kBlock), 0, s, tk_s, tk_i, C,
                       n_pods, node_offset, out_s, out_i);
  else
    hipLaunchKernelGGL(k_topk_merge<kTopKCap>, pod_grid(n_pods), dim3(kBlock), 0, s, tk_s, tk_i,
                       C, n_pods, node_offset, out_s, out_i);
  return hipGetLastError();
}

// Tighten the blocks' CardNumber bounds again (BlockSumWord cn_min / cn_max) from the K1
// summaries' current values, one wave per 64-node block.
__global__ __launch_bounds__(kWave) void k_bsum_cn(const uint32_t* __restrict__ sum,
                                                   uint32_t sum_stride, uint32_t n_nodes,
                                                   uint32_t* __restrict__ bsum, uint32_t bsw) {
  const uint32_t b = blockIdx.x, n = b * 64u + threadIdx.x;
  const bool v = n < n_nodes;
  uint64_t cn = 0;
  if (v)
    cn = (uint64_t)sum[sum_index(n, kSumCnLo, sum_stride)] |
         ((uint64_t)sum[sum_index(n, kSumCnHi, sum_stride)] << 32);
  const uint64_t lo = wave_min_u64(v ? cn : ~0ull), hi = wave_max_u64(v ? cn : 0ull);
  if (threadIdx.x == 0) {
    bsum[sum_index(b, kBsCnMin, 4u * bsw)] = (uint32_t)min(lo, (uint64_t)0xffffffffu);
    bsum[sum_index(b, kBsCnMax, 4u * bsw)] = (uint32_t)min(hi, (uint64_t)0xffffffffu);
  }
}

hipError_t launch_bsum_cn(const unsigned char* sum, uint32_t sum_stride, uint32_t n_nodes,
                          uint32_t* bsum, uint32_t bsw, hipStream_t s) {
  if (n_nodes == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bsum_cn, dim3((n_nodes + 63) / 64), dim3(kWave), 0, s,
                     reinterpret_cast<const uint32_t*>(sum), sum_stride, n_nodes, bsum, bsw);
  return hipGetLastError();
}

hipError_t launch_set_static(unsigned char* nodes, uint32_t stride, const uint32_t* node,
                             const uint64_t* value, const uint64_t* card_number, uint32_t count,
                             unsigned char* sum, uint32_t sum_stride, unsigned char* sum2,
                             uint32_t sum2_stride, const PermCopy& pc, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_set_static, pod_grid(count), dim3(kBlock), 0, s, nodes, stride, node,
                     value, card_number, count, sum, sum_stride, sum2, sum2_stride, pc);
  return hipGetLastError();
}

int topk_k() { return kTopK; }
int topk_k_capacity() { return kTopKCap; }

// Partials of k_greedy_one: at most this many blocks (grid-stride over the nodes).
constexpr uint32_t kGreedyOneBlocks = 512;
uint32_t greedy_one_blocks() { return kGreedyOneBlocks; }

hipError_t launch_greedy_one(int K, Path path, const unsigned char* nodes,
                             const unsigned char* sum2, uint32_t n_nodes,
                             const PodParams& pp, const double* rcp,
                             uint32_t n_pods, uint32_t s, const uint64_t* bm, uint32_t bm_stride,
                             const BlockMask* bs, uint32_t bs_stride, const uint64_t* blk,
                             uint32_t blk_stride, double* part_s, uint32_t* part_i,
                             uint32_t* done, uint32_t* out, hipStream_t st) {
  ScoreArgs a{pp.m_f, pp.c_f, pp.m_32, pp.c_32, rcp};
  a.g = pp.g;
  a.mt = pp.mt;
  const MaskSrc ms{bm, bs, bm_stride, bs_stride, blk, blk_stride};
  if (bs && !blk) return hipErrorInvalidValue;  // sparse masks are read through their block list
  const uint32_t* s2 = reinterpret_cast<const uint32_t*>(sum2);
  const dim3 grid(std::max<uint32_t>(1, std::min<uint32_t>(kGreedyOneBlocks,
                                                           (n_nodes + kBlock - 1) / kBlock)));
  switch (path) {
    case Path::N32:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k_greedy_one<KK, Path::N32>), grid, dim3(kBlock), 0,
                                          st, nodes, s2, n_nodes, a, n_pods, s, ms, part_s,
                                          part_i, done, out));
      break;
    case Path::F64:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k_greedy_one<KK, Path::F64>), grid, dim3(kBlock), 0,
                                          st, nodes, nullptr, n_nodes, a, n_pods, s, ms, part_s,
                                          part_i, done, out));
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_k2(int K, Path path, const unsigned char* nodes, const unsigned char* sum2,
                     const uint64_t* blk, uint32_t blk_stride, uint32_t n_nodes,
                     uint32_t chunk_nodes, uint32_t C, const PodParams& pp, const uint64_t* maxima,
                     const double* rcp, uint32_t n_pods,
                     const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                     uint32_t bs_stride, const Partials& part, int64_t* rows,
                     unsigned long long* stats, const uint32_t* counts, hipStream_t s) {
  if (rows)
    return launch_k2_t<OUT_ROWS>(K, path, nodes, nullptr, blk, blk_stride, n_nodes, chunk_nodes, C, pp, maxima, rcp, n_pods, bm, bm_stride, bs, bs_stride, part, rows, nullptr,
                                 nullptr, stats, counts, s);
  return launch_k2_t<OUT_ARGMAX>(K, path, nodes, sum2, blk, blk_stride, n_nodes, chunk_nodes, C, pp, maxima, rcp, n_pods, bm, bm_stride, bs, bs_stride, part, rows, nullptr,
                                 nullptr, stats, counts, s);
}

hipError_t launch_k2b_rows(const NodeRecB* nodes, uint32_t n_nodes, const PodParams& pp,
                           uint32_t n_pods, const Partials& part, int64_t* rows, hipStream_t s) {
  if (n_nodes == 0 || n_pods == 0) return hipSuccess;
  hipLaunchKernelGGL(k2b_rows, dim3((n_nodes + kBlock - 1) / kBlock), dim3(kBlock), 0, s, nodes,
                     n_nodes, pp.alpha, pp.beta, n_pods, part.best_f, part.idx, part.ties,
                     part.low_f, rows);
  return hipGetLastError();
}

hipError_t launch_k2_diskio(const NodeRecB* nodes, uint32_t n_nodes, uint32_t chunk_nodes,
                            uint32_t C, const PodParams& pp, uint32_t n_pods, const Partials& part,
                            int64_t* rows, hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  if (rows)
    hipLaunchKernelGGL(k2_diskio<true>, grid, dim3(kBlock), 0, s, nodes, n_nodes, chunk_nodes,
                       pp.alpha, pp.beta, n_pods, part.best_f, part.idx, part.ties, part.low_f,
                       rows);
  else
    hipLaunchKernelGGL(k2_diskio<false>, grid, dim3(kBlock), 0, s, nodes, n_nodes, chunk_nodes,
                       pp.alpha, pp.beta, n_pods, part.best_f, part.idx, part.ties, part.low_f,
                       rows);
  return hipGetLastError();
}

// Mode B batch plan: few classes (<= 64) run lane = node in chunks of 2048 nodes, one
// workgroup per (chunk, class); more run lane = class (4 per lane) in enough node chunks for
// ~8 resident waves per SIMD.
constexpr uint32_t kDiskNodeLaneMaxCls = 64;
constexpr uint32_t kDiskNodeLaneChunk = 2048;
constexpr int kDiskCPL = 4;

DiskPlan diskio_plan(uint32_t n_nodes, uint32_t n_cls) {
  DiskPlan pl{};
  if (n_nodes == 0 || n_cls == 0) return pl;
  pl.node_lanes = n_cls <= kDiskNodeLaneMaxCls;
  if (pl.node_lanes) {
    pl.chunk = kDiskNodeLaneChunk;
  } else {
    const uint32_t waves = (n_cls + kWave * kDiskCPL - 1) / (kWave * kDiskCPL);
    uint32_t C = (8192u + waves - 1) / waves;
    C = std::max(1u, std::min(C, (n_nodes + 63u) / 64u));
    pl.chunk = (n_nodes + C - 1) / C;
  }
  pl.C = (n_nodes + pl.chunk - 1) / pl.chunk;
  return pl;
}

hipError_t launch_k2b(const NodeRecB* nodes, uint32_t n_nodes, const double* cab,
                      uint32_t n_cls, const DiskLevels& lv, const DiskPlan& pl, uint32_t* plc,
                      uint32_t* pidx, hipStream_t s) {
  if (pl.C == 0) return hipSuccess;
  if (pl.node_lanes) {
    hipLaunchKernelGGL(k2b_node_lanes, dim3(pl.C, n_cls), dim3(kBlock), 0, s, nodes, n_nodes,
                       pl.chunk, cab, n_cls, lv, plc, pidx);
  } else {
    const uint32_t cb = (n_cls + kBlock * kDiskCPL - 1) / (kBlock * kDiskCPL);
    hipLaunchKernelGGL(k2b_class_lanes<kDiskCPL>, dim3(cb, pl.C), dim3(kBlock), 0, s, nodes,
                       n_nodes, pl.chunk, cab, n_cls, lv, plc, pidx);
  }
  return hipGetLastError();
}

hipError_t launch_reduce2b(const uint32_t* plc, const uint32_t* pidx, uint32_t C, uint32_t n_cls,
                           const uint32_t* cls, uint32_t n_pods, uint32_t node_offset,
                           int64_t* best, uint32_t* idx, uint32_t* ties, int64_t* low,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_reduce2b, pod_grid(n_pods), dim3(kBlock), 0, s, plc, pidx, C, n_cls, cls,
                     n_pods, node_offset, best, idx, ties, low);
  return hipGetLastError();
}

// rows [N][P] (coalesced for the kernels) -> [P][N] (host API layout).
__global__ __launch_bounds__(kBlock) void k_rows_transpose(const int64_t* __restrict__ in,
                                                           uint32_t n_nodes, uint32_t n_pods,
                                                           const uint32_t* __restrict__ perm,
                                                           int64_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (uint64_t)n_nodes * n_pods) return;
  const uint32_t p = (uint32_t)(t / n_nodes), n = (uint32_t)(t % n_nodes);
  const uint32_t q = perm ? perm[p] : p;
  out[(size_t)q * n_nodes + n] = in[(size_t)n * n_pods + p];
}

hipError_t launch_rows_transpose(const int64_t* in, uint32_t n_nodes, uint32_t n_pods,
                                 const uint32_t* perm, int64_t* out, hipStream_t s) {
  const uint64_t total = (uint64_t)n_nodes * n_pods;
  dim3 grid((unsigned)((total + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_rows_transpose, grid, dim3(kBlock), 0, s, in, n_nodes, n_pods, perm,
                     out);
  return hipGetLastError();
}

hipError_t launch_reduce2(const Partials& part, uint32_t C, uint32_t n_pods, bool is_f64,
                          uint32_t node_offset, int64_t* best, uint32_t* idx, uint32_t* ties,
                          int64_t* low, hipStream_t s, const uint64_t* cmask) {
  if (cmask != nullptr && C > kWaveReduceChunks) return hipErrorInvalidValue;
  if (C > kWaveReduceChunks) {
    hipLaunchKernelGGL(k_reduce2_wave, dim3(n_pods), dim3(kWave), 0, s, part.best_f, part.best_i,
                       part.idx, part.ties, part.low_f, part.low_i, C, n_pods, is_f64 ? 1 : 0,
                       node_offset, best, idx, ties, low);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_reduce2, pod_grid(n_pods), dim3(kBlock), 0, s, part.best_f, part.best_i,
                     part.idx, part.ties, part.low_f, part.low_i, C, n_pods, is_f64 ? 1 : 0,
                     node_offset, best, idx, ties, low,
                     reinterpret_cast<const unsigned long long*>(cmask));
  return hipGetLastError();
}

hipError_t launch_merge_prepare(const int64_t* best_global, const int64_t* best_local,
                                uint32_t n_pods, uint32_t* idx, uint32_t* ties, hipStream_t s) {
  hipLaunchKernelGGL(k_merge_prepare, pod_grid(n_pods), dim3(kBlock), 0, s, best_global,
                     best_local, n_pods, idx, ties);
  return hipGetLastError();
}

hipError_t launch_fill_diskio_state(uint32_t n_pods, uint32_t n_nodes, uint64_t* maxima,
                                    uint32_t* counts, hipStream_t s) {
  hipLaunchKernelGGL(k_fill_diskio_state, pod_grid(n_pods), dim3(kBlock), 0, s, n_pods, n_nodes,
                     maxima, counts);
  return hipGetLastError();
}

hipError_t launch_finalize(const uint32_t* counts, const int64_t* best, const uint32_t* idx,
                           const uint32_t* ties_in, const int64_t* lowest, uint32_t n_pods,
                           bool generic, int32_t* pick, int32_t* status, uint32_t* ties_out,
                           uint32_t* flagged, uint32_t* n_flagged, const FinalScatter& sc,
                           hipStream_t s) {
  if (sc.perm && generic) return hipErrorInvalidValue;  // K3 still needs the sorted outputs
  hipLaunchKernelGGL(k_finalize, pod_grid(n_pods), dim3(kBlock), 0, s, counts, best, idx, ties_in,
                     lowest, n_pods, generic ? 1 : 0, pick, status, ties_out, flagged, n_flagged,
                     sc);
  return hipGetLastError();
}

hipError_t launch_k3(int K, const unsigned char* nodes, uint32_t n_nodes, uint32_t chunk_nodes,
                     uint32_t C, const PodParams& pp, const uint64_t* maxima, uint32_t n_pods,
                     const uint64_t* bm, uint32_t bm_stride, const uint32_t* flagged, const uint32_t* n_flagged,
                     const int64_t* best, const int64_t* low, const Partials& part,
                     uint32_t max_flagged, hipStream_t s) {
  dim3 grid((max_flagged + kBlock - 1) / kBlock, C);
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k3_exact_normalize<KK>), grid, dim3(kBlock), 0, s, nodes,
                                      n_nodes, chunk_nodes, pp.m_u, pp.c_u, maxima, n_pods,
                                      bm, bm_stride, flagged, n_flagged, best, low, part.best_i,
                                      part.idx, part.ties, part.err, max_flagged));
  return hipGetLastError();
}

hipError_t launch_reduce3(const Partials& part, uint32_t C, const uint32_t* flagged,
                          const uint32_t* n_flagged, uint32_t max_flagged, uint32_t node_offset,
                          int32_t* pick, int32_t* status, uint32_t* ties, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce3, pod_grid(max_flagged), dim3(kBlock), 0, s, part.best_i, part.idx,
                     part.ties, part.err, C, flagged, n_flagged, max_flagged, node_offset, pick,
                     status, ties);
  return hipGetLastError();
}

hipError_t launch_bitmask_transpose(const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                                    uint32_t bs_stride, const uint64_t* blk, uint32_t blk_stride,
                                    uint32_t n_nodes,
                                    uint32_t W, uint32_t n_pods, const uint32_t* perm,
                                    uint32_t* out, hipStream_t s) {
  const uint64_t total = (uint64_t)W * n_pods;
  dim3 grid((unsigned)((total + kBlock - 1) / kBlock));
  const MaskSrc ms{bm, bs, bm_stride, bs_stride, blk, blk_stride};
  if (bs && !blk) return hipErrorInvalidValue;  // sparse masks are read through their block list
  hipLaunchKernelGGL(k_bitmask_transpose, grid, dim3(kBlock), 0, s, ms, n_nodes, W,
                     n_pods, perm, out);
  return hipGetLastError();
}

// The block K1 with witnesses (one-model N32 snapshots with summaries): sparse masks, blk.
hipError_t launch_k1_block_witness(int K, const unsigned char* nodes, const unsigned char* sum,
                                   const unsigned char* sum2, const unsigned char* mix,
                                   uint32_t n_nodes, uint32_t chunk_nodes, uint32_t C,
                                   const PodParams& pp, uint32_t n_pods, uint64_t* pmax,
                                   uint32_t* pwit, uint32_t* pcnt, uint64_t* bm,
                                   uint32_t bm_stride, BlockMask* bs, uint32_t bs_stride,
                                   uint64_t* blk, uint32_t blk_stride, hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_block_n32<KK, false, false, true>), grid, dim3(kBlock),
                                      0, s, nodes, sum, reinterpret_cast<const uint32_t*>(sum2),
                                      reinterpret_cast<const uint32_t*>(mix), pp.x1, n_nodes,
                                      chunk_nodes, pp.m_32, pp.c_32, pp.number, pp.need_mem,
                                      pp.need_clk, n_pods, pmax, pcnt, bm, bm_stride, bs,
                                      bs_stride, blk, blk_stride, nullptr, pwit, pp.bsum));
  return hipGetLastError();
}

hipError_t launch_k1_witness(int K, Path path, const unsigned char* nodes, uint32_t n_nodes,
                             uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                             uint32_t n_pods, uint64_t* pmax, uint32_t* pwit, uint32_t* pcnt,
                             uint64_t* bm, uint32_t bm_stride, hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  switch (path) {
    case Path::N32:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_witness<KK, Path::N32>), grid, dim3(kBlock), 0, s,
                                          nodes, n_nodes, chunk_nodes, pp.m_32, pp.c_32,
                                          pp.number, pp.need_mem, pp.need_clk, n_pods, pmax, pwit,
                                          pcnt, bm, bm_stride));
      break;
    case Path::F64:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_witness<KK, Path::F64>), grid, dim3(kBlock), 0, s,
                                          nodes, n_nodes, chunk_nodes, pp.m_f, pp.c_f, pp.number,
                                          pp.need_mem, pp.need_clk, n_pods, pmax, pwit, pcnt, bm,
                                          bm_stride));
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Split variant of k_reduce_wit for many chunks: threads = (pod, field) coalesced over pods,
// grid.z splits the chunks.  PHASE 0 folds the maxima (atomicMax) and the feasible counts
// (atomicAdd); PHASE 1, once the maxima are final, adds up the witnesses of the chunks that
// reach a field's maximum and takes their lowest node (atomicMin).  Outputs zeroed before
// (wnode to 0xFFFFFFFF).
template <int PHASE>
__global__ __launch_bounds__(kBlock) void k_reduce_wit_split(
    const uint64_t* __restrict__ pmax, const uint32_t* __restrict__ pwit,
    const uint32_t* __restrict__ pcnt, uint32_t C, uint32_t n_pods, uint32_t node_offset,
    uint64_t* __restrict__ maxima, uint32_t* __restrict__ counts, uint32_t* __restrict__ wcount,
    uint32_t* __restrict__ wnode) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x, f = blockIdx.y;
  if (p >= n_pods) return;
  const uint32_t S = gridDim.z, per = (C + S - 1) / S;
  const uint32_t c0 = blockIdx.z * per, c1 = min(C, c0 + per);
  if (c0 >= c1) return;
  if (PHASE == 0) {
    if (f < 6) {
      uint64_t mx = 0;
      for (uint32_t c = c0; c < c1; ++c) mx = umax64(mx, pmax[((size_t)f * C + c) * n_pods + p]);
      atomicMax(reinterpret_cast<unsigned long long*>(maxima + (size_t)f * n_pods + p),
                (unsigned long long)mx);
    } else {
      uint32_t sum = 0;
      for (uint32_t c = c0; c < c1; ++c) sum += pcnt[((size_t)(f - 6) * C + c) * n_pods + p];
      atomicAdd(counts + (size_t)(f - 6) * n_pods + p, sum);
    }
  } else {
    if (f >= 6) return;
    const uint64_t mx = maxima[(size_t)f * n_pods + p];
    uint32_t wc = 0, wn = 0xffffffffu;
    for (uint32_t c = c0; c < c1; ++c) {
      const size_t o = ((size_t)f * C + c) * n_pods + p;
      if (pmax[o] == mx) {
        wc += pwit[o];
        wn = min(wn, pwit[(size_t)6 * C * n_pods + o]);
      }
    }
    if (wc) atomicAdd(wcount + (size_t)f * n_pods + p, wc);
    if (wn != 0xffffffffu) atomicMin(wnode + (size_t)f * n_pods + p, wn + node_offset);
  }
}

// The split witness reduction's atomic targets, in one launch instead of four fills:
// maxima 0, counts 0, witness counts 0, witness nodes 0xFFFFFFFF.
__global__ __launch_bounds__(kBlock) void k_init_wit(uint64_t* __restrict__ maxima,
                                                     uint32_t* __restrict__ counts,
                                                     uint32_t* __restrict__ wcount,
                                                     uint32_t* __restrict__ wnode,
                                                     uint32_t n_pods) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= 6u * n_pods) return;
  maxima[i] = 0ull;
  wcount[i] = 0u;
  wnode[i] = 0xffffffffu;
  if (i < 2u * n_pods) counts[i] = 0u;
}

hipError_t launch_reduce_wit(const uint64_t* pmax, const uint32_t* pwit, const uint32_t* pcnt,
                             uint32_t C, uint32_t n_pods, uint32_t node_offset, uint64_t* maxima,
                             uint32_t* counts, uint32_t* wcount, uint32_t* wnode, const MemTab& mt,
                             hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  // many chunks (greedy windows: 64-node chunks): the chunk-split two-phase reduction, also
  // for windows under 256 pods (the wave-per-pod kernel below read ~125 KB per pod there:
  // ~88 us a window against ~30)
  if (C > kWaveReduceChunks) {
    const uint32_t pb = (n_pods + kBlock - 1) / kBlock;
    const uint32_t S = std::max<uint32_t>(1, std::min<uint32_t>(C / 16, 256 / pb + 1));
    hipLaunchKernelGGL(k_init_wit, dim3((6 * n_pods + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                       maxima, counts, wcount, wnode, n_pods);
    hipLaunchKernelGGL(k_reduce_wit_split<0>, dim3(pb, 8, S), dim3(kBlock), 0, s, pmax, pwit,
                       pcnt, C, n_pods, node_offset, maxima, counts, wcount, wnode);
    hipLaunchKernelGGL(k_reduce_wit_split<1>, dim3(pb, 6, S), dim3(kBlock), 0, s, pmax, pwit,
                       pcnt, C, n_pods, node_offset, maxima, counts, wcount, wnode);
    if (mt.vf)  // both phases ran in rank space
      hipLaunchKernelGGL(k_rank_maxima, pod_grid(n_pods), dim3(kBlock), 0, s, maxima, n_pods, mt);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_reduce_wit, dim3(n_pods), dim3(kWave), 0, s, pmax, pwit, pcnt, C, n_pods,
                     node_offset, maxima, counts, wcount, wnode, mt);
  return hipGetLastError();
}

// Sharded capacity greedy: after the MAX all-reduce of the maxima, a shard whose own maximum
// of a field is below the global one has no witness of it: zero its count and clear its node
// (then the caller SUM-reduces the counts and MIN-reduces the nodes).
__global__ __launch_bounds__(kBlock) void k_wit_prepare(const uint64_t* __restrict__ gmax,
                                                        const uint64_t* __restrict__ lmax,
                                                        uint32_t n, uint32_t* __restrict__ wit) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  if (lmax[i] != gmax[i]) {
    wit[i] = 0u;
    wit[n + i] = 0xffffffffu;
  }
}

hipError_t launch_wit_prepare(const uint64_t* gmax, const uint64_t* lmax, uint32_t n_pods,
                              uint32_t* wit, hipStream_t s) {
  const uint32_t n = 6u * n_pods;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_wit_prepare, pod_grid(n), dim3(kBlock), 0, s, gmax, lmax, n, wit);
  return hipGetLastError();
}

// Blocks of the k_one_* launches (grid-stride over the nodes).
constexpr uint32_t kOneBlocks = 512;
uint32_t one_blocks() { return kOneBlocks; }

hipError_t launch_one(int K, Path path, const unsigned char* nodes, uint32_t n_nodes,
                      const OnePod& pod, uint64_t* feas, void* part, uint32_t* done,
                      OneOut* out, const MemTab& mt, hipStream_t s) {
  const dim3 grid(std::max<uint32_t>(1, std::min<uint32_t>(kOneBlocks,
                                                           (n_nodes + kBlock - 1) / kBlock)));
  uint64_t* p1 = static_cast<uint64_t*>(part);
  double* p2 = static_cast<double*>(part);
  switch (path) {
    case Path::N32:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k_one_filter<KK, Path::N32>), grid, dim3(kBlock), 0, s,
                                          nodes, n_nodes, pod, feas, p1, done, out, mt);
                    hipLaunchKernelGGL((k_one_score<KK, Path::N32>), grid, dim3(kBlock), 0, s,
                                       nodes, n_nodes, pod, feas, p2, done + 1, out));
      break;
    case Path::F64:
      YODA_K_SWITCH(K, hipLaunchKernelGGL((k_one_filter<KK, Path::F64>), grid, dim3(kBlock), 0, s,
                                          nodes, n_nodes, pod, feas, p1, done, out, MemTab{});
                    hipLaunchKernelGGL((k_one_score<KK, Path::F64>), grid, dim3(kBlock), 0, s,
                                       nodes, n_nodes, pod, feas, p2, done + 1, out));
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// NormalizeScore (scheduler.go:158-183) of the plugin row mode, on the device: for every
// (node, pod) of rows [N][P] (the raw Score, -1 where Filter failed), over the pod's feasible
// nodes: highest = max(0, max raw) (init 0, :162), lowest = min raw (init the first score,
// :163), lowest-- when equal (:173-175), norm = (raw - lowest) * 100 / (highest - lowest) in
// Go's int64 arithmetic (wrapping multiply, truncating divide, :178).  best / lowest come
// from the row-mode K2's reduction (same pod order as rows).  -1 where Filter failed.
__global__ __launch_bounds__(kBlock) void k_norm_rows(const int64_t* __restrict__ rows,
                                                      uint32_t n_nodes, uint32_t n_pods,
                                                      const int64_t* __restrict__ best,
                                                      const int64_t* __restrict__ lowest,
                                                      int64_t* __restrict__ norm) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (uint64_t)n_nodes * n_pods) return;
  const uint32_t p = (uint32_t)(t % n_pods);
  const int64_t s = rows[t];
  if (s < 0) {
    norm[t] = -1;
    return;
  }
  const int64_t h = best[p] > 0 ? best[p] : 0;
  int64_t l = lowest[p];
  if (h == l) --l;
  norm[t] = (int64_t)((uint64_t)(s - l) * 100u) / (h - l);
}

hipError_t launch_norm_rows(const int64_t* rows, uint32_t n_nodes, uint32_t n_pods,
                            const int64_t* best, const int64_t* lowest, int64_t* norm,
                            hipStream_t s) {
  const uint64_t total = (uint64_t)n_nodes * n_pods;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_norm_rows, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     s, rows, n_nodes, n_pods, best, lowest, norm);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_pack_rec(const int64_t* __restrict__ best,
                                                     const uint32_t* __restrict__ idx,
                                                     const uint32_t* __restrict__ ties,
                                                     const int64_t* __restrict__ low,
                                                     uint32_t n_pods, ShardRec* __restrict__ rec) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  rec[p] = ShardRec{best[p], idx[p], ties[p], low[p]};
}

// Fold the ranks' records of each pod: the highest best, the lowest node reaching it, the
// tie counts of the ranks reaching it summed, the lowest low (the merges of merge_phase2).
__global__ __launch_bounds__(kBlock) void k_merge_rec(const ShardRec* __restrict__ all,
                                                      uint32_t n_pods, uint32_t world,
                                                      int64_t* __restrict__ best,
                                                      uint32_t* __restrict__ idx,
                                                      uint32_t* __restrict__ ties,
                                                      int64_t* __restrict__ low) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  int64_t b = -1, l = kI64Max;
  uint32_t i = 0xffffffffu, t = 0;
  for (uint32_t r = 0; r < world; ++r) {
    const ShardRec x = all[(size_t)r * n_pods + p];
    l = x.low < l ? x.low : l;
    if (x.best < 0) continue;
    if (x.best > b) {
      b = x.best;
      i = x.idx;
      t = x.ties;
    } else if (x.best == b) {
      i = min(i, x.idx);
      t += x.ties;
    }
  }
  best[p] = b;
  idx[p] = i;
  ties[p] = t;
  low[p] = l;
}

// In-process exchange (several shard handles on one device): elementwise MAX of n u64 over
// the handles' buffers into dst.
__global__ __launch_bounds__(kBlock) void k_max_multi(PtrList src, uint32_t k, uint64_t n,
                                                      uint64_t* __restrict__ dst) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= n) return;
  uint64_t m = 0;
  for (uint32_t j = 0; j < k; ++j) m = umax64(m, static_cast<const uint64_t*>(src.p[j])[t]);
  dst[t] = m;
}

hipError_t launch_pack_rec(const int64_t* best, const uint32_t* idx, const uint32_t* ties,
                           const int64_t* low, uint32_t n_pods, ShardRec* rec, hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_rec, pod_grid(n_pods), dim3(kBlock), 0, s, best, idx, ties, low,
                     n_pods, rec);
  return hipGetLastError();
}

hipError_t launch_merge_rec(const ShardRec* all, uint32_t n_pods, uint32_t world, int64_t* best,
                            uint32_t* idx, uint32_t* ties, int64_t* low, hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge_rec, pod_grid(n_pods), dim3(kBlock), 0, s, all, n_pods, world, best,
                     idx, ties, low);
  return hipGetLastError();
}

// In-process exchange: elementwise SUM of n u32 over the handles' buffers into dst.
__global__ __launch_bounds__(kBlock) void k_sum_multi_u32(PtrList src, uint32_t k, uint64_t n,
                                                          uint32_t* __restrict__ dst) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= n) return;
  uint32_t a = 0;
  for (uint32_t j = 0; j < k; ++j) a += static_cast<const uint32_t*>(src.p[j])[t];
  dst[t] = a;
}

// Packed-key merge of the sharded phase 2 (fast record paths): each shard's
// (best score, lowest node reaching it) as one u64  best << ib | (2^ib - 1 - node)  (0: none),
// MAX-reduced across the shards; then every shard reads the winner back and keeps its tie
// count only if it holds the winning score (SUM-reduced after).  lowest := the winning score
// (only the U64 path's normalize check reads it, and that path keeps the record merge).
__global__ __launch_bounds__(kBlock) void k_pack_key(const int64_t* __restrict__ best,
                                                     const uint32_t* __restrict__ idx,
                                                     uint32_t n_pods, uint32_t ib,
                                                     uint64_t* __restrict__ key) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const uint64_t imax = (1ull << ib) - 1ull;
  key[p] = best[p] < 0 ? 0ull : ((uint64_t)best[p] << ib) | (imax - (uint64_t)idx[p]);
}

__global__ __launch_bounds__(kBlock) void k_unpack_key(const uint64_t* __restrict__ key,
                                                       uint32_t n_pods, uint32_t ib,
                                                       int64_t* __restrict__ best,
                                                       uint32_t* __restrict__ idx,
                                                       uint32_t* __restrict__ ties,
                                                       int64_t* __restrict__ low) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const uint64_t imax = (1ull << ib) - 1ull, k = key[p];
  const int64_t bg = k ? (int64_t)(k >> ib) : -1;
  ties[p] = (k && best[p] == bg) ? ties[p] : 0u;
  best[p] = bg;
  idx[p] = k ? (uint32_t)(imax - (k & imax)) : 0xffffffffu;
  low[p] = bg;
}

hipError_t launch_sum_multi_u32(const PtrList& src, uint32_t k, uint64_t n, uint32_t* dst,
                                hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sum_multi_u32, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock),
                     0, s, src, k, n, dst);
  return hipGetLastError();
}

hipError_t launch_pack_key(const int64_t* best, const uint32_t* idx, uint32_t n_pods, uint32_t ib,
                           uint64_t* key, hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_key, pod_grid(n_pods), dim3(kBlock), 0, s, best, idx, n_pods, ib, key);
  return hipGetLastError();
}

hipError_t launch_unpack_key(const uint64_t* key, uint32_t n_pods, uint32_t ib, int64_t* best,
                             uint32_t* idx, uint32_t* ties, int64_t* low, hipStream_t s) {
  if (n_pods == 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_key, pod_grid(n_pods), dim3(kBlock), 0, s, key, n_pods, ib, best,
                     idx, ties, low);
  return hipGetLastError();
}

hipError_t launch_max_multi(const PtrList& src, uint32_t k, uint64_t n, uint64_t* dst,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_max_multi, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     src, k, n, dst);
  return hipGetLastError();
}

}  // namespace yoda
