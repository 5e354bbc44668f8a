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

#include "yoda_layout.h"

#pragma clang fp contract(off)

namespace yoda {

constexpr int64_t kI64Max = 0x7fffffffffffffffll;

template <bool Fast>
struct Num;
template <>
struct Num<true> {
  using T = double;
  using Hdr = NodeHdrF;
};
template <>
struct Num<false> {
  using T = uint64_t;
  using Hdr = NodeHdrG;
};

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// ---------------------------------------------------------------------------------------
// K1: Filter (PodFitsNumber ∧ PodFitsMemory ∧ PodFitsClock, collection.go:41-44) and the
// PreScore maxima (CollectMaxValues).  Writes the feasibility bitmask [W][P] and per-chunk
// partials.
template <int K, bool Fast>
__global__ __launch_bounds__(kBlock) void k1_filter_maxima(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const double* __restrict__ m_f, const double* __restrict__ c_f,
    const uint64_t* __restrict__ m_u, const uint64_t* __restrict__ c_u,
    const uint64_t* __restrict__ number_in, const uint32_t* __restrict__ need_mem_in,
    const uint32_t* __restrict__ need_clk_in, uint32_t n_pods, double* __restrict__ pmax_f,
    uint64_t* __restrict__ pmax_u, uint32_t* __restrict__ pcnt, uint32_t* __restrict__ bitmask) {
  using T = typename Num<Fast>::T;
  using Hdr = typename Num<Fast>::Hdr;
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t chunk = blockIdx.y, C = gridDim.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;

  T m = 0, c = 0;
  uint64_t number = ~0ull;  // padding lanes never fit
  uint32_t need_mem = 0, need_clk = 0;
  if (live) {
    if constexpr (Fast) {
      m = m_f[p];
      c = c_f[p];
    } else {
      m = m_u[p];
      c = c_u[p];
    }
    number = number_in[p];
    need_mem = need_mem_in[p];
    need_clk = need_clk_in[p];
  }
  T mx[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) mx[f] = T(1);  // floor 1 (collection.go:31-38)
  uint32_t nf = 0, nz = 0, bits = 0;

  for (uint32_t n = n0; n < n1; ++n) {
    const unsigned char* rec = nodes + (size_t)n * node_stride(K);
    const Hdr* h = reinterpret_cast<const Hdr*>(rec);
    const T* fld = reinterpret_cast<const T*>(rec + sizeof(Hdr));
    const uint32_t hm = h->healthy_mask;
    uint32_t cm = 0, cc = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const bool hj = (hm >> j) & 1u;
      cm += (hj && fld[kFree * K + j] >= m) ? 1u : 0u;   // CardFitsMemory (filter.go:52-54)
      cc += (hj && fld[kClock * K + j] == c) ? 1u : 0u;  // CardFitsClock  (filter.go:56-58)
    }
    const bool feas = (number <= h->card_number) && cm >= need_mem && cc >= need_clk;
    bits |= (uint32_t)feas << (n & 31u);
    if (feas) {
      ++nf;
      nz += h->zero_total;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const T fr = fld[kFree * K + j], ck = fld[kClock * K + j];
        if (fr >= m && ck >= c) {  // collection.go:46: no health check, >= clock
          if constexpr (Fast) {
            mx[kMaxBw] = fmax(mx[kMaxBw], fld[kBandwidth * K + j]);
            mx[kMaxClock] = fmax(mx[kMaxClock], ck);
            mx[kMaxCore] = fmax(mx[kMaxCore], fld[kCore * K + j]);
            mx[kMaxFree] = fmax(mx[kMaxFree], fr);
            mx[kMaxPower] = fmax(mx[kMaxPower], fld[kPower * K + j]);
            mx[kMaxTotal] = fmax(mx[kMaxTotal], fld[kTotal * K + j]);
          } else {
            mx[kMaxBw] = umax64(mx[kMaxBw], fld[kBandwidth * K + j]);
            mx[kMaxClock] = umax64(mx[kMaxClock], ck);
            mx[kMaxCore] = umax64(mx[kMaxCore], fld[kCore * K + j]);
            mx[kMaxFree] = umax64(mx[kMaxFree], fr);
            mx[kMaxPower] = umax64(mx[kMaxPower], fld[kPower * K + j]);
            mx[kMaxTotal] = umax64(mx[kMaxTotal], fld[kTotal * K + j]);
          }
        }
      }
    }
    if ((n & 31u) == 31u || n + 1 == n1) {
      if (live) bitmask[(size_t)(n >> 5) * n_pods + p] = bits;
      bits = 0;
    }
  }
  if (!live) return;
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    const size_t o = ((size_t)f * C + chunk) * n_pods + p;
    if constexpr (Fast)
      pmax_f[o] = mx[f];
    else
      pmax_u[o] = mx[f];
  }
  pcnt[((size_t)0 * C + chunk) * n_pods + p] = nf;
  pcnt[((size_t)1 * C + chunk) * n_pods + p] = nz;
}

// Per-pod merge of K1 chunk partials -> maxima [6][P] (u64) and counts [2][P].
__global__ __launch_bounds__(kBlock) void k_reduce1(const double* __restrict__ pmax_f,
                                                    const uint64_t* __restrict__ pmax_u,
                                                    const uint32_t* __restrict__ pcnt, uint32_t C,
                                                    uint32_t n_pods, int fast,
                                                    uint64_t* __restrict__ maxima,
                                                    uint32_t* __restrict__ counts) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  for (int f = 0; f < 6; ++f) {
    uint64_t mx = 1;
    for (uint32_t c = 0; c < C; ++c) {
      const size_t o = ((size_t)f * C + c) * n_pods + p;
      mx = umax64(mx, fast ? (uint64_t)pmax_f[o] : pmax_u[o]);
    }
    maxima[(size_t)f * n_pods + p] = mx;
  }
  for (int f = 0; f < 2; ++f) {
    uint32_t s = 0;
    for (uint32_t c = 0; c < C; ++c) s += pcnt[((size_t)f * C + c) * n_pods + p];
    counts[(size_t)f * n_pods + p] = s;
  }
}

// RU(100 / M): the smallest double >= 100/M.  With every card field <= 2^44,
// floor(x * RU(100/M)) == floor(100 x / M) exactly.
__device__ __forceinline__ double ru_100_over(double M) {
  double r = 100.0 / M;  // IEEE round-to-nearest
  const double e = __builtin_fma(r, M, -100.0);  // exact sign of r*M - 100
  if (e < 0.0) r = __longlong_as_double(__double_as_longlong(r) + 1);
  return r;
}

// Fast path: per-pod reciprocals of the (all-reduced) maxima.
__global__ __launch_bounds__(kBlock) void k_prep2(const uint64_t* __restrict__ maxima,
                                                  uint32_t n_pods, double* __restrict__ rcp) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const int src[5] = {kMaxBw, kMaxCore, kMaxPower, kMaxFree, kMaxTotal};
#pragma unroll
  for (int k = 0; k < 5; ++k)
    rcp[(size_t)k * n_pods + p] = ru_100_over((double)maxima[(size_t)src[k] * n_pods + p]);
}

// ---------------------------------------------------------------------------------------
// K2 fast path: CalculateBasicScore + Allocate + Actual in exact f64, running argmax with
// lowest-index ties, tie count and min over the feasible nodes of the chunk.
template <int K>
__global__ __launch_bounds__(kBlock) void k2_score_fast(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const double* __restrict__ m_f, const double* __restrict__ c_f,
    const double* __restrict__ rcp, uint32_t n_pods, const uint32_t* __restrict__ bitmask,
    double* __restrict__ pbest, uint32_t* __restrict__ pidx, uint32_t* __restrict__ pties,
    double* __restrict__ plow) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t chunk = blockIdx.y;
  const uint32_t n0 = chunk * chunk_nodes;
  const uint32_t n1 = min(n0 + chunk_nodes, n_nodes);
  const bool live = p < n_pods;
  double m = 0, c = 0, r_bw = 0, r_core = 0, r_pow = 0, r_free = 0, r_tot = 0;
  if (live) {
    m = m_f[p];
    c = c_f[p];
    r_bw = rcp[0 * (size_t)n_pods + p];
    r_core = rcp[1 * (size_t)n_pods + p];
    r_pow = rcp[2 * (size_t)n_pods + p];
    r_free = rcp[3 * (size_t)n_pods + p];
    r_tot = rcp[4 * (size_t)n_pods + p];
  }
  double best = -1.0, low = 1.0e300;
  uint32_t idx = 0xffffffffu, ties = 0, word = 0;
  for (uint32_t n = n0; n < n1; ++n) {
    if ((n & 31u) == 0u) word = live ? bitmask[(size_t)(n >> 5) * n_pods + p] : 0u;
    const bool feas = (word >> (n & 31u)) & 1u;
    if (feas) {
      const unsigned char* rec = nodes + (size_t)n * node_stride(K);
      const NodeHdrF* h = reinterpret_cast<const NodeHdrF*>(rec);
      const double* fld = reinterpret_cast<const double*>(rec + sizeof(NodeHdrF));
      double basic = 0.0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const double fr = fld[kFree * K + j], ck = fld[kClock * K + j];
        if (fr >= m && ck >= c) {  // algorithm.go:271
          // CalculateCardScore (algorithm.go:280-291): each quotient truncates before its
          // weight; clock is divided by MaxBandwidth (:283).
          double s = __builtin_trunc(fld[kBandwidth * K + j] * r_bw);
          s += __builtin_trunc(ck * r_bw);
          s += 2.0 * __builtin_trunc(fld[kCore * K + j] * r_core);
          s += __builtin_trunc(fld[kPower * K + j] * r_pow);
          s += 3.0 * __builtin_trunc(fr * r_free);
          s += __builtin_trunc(fld[kTotal * K + j] * r_tot);
          basic += s;
        }
      }
      const double raw = basic + h->static_score;  // algorithm.go:96
      if (raw > best) {
        best = raw;
        idx = n;
        ties = 1;
      } else if (raw == best) {
        ++ties;
      }
      low = fmin(low, raw);
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

template <int K>
__global__ __launch_bounds__(kBlock) void k2_score_generic(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const uint64_t* __restrict__ m_u, const uint64_t* __restrict__ c_u,
    const uint64_t* __restrict__ maxima, uint32_t n_pods, const uint32_t* __restrict__ bitmask,
    int64_t* __restrict__ pbest, uint32_t* __restrict__ pidx, uint32_t* __restrict__ pties,
    int64_t* __restrict__ plow) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t chunk = blockIdx.y;
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
  uint32_t idx = 0xffffffffu, ties = 0, word = 0;
  for (uint32_t n = n0; n < n1; ++n) {
    if ((n & 31u) == 0u) word = live ? bitmask[(size_t)(n >> 5) * n_pods + p] : 0u;
    if ((word >> (n & 31u)) & 1u) {
      const int64_t s = raw_score_u64<K>(nodes + (size_t)n * node_stride(K), m, c, M);
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
__global__ __launch_bounds__(kBlock) void k2_diskio(const NodeRecB* __restrict__ nodes,
                                                    uint32_t n_nodes, uint32_t chunk_nodes,
                                                    const double* __restrict__ alpha_in,
                                                    const double* __restrict__ beta_in,
                                                    uint32_t n_pods, double* __restrict__ pbest,
                                                    uint32_t* __restrict__ pidx,
                                                    uint32_t* __restrict__ pties,
                                                    double* __restrict__ plow) {
#pragma clang fp contract(off)
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t chunk = blockIdx.y;
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
                                                    int64_t* __restrict__ low_out) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  int64_t best = -1, low = kI64Max;
  uint32_t idx = 0xffffffffu, ties = 0;
  for (uint32_t c = 0; c < C; ++c) {
    const size_t o = (size_t)c * n_pods + p;
    int64_t b, l;
    if (is_f64) {
      const double bf = pbest_f[o], lf = plow_f[o];
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
    }
    low = l < low ? l : low;
  }
  best_out[p] = best;
  idx_out[p] = idx == 0xffffffffu ? idx : idx + node_offset;
  ties_out[p] = ties;
  low_out[p] = low;
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
                                                     uint32_t* __restrict__ n_flagged) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  const uint32_t nf = counts[p], nz = counts[(size_t)n_pods + p];
  uint32_t t = ties_io[p];
  if (nf == 0) {
    pick[p] = -1;
    status[p] = 1;
    t = 0;
  } else if (nf == 1) {  // k8s: the only feasible node is returned without scoring
    pick[p] = (int32_t)idx[p];
    status[p] = 0;
    t = 1;
  } else if (nz > 0) {  // Score would divide by TotalMemorySum == 0: Go panics
    pick[p] = -2;
    status[p] = 2;
    t = 0;
  } else {
    const int64_t h = best[p];
    int64_t l = lowest[p];
    if (h == l) --l;  // scheduler.go:173-175
    if (generic && (uint64_t)(h - l) > (uint64_t)(kI64Max / 100)) {
      pick[p] = -3;  // pending: exact normalize (K3)
      status[p] = -1;
      flagged[atomicAdd(n_flagged, 1u)] = p;
    } else {
      pick[p] = (int32_t)idx[p];
      status[p] = 0;
    }
  }
  ties_out[p] = t;
}

// ---------------------------------------------------------------------------------------
// K3 (generic path, rare): NormalizeScore with Go's int64 wrap-around for pods whose
// (highest - lowest) * 100 can overflow, then the k8s range check and selectHost.  One lane
// per flagged pod.
template <int K>
__global__ __launch_bounds__(kBlock) void k3_exact_normalize(
    const unsigned char* __restrict__ nodes, uint32_t n_nodes, uint32_t chunk_nodes,
    const uint64_t* __restrict__ m_u, const uint64_t* __restrict__ c_u,
    const uint64_t* __restrict__ maxima, uint32_t n_pods, const uint32_t* __restrict__ bitmask,
    const uint32_t* __restrict__ flagged, const uint32_t* __restrict__ n_flagged_p,
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
    const uint32_t word = bitmask[(size_t)(n >> 5) * n_pods + p];
    if (!((word >> (n & 31u)) & 1u)) continue;
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

// Bitmask [W][P] (device, coalesced for the kernels) -> [P][W] (host API layout).
__global__ __launch_bounds__(kBlock) void k_bitmask_transpose(const uint32_t* __restrict__ in,
                                                              uint32_t W, uint32_t n_pods,
                                                              uint32_t* __restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (uint64_t)W * n_pods) return;
  const uint32_t p = (uint32_t)(t / W), w = (uint32_t)(t % W);
  out[t] = in[(size_t)w * n_pods + p];
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

static inline dim3 pod_grid(uint32_t n) { return dim3((n + kBlock - 1) / kBlock); }

hipError_t launch_k1(int K, bool fast, const unsigned char* nodes, uint32_t n_nodes,
                     uint32_t chunk_nodes, uint32_t C, const PodParams& pp, uint32_t n_pods,
                     const Partials& part, uint32_t* bitmask, hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  if (fast) {
    YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_filter_maxima<KK, true>), grid, dim3(kBlock), 0, s,
                                        nodes, n_nodes, chunk_nodes, pp.m_f, pp.c_f, pp.m_u,
                                        pp.c_u, pp.number, pp.need_mem, pp.need_clk, n_pods,
                                        part.max_f, part.max_u, part.cnt, bitmask));
  } else {
    YODA_K_SWITCH(K, hipLaunchKernelGGL((k1_filter_maxima<KK, false>), grid, dim3(kBlock), 0, s,
                                        nodes, n_nodes, chunk_nodes, pp.m_f, pp.c_f, pp.m_u,
                                        pp.c_u, pp.number, pp.need_mem, pp.need_clk, n_pods,
                                        part.max_f, part.max_u, part.cnt, bitmask));
  }
  return hipGetLastError();
}

hipError_t launch_reduce1(const Partials& part, uint32_t C, uint32_t n_pods, bool fast,
                          uint64_t* maxima, uint32_t* counts, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce1, pod_grid(n_pods), dim3(kBlock), 0, s, part.max_f, part.max_u,
                     part.cnt, C, n_pods, fast ? 1 : 0, maxima, counts);
  return hipGetLastError();
}

hipError_t launch_prep2(const uint64_t* maxima, uint32_t n_pods, double* rcp, hipStream_t s) {
  hipLaunchKernelGGL(k_prep2, pod_grid(n_pods), dim3(kBlock), 0, s, maxima, n_pods, rcp);
  return hipGetLastError();
}

hipError_t launch_k2(int K, bool fast, const unsigned char* nodes, uint32_t n_nodes,
                     uint32_t chunk_nodes, uint32_t C, const PodParams& pp, const uint64_t* maxima,
                     const double* rcp, uint32_t n_pods, const uint32_t* bitmask,
                     const Partials& part, hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  if (fast) {
    YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_score_fast<KK>), grid, dim3(kBlock), 0, s, nodes,
                                        n_nodes, chunk_nodes, pp.m_f, pp.c_f, rcp, n_pods,
                                        bitmask, part.best_f, part.idx, part.ties, part.low_f));
  } else {
    YODA_K_SWITCH(K, hipLaunchKernelGGL((k2_score_generic<KK>), grid, dim3(kBlock), 0, s, nodes,
                                        n_nodes, chunk_nodes, pp.m_u, pp.c_u, maxima, n_pods,
                                        bitmask, part.best_i, part.idx, part.ties, part.low_i));
  }
  return hipGetLastError();
}

hipError_t launch_k2_diskio(const NodeRecB* nodes, uint32_t n_nodes, uint32_t chunk_nodes,
                            uint32_t C, const PodParams& pp, uint32_t n_pods, const Partials& part,
                            hipStream_t s) {
  dim3 grid((n_pods + kBlock - 1) / kBlock, C);
  hipLaunchKernelGGL(k2_diskio, grid, dim3(kBlock), 0, s, nodes, n_nodes, chunk_nodes, pp.alpha,
                     pp.beta, n_pods, part.best_f, part.idx, part.ties, part.low_f);
  return hipGetLastError();
}

hipError_t launch_reduce2(const Partials& part, uint32_t C, uint32_t n_pods, bool is_f64,
                          uint32_t node_offset, int64_t* best, uint32_t* idx, uint32_t* ties,
                          int64_t* low, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce2, pod_grid(n_pods), dim3(kBlock), 0, s, part.best_f, part.best_i,
                     part.idx, part.ties, part.low_f, part.low_i, C, n_pods, is_f64 ? 1 : 0,
                     node_offset, best, idx, ties, low);
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
                           uint32_t* flagged, uint32_t* n_flagged, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, pod_grid(n_pods), dim3(kBlock), 0, s, counts, best, idx, ties_in,
                     lowest, n_pods, generic ? 1 : 0, pick, status, ties_out, flagged, n_flagged);
  return hipGetLastError();
}

hipError_t launch_k3(int K, const unsigned char* nodes, uint32_t n_nodes, uint32_t chunk_nodes,
                     uint32_t C, const PodParams& pp, const uint64_t* maxima, uint32_t n_pods,
                     const uint32_t* bitmask, const uint32_t* flagged, const uint32_t* n_flagged,
                     const int64_t* best, const int64_t* low, const Partials& part,
                     uint32_t max_flagged, hipStream_t s) {
  dim3 grid((max_flagged + kBlock - 1) / kBlock, C);
  YODA_K_SWITCH(K, hipLaunchKernelGGL((k3_exact_normalize<KK>), grid, dim3(kBlock), 0, s, nodes,
                                      n_nodes, chunk_nodes, pp.m_u, pp.c_u, maxima, n_pods,
                                      bitmask, flagged, n_flagged, best, low, part.best_i,
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

hipError_t launch_bitmask_transpose(const uint32_t* in, uint32_t W, uint32_t n_pods,
                                    uint32_t* out, hipStream_t s) {
  const uint64_t total = (uint64_t)W * n_pods;
  dim3 grid((unsigned)((total + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_bitmask_transpose, grid, dim3(kBlock), 0, s, in, W, n_pods, out);
  return hipGetLastError();
}

}  // namespace yoda
