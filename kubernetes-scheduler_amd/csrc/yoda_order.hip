// yoda_order.hip — batch pod ordering for the independent-cycle paths.
//
// The pods of a batch are independent scheduling cycles (the reference runs one
// scheduleOne per pod), so the kernels may visit them in any order.  K1 and K2 map lane =
// pod and skip a node when no lane of the wave is feasible on it; a random batch keeps
// every wave busy on every node.  Sorting the batch by the Filter's inputs (clock, number,
// memory) groups pods that fail together, so whole waves skip: ~43% of (wave, node) pairs
// stay busy on config 3 instead of 100%.  The permutation is
// computed on the device inside every run (its cost is in the measured step), the pod
// arrays are gathered into sorted order, and every per-pod output is scattered back before
// it leaves the library — results do not depend on the order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

#include "yoda_layout.h"

namespace yoda {

// key = clock (clamped to 24 bits) | number (8 bits) | has-memory (1 bit) | memory (32
// bits), lexicographic: ascending clock puts the K1 `clock >= c` skips together too.  Any
// key is correct; this one is just fast.  The fields are packed at the widths the batch
// actually uses (host: the OR of each clamped field at upload), so the radix sort runs over
// bc + bn + 1 + bm bits only -- same order as the full-width key, fewer passes.  (Without
// room for the has-memory bit in 64, it is left out.)
//
// Serpentine: memory ascends in the even (clock, number, has-memory) groups and descends in
// the odd ones (rank among the batch's groups, host-built sorted list `groups`).  A wave
// that straddles two groups then holds pods of similar memory from both ends instead of the
// largest requests of one group next to the smallest of the next: its pods qualify the
// same cards on most nodes, where a straddling ascending wave spans every memory size and
// leaves the block K2 nothing but per-pod work.
struct KeyShape {
  uint32_t bm, f_shift, n_shift, c_shift;  // field positions; f_shift == 64: no flag bit
};

// m32 (memory ranks, yoda_layout.h MemTab): the pods' rank thresholds, monotone in scv/memory,
// stand in for the 32-bit clamp of the value.
__device__ __forceinline__ uint64_t order_key(uint64_t number, uint64_t m_u, uint64_t c_u,
                                              uint32_t need_mem, KeyShape k,
                                              const uint64_t* __restrict__ groups,
                                              uint32_t n_groups, const uint32_t* m32, uint32_t p) {
  const uint64_t c = c_u < 0xffffffull ? c_u : 0xffffffull;
  const uint64_t n = number < 0xffull ? number : 0xffull;
  const uint64_t f = need_mem != 0u ? 1ull : 0ull;
  uint64_t m = m32 ? (uint64_t)m32[p] : (m_u < 0xffffffffull ? m_u : 0xffffffffull);
  if (groups) {
    const uint64_t g = (c << 9) | (n << 1) | f;
    uint32_t lo = 0, hi = n_groups;  // lower_bound: the group's rank
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (groups[mid] < g) lo = mid + 1; else hi = mid;
    }
    const uint64_t m_all = k.bm >= 32 ? 0xffffffffull : (1ull << k.bm) - 1ull;
    if (lo & 1u) m = m_all - m;  // m <= m_all: bm is the width of the batch's m field
  }
  return (c << k.c_shift) | (n << k.n_shift) | (k.f_shift < 64 ? f << k.f_shift : 0ull) | m;
}

__global__ __launch_bounds__(kBlock) void k_order_keys(const uint64_t* __restrict__ number,
                                                       const uint64_t* __restrict__ m_u,
                                                       const uint64_t* __restrict__ c_u,
                                                       const uint32_t* __restrict__ need_mem,
                                                       uint32_t n_pods, KeyShape k,
                                                       const uint64_t* __restrict__ groups,
                                                       uint32_t n_groups,
                                                       uint64_t* __restrict__ keys,
                                                       uint32_t* __restrict__ idx,
                                                       const uint32_t* __restrict__ m32) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  keys[p] = order_key(number[p], m_u[p], c_u[p], need_mem[p], k, groups, n_groups, m32, p);
  idx[p] = p;
}

// The same key when it fits 32 bits (the usual case: clock < 2^11, number < 2^4, memory in
// MiB < 2^17): half the bytes per radix pass.
__global__ __launch_bounds__(kBlock) void k_order_keys32(const uint64_t* __restrict__ number,
                                                         const uint64_t* __restrict__ m_u,
                                                         const uint64_t* __restrict__ c_u,
                                                         const uint32_t* __restrict__ need_mem,
                                                         uint32_t n_pods, KeyShape k,
                                                         const uint64_t* __restrict__ groups,
                                                         uint32_t n_groups,
                                                         uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ idx,
                                                         const uint32_t* __restrict__ m32) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  keys[p] = (uint32_t)order_key(number[p], m_u[p], c_u[p], need_mem[p], k, groups, n_groups,
                                m32, p);
  idx[p] = p;
}

// gather (dst[i] = src[perm[i]]) or scatter (dst[perm[i]] = src[i]) of up to kPermArrays
// per-pod arrays of 4 or 8 bytes; grid.y = array.
__global__ __launch_bounds__(kBlock) void k_permute(PermTable t, const uint32_t* __restrict__ perm,
                                                    uint32_t n_pods, int scatter) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t a = blockIdx.y;
  if (i >= n_pods || a >= t.n) return;
  const uint32_t j = perm[i];
  const uint32_t s = scatter ? i : j, d = scatter ? j : i;
  if (t.bytes[a] == 8)
    static_cast<uint64_t*>(t.dst[a])[d] = static_cast<const uint64_t*>(t.src[a])[s];
  else
    static_cast<uint32_t*>(t.dst[a])[d] = static_cast<const uint32_t*>(t.src[a])[s];
}

// Scratch for the sort: keys[2][P] u64, idx[2][P] u32, then hipcub's temp storage.
size_t order_scratch_bytes(uint32_t n_pods) {
  size_t temp = 0, temp32 = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const uint64_t*)nullptr,
                                           (uint64_t*)nullptr, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)n_pods);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp32, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)n_pods);
  return 16ull * n_pods + 8ull * n_pods + 256 + (temp > temp32 ? temp : temp32);
}

// perm[i] = the original index of the i-th pod in sorted order.
hipError_t launch_order_pods(const uint64_t* number, const uint64_t* m_u, const uint64_t* c_u,
                             const uint32_t* need_mem, uint32_t n_pods, const uint32_t key_bits[3],
                             const uint64_t* groups, uint32_t n_groups, void* scratch,
                             size_t scratch_bytes, uint32_t* perm, const uint32_t* m32,
                             hipStream_t s) {
  // key_bits = widths of (c, n, m); each <= its clamp (24, 8, 32)
  const uint32_t bc = key_bits[0] < 24 ? key_bits[0] : 24;
  const uint32_t bn = key_bits[1] < 8 ? key_bits[1] : 8;
  const uint32_t bm = key_bits[2] < 32 ? key_bits[2] : 32;
  const bool flag = bc + bn + 1 + bm <= 64;
  KeyShape k;
  k.bm = bm;
  k.f_shift = flag ? bm : 64;
  k.n_shift = bm + (flag ? 1 : 0);
  k.c_shift = k.n_shift + bn;
  const uint32_t bits = k.c_shift + bc;
  const int end_bit = bits > 0 ? (int)bits : 1;
  unsigned char* b = static_cast<unsigned char*>(scratch);
  uint64_t* keys_in = reinterpret_cast<uint64_t*>(b);
  uint64_t* keys_out = keys_in + n_pods;
  uint32_t* idx_in = reinterpret_cast<uint32_t*>(keys_out + n_pods);
  unsigned char* temp = b + ((16ull * n_pods + 4ull * n_pods + 255) / 256 * 256);
  size_t temp_bytes = scratch_bytes - (size_t)(temp - b);
  if (end_bit <= 32) {
    uint32_t* k32_in = reinterpret_cast<uint32_t*>(keys_in);
    uint32_t* k32_out = reinterpret_cast<uint32_t*>(keys_out);
    hipLaunchKernelGGL(k_order_keys32, dim3((n_pods + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                       number, m_u, c_u, need_mem, n_pods, k, groups, n_groups, k32_in, idx_in, m32);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k32_in, k32_out, idx_in, perm,
                                              (int)n_pods, 0, end_bit, s);
  }
  hipLaunchKernelGGL(k_order_keys, dim3((n_pods + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                     number, m_u, c_u, need_mem, n_pods, k, groups, n_groups, keys_in, idx_in, m32);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, idx_in, perm,
                                            (int)n_pods, 0, end_bit, s);
}

hipError_t launch_permute(const PermTable& t, const uint32_t* perm, uint32_t n_pods, bool scatter,
                          hipStream_t s) {
  if (t.n == 0 || n_pods == 0) return hipSuccess;
  dim3 grid((n_pods + kBlock - 1) / kBlock, t.n);
  hipLaunchKernelGGL(k_permute, grid, dim3(kBlock), 0, s, t, perm, n_pods, scatter ? 1 : 0);
  return hipGetLastError();
}

// ---- counting-sort order with group padding ------------------------------------------
// The batch's pods fall into a few (clock, number, has-memory) groups (host: the distinct
// group keys, ascending, and each group's first sorted position).  Within a group the pods
// are ordered by memory in NB buckets, ascending in even groups and descending in odd ones
// (serpentine, as above); the order inside one bucket is whatever the atomics give (any
// order is correct, results do not depend on it).  With padding every group starts on a
// wave boundary: the free slots at a group's end are filled with copies of its last pod
// (a sorted position that maps to the same caller pod: identical inputs, identical
// results, written back twice), so no wave mixes two groups -- a mixed wave leaves the
// block kernels nothing but per-pod work on every node.
// (m32 / c32: scv/memory / scv/clock clamped to 32 bits -- or the memory rank -- whose 32- and
// 24-bit clamps below equal those of the 64-bit labels: the counting order reads only the pod
// arrays the block kernels read)
__device__ __forceinline__ uint32_t order_bucket(const OrderMeta& o, uint64_t number,
                                                 uint32_t m32, uint32_t c32, uint32_t need_mem) {
  const uint64_t c = c32 < 0xffffffu ? c32 : 0xffffffu;
  const uint64_t n = number < 0xffull ? number : 0xffull;
  const uint64_t key = (c << 9) | (n << 1) | (need_mem != 0u ? 1ull : 0ull);
  uint32_t lo = 0, hi = o.n_groups;  // lower_bound: the group's rank (the key is present)
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (o.groups[mid] < key) lo = mid + 1; else hi = mid;
  }
  // (memory ranks: the rank thresholds, monotone in scv/memory)
  const uint64_t m = m32;
  const uint32_t nb = 1u << o.nb_log2;
  uint32_t b = (uint32_t)(m >> o.m_shift);
  b = b < nb ? b : nb - 1u;
  if (lo & 1u) b = nb - 1u - b;
  return (lo << o.nb_log2) | b;
}

// Per workgroup: an LDS histogram of the buckets (each pod's rank inside its workgroup's
// share of the bucket), then one global atomic per (workgroup, bucket): the share's base.
__global__ __launch_bounds__(1024) void k_order_hist(OrderMeta o, const uint64_t* __restrict__ number,
                                                     const uint32_t* __restrict__ m32,
                                                     const uint32_t* __restrict__ c32,
                                                     const uint32_t* __restrict__ need_mem,
                                                     uint32_t n_pods, uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ slot,
                                                     uint32_t* __restrict__ bkt) {
  extern __shared__ uint32_t lh[];
  const uint32_t nbk = o.n_groups << o.nb_log2;
  for (uint32_t i = threadIdx.x; i < nbk; i += blockDim.x) lh[i] = 0u;
  __syncthreads();
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t b = 0, local = 0;
  if (p < n_pods) {
    b = order_bucket(o, number[p], m32[p], c32[p], need_mem[p]);
    local = atomicAdd(&lh[b], 1u);
  }
  __syncthreads();
  // one global add per (workgroup, bucket) in use: all of a thread's adds in flight at once
  // (nbk <= 16 * blockDim.x), then their returns -- the shares' bases -- back into LDS
  constexpr int kAdds = 16;
  uint32_t base[kAdds];
#pragma unroll
  for (int k = 0; k < kAdds; ++k) {
    const uint32_t i = threadIdx.x + (uint32_t)k * blockDim.x;
    const uint32_t c = i < nbk ? lh[i] : 0u;
    base[k] = c ? atomicAdd(&hist[i], c) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kAdds; ++k) {
    const uint32_t i = threadIdx.x + (uint32_t)k * blockDim.x;
    if (i < nbk) lh[i] = base[k];
  }
  __syncthreads();
  if (p < n_pods) {
    slot[p] = lh[b] + local;
    bkt[p] = b;
  }
}

// One workgroup per group: exclusive scan of its NB bucket counts from the group's first
// sorted position; the counts are cleared for the next run.
constexpr uint32_t kOrderMaxBuckets = 1024;  // buckets per group (nb_log2 <= 10)
__global__ __launch_bounds__(kOrderMaxBuckets) void k_order_scan(OrderMeta o,
                                                                 uint32_t* __restrict__ hist,
                                                                 uint32_t* __restrict__ bstart) {
  __shared__ uint32_t sc[kOrderMaxBuckets];
  const uint32_t g = blockIdx.x, t = threadIdx.x, nb = 1u << o.nb_log2;
  const uint32_t i = (g << o.nb_log2) + t;
  const uint32_t c = t < nb ? hist[i] : 0u;
  sc[t] = c;
  __syncthreads();
  for (uint32_t d = 1; d < nb; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = t >= d ? sc[t - d] : 0u;
    __syncthreads();
    sc[t] += v;
    __syncthreads();
  }
  if (t < nb) {
    bstart[i] = o.gstart[g] + sc[t] - c;
    hist[i] = 0u;
  }
}

// Sorted position of every pod: perm[pos] = p, and every pod array scattered to pos.  The
// threads past the batch fill the padding slots (pad: (slot, caller pod) pairs, the pod a
// copy of the group's last in memory order) and clear the `zero` words (the K1 block list).
__global__ __launch_bounds__(kBlock) void k_order_scatter(PermTable t,
                                                          const uint32_t* __restrict__ slot,
                                                          const uint32_t* __restrict__ bkt,
                                                          const uint32_t* __restrict__ bstart,
                                                          uint32_t n_pods,
                                                          const uint32_t* __restrict__ pad,
                                                          uint32_t n_pad, uint64_t* __restrict__ zero,
                                                          uint32_t n_zero,
                                                          uint32_t* __restrict__ perm) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  for (uint32_t z = i; z < n_zero; z += gridDim.x * kBlock) zero[z] = 0ull;
  uint32_t p, pos;
  if (i < n_pods) {
    p = i;
    pos = bstart[bkt[p]] + slot[p];
  } else if (i - n_pods < n_pad) {
    pos = pad[2 * (i - n_pods)];
    p = pad[2 * (i - n_pods) + 1];
  } else {
    return;
  }
  perm[pos] = p;
  for (uint32_t a = 0; a < t.n; ++a) {
    if (t.bytes[a] == 8)
      static_cast<uint64_t*>(t.dst[a])[pos] = static_cast<const uint64_t*>(t.src[a])[p];
    else
      static_cast<uint32_t*>(t.dst[a])[pos] = static_cast<const uint32_t*>(t.src[a])[p];
  }
}

// t: the pod arrays (src = caller order, dst = sorted order); scratch: slot, bkt [P] u32.
hipError_t launch_order_count(const OrderMeta& o, const uint64_t* number, const uint32_t* m32,
                              const uint32_t* c32, const uint32_t* need_mem, uint32_t n_pods,
                              uint32_t* hist, uint32_t* bstart, uint32_t* slot, uint32_t* bkt,
                              const PermTable& t, const uint32_t* pad, uint32_t n_pad,
                              uint64_t* zero, uint32_t n_zero, uint32_t* perm, hipStream_t s) {
  const uint32_t nbk = o.n_groups << o.nb_log2;
  if (o.nb_log2 > 10 || nbk > 16u * 1024u) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_order_hist, dim3((n_pods + 1023) / 1024), dim3(1024), nbk * 4, s, o,
                     number, m32, c32, need_mem, n_pods, hist, slot, bkt);
  hipLaunchKernelGGL(k_order_scan, dim3(o.n_groups), dim3(1u << o.nb_log2), 0, s, o, hist,
                     bstart);
  hipLaunchKernelGGL(k_order_scatter, dim3((n_pods + n_pad + kBlock - 1) / kBlock), dim3(kBlock),
                     0, s, t, slot, bkt, bstart, n_pods, pad, n_pad, zero, n_zero, perm);
  return hipGetLastError();
}

}  // namespace yoda
