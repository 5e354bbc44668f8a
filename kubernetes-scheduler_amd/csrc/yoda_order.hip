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

// key = clock (clamped to 24 bits) | number (8 bits) | memory (32 bits), lexicographic:
// ascending clock puts the K1 `clock >= c` skips together too.  Any key is correct; this one
// is just fast.  The fields are packed at the widths the batch actually uses (host: the OR
// of each clamped field at upload), so the radix sort runs over bn + bm + bc bits only —
// same order as the full-width key, fewer passes.
//
// Serpentine: memory ascends in the even (clock, number) groups and descends in the odd
// ones (rank among the batch's groups, host-built sorted list `groups`).  A wave that
// straddles two groups then holds pods of similar memory from both ends instead of the
// largest requests of one group next to the smallest of the next: its pods qualify the
// same cards on most nodes, where a straddling ascending wave spans every memory size and
// leaves the block K2 nothing but per-pod work.
__device__ __forceinline__ uint64_t order_key(uint64_t number, uint64_t m_u, uint64_t c_u,
                                              uint32_t n_shift, uint32_t c_shift,
                                              const uint32_t* __restrict__ groups,
                                              uint32_t n_groups) {
  const uint64_t c = c_u < 0xffffffull ? c_u : 0xffffffull;
  const uint64_t n = number < 0xffull ? number : 0xffull;
  uint64_t m = m_u < 0xffffffffull ? m_u : 0xffffffffull;
  if (groups) {
    const uint32_t g = (uint32_t)(c << 8) | (uint32_t)n;
    uint32_t lo = 0, hi = n_groups;  // lower_bound: the group's rank
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (groups[mid] < g) lo = mid + 1; else hi = mid;
    }
    const uint64_t m_all = n_shift >= 32 ? 0xffffffffull : (1ull << n_shift) - 1ull;
    if (lo & 1u) m = m_all - m;  // m <= m_all: n_shift is the width of the batch's m field
  }
  return (c << c_shift) | (n << n_shift) | m;
}

__global__ __launch_bounds__(kBlock) void k_order_keys(const uint64_t* __restrict__ number,
                                                       const uint64_t* __restrict__ m_u,
                                                       const uint64_t* __restrict__ c_u,
                                                       uint32_t n_pods, uint32_t n_shift,
                                                       uint32_t c_shift,
                                                       const uint32_t* __restrict__ groups,
                                                       uint32_t n_groups,
                                                       uint64_t* __restrict__ keys,
                                                       uint32_t* __restrict__ idx) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  keys[p] = order_key(number[p], m_u[p], c_u[p], n_shift, c_shift, groups, n_groups);
  idx[p] = p;
}

// The same key when it fits 32 bits (the usual case: clock < 2^11, number < 2^4, memory in
// MiB < 2^17): half the bytes per radix pass.
__global__ __launch_bounds__(kBlock) void k_order_keys32(const uint64_t* __restrict__ number,
                                                         const uint64_t* __restrict__ m_u,
                                                         const uint64_t* __restrict__ c_u,
                                                         uint32_t n_pods, uint32_t n_shift,
                                                         uint32_t c_shift,
                                                         const uint32_t* __restrict__ groups,
                                                         uint32_t n_groups,
                                                         uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ idx) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= n_pods) return;
  keys[p] = (uint32_t)order_key(number[p], m_u[p], c_u[p], n_shift, c_shift, groups, n_groups);
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
                             uint32_t n_pods, const uint32_t key_bits[3],
                             const uint32_t* groups, uint32_t n_groups, void* scratch,
                             size_t scratch_bytes, uint32_t* perm, hipStream_t s) {
  // key_bits = widths of (c, n, m); each <= its clamp (24, 8, 32), so the total is <= 64
  const uint32_t bc = key_bits[0] < 24 ? key_bits[0] : 24;
  const uint32_t bn = key_bits[1] < 8 ? key_bits[1] : 8;
  const uint32_t bm = key_bits[2] < 32 ? key_bits[2] : 32;
  const uint32_t n_shift = bm, c_shift = bm + bn;
  const int end_bit = (int)(bc + bn + bm) > 0 ? (int)(bc + bn + bm) : 1;
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
                       number, m_u, c_u, n_pods, n_shift, c_shift, n_groups ? groups : nullptr,
                       n_groups, k32_in, idx_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k32_in, k32_out, idx_in, perm,
                                              (int)n_pods, 0, end_bit, s);
  }
  hipLaunchKernelGGL(k_order_keys, dim3((n_pods + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                     number, m_u, c_u, n_pods, n_shift, c_shift, n_groups ? groups : nullptr,
                     n_groups, keys_in, idx_in);
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

}  // namespace yoda
