// yoda_capi.cpp — host side of libyoda: the C-ABI of include/yoda.h.
//
// Packs the node snapshot and pod requests into the device layout of yoda_layout.h, picks
// the exact-f64 fast path or the exact-u64 generic path, and sequences the kernels of
// yoda_kernels.hip on the handle's stream.  No exception crosses the C boundary.
#include <dlfcn.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: librccl is opened at yoda_comm_init (dlopen)

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>
#include <thread>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <array>

#include "../../include/yoda.h"
#include "yoda_layout.h"

namespace yoda {
// launchers (yoda_kernels.hip)
hipError_t launch_k1(int K, Path path, const unsigned char* nodes, const unsigned char* sum,
                     const unsigned char* sum2, const unsigned char* mix,
                     uint32_t n_nodes, uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                     uint32_t n_pods, const Partials& part, uint64_t* bm, uint32_t bm_stride,
                     BlockMask* bs, uint32_t bs_stride, uint64_t* blk, uint32_t blk_stride,
                     unsigned long long* stats, hipStream_t s, uint32_t sub);
hipError_t launch_reduce1(const Partials& part, uint32_t C, uint32_t n_pods, uint32_t nw,
                          uint64_t* maxima, uint32_t* counts, double* rcp,
                          const MemTab& mt, hipStream_t s,
                          uint32_t* lpt_w = nullptr, uint32_t* lpt_order = nullptr,
                          const uint64_t* cmask = nullptr);
hipError_t launch_k1_order(int K, const PodParams& pp, uint32_t n_pods, uint32_t n_nodes,
                           uint32_t* wts, uint32_t* order, hipStream_t s);
hipError_t launch_mem_rank(const uint64_t* m_u, uint32_t n_pods, const MemTab& mt, uint32_t* m32,
                           hipStream_t s);
hipError_t launch_prep2(const uint64_t* maxima, uint32_t n_pods, double* rcp,
                        hipStream_t s);
hipError_t launch_window_out(const uint32_t* counts, const uint64_t* maxima, const uint32_t* wit,
                             const double* tk_s, const uint32_t* tk_i, const uint32_t* perm,
                             uint32_t wn, uint32_t kt, bool lists_row_major, unsigned char* out,
                             uint32_t* inv_scratch, hipStream_t s);
hipError_t launch_k2(int K, Path path, const unsigned char* nodes, const unsigned char* sum2,
                     const uint64_t* blk, uint32_t blk_stride, uint32_t n_nodes,
                     uint32_t chunk_nodes, uint32_t C, const PodParams& pp, const uint64_t* maxima,
                     const double* rcp, uint32_t n_pods,
                     const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                     uint32_t bs_stride, const Partials& part, int64_t* rows,
                     unsigned long long* stats, const uint32_t* counts, hipStream_t s);
hipError_t launch_k2b_rows(const NodeRecB* nodes, uint32_t n_nodes, const PodParams& pp,
                           uint32_t n_pods, const Partials& part, int64_t* rows, hipStream_t s);
hipError_t launch_k2_diskio(const NodeRecB* nodes, uint32_t n_nodes, uint32_t chunk_nodes,
                            uint32_t C, const PodParams& pp, uint32_t n_pods, const Partials& part,
                            int64_t* rows, hipStream_t s);
DiskPlan diskio_plan(uint32_t n_nodes, uint32_t n_cls);
hipError_t launch_k2b(const NodeRecB* nodes, uint32_t n_nodes, const double* cab,
                      uint32_t n_cls, const DiskLevels& lv, const DiskPlan& pl, uint32_t* plc,
                      uint32_t* pidx, hipStream_t s);
hipError_t launch_reduce2b(const uint32_t* plc, const uint32_t* pidx, uint32_t C, uint32_t n_cls,
                           const uint32_t* cls, uint32_t n_pods, uint32_t node_offset,
                           int64_t* best, uint32_t* idx, uint32_t* ties, int64_t* low,
                           hipStream_t s);
hipError_t launch_rows_transpose(const int64_t* in, uint32_t n_nodes, uint32_t n_pods,
                                 const uint32_t* perm,
                                 int64_t* out, hipStream_t s);
hipError_t launch_reduce2(const Partials& part, uint32_t C, uint32_t n_pods, bool is_f64,
                          uint32_t node_offset, int64_t* best, uint32_t* idx, uint32_t* ties,
                          int64_t* low, hipStream_t s, const uint64_t* cmask = nullptr);
hipError_t launch_merge_prepare(const int64_t* best_global, const int64_t* best_local,
                                uint32_t n_pods, uint32_t* idx, uint32_t* ties, hipStream_t s);
hipError_t launch_fill_diskio_state(uint32_t n_pods, uint32_t n_nodes, uint64_t* maxima,
                                    uint32_t* counts, hipStream_t s);
hipError_t launch_finalize(const uint32_t* counts, const int64_t* best, const uint32_t* idx,
                           const uint32_t* ties_in, const int64_t* lowest, uint32_t n_pods,
                           bool generic, int32_t* pick, int32_t* status, uint32_t* ties_out,
                           uint32_t* flagged, uint32_t* n_flagged, const FinalScatter& sc,
                           hipStream_t s);
hipError_t launch_k3(int K, const unsigned char* nodes, uint32_t n_nodes, uint32_t chunk_nodes,
                     uint32_t C, const PodParams& pp, const uint64_t* maxima, uint32_t n_pods,
                     const uint64_t* bm, uint32_t bm_stride, const uint32_t* flagged,
                     const uint32_t* n_flagged,
                     const int64_t* best, const int64_t* low, const Partials& part,
                     uint32_t max_flagged, hipStream_t s);
hipError_t launch_reduce3_rec(const Partials& part, uint32_t C, const uint32_t* flagged,
                              const uint32_t* n_flagged, uint32_t max_flagged,
                              uint32_t node_offset, ShardRec* rec, hipStream_t s);
hipError_t launch_merge3(const ShardRec* all, uint32_t n_pods, uint32_t world,
                         const uint32_t* flagged, const uint32_t* n_flagged, uint32_t max_flagged,
                         int32_t* pick, int32_t* status, uint32_t* ties, hipStream_t s);
hipError_t launch_reduce3(const Partials& part, uint32_t C, const uint32_t* flagged,
                          const uint32_t* n_flagged, uint32_t max_flagged, uint32_t node_offset,
                          int32_t* pick, int32_t* status, uint32_t* ties, hipStream_t s);
hipError_t launch_bitmask_transpose(const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                                    uint32_t bs_stride, const uint64_t* blk, uint32_t blk_stride,
                                    uint32_t n_nodes,
                                    uint32_t W, uint32_t n_pods, const uint32_t* perm,
                                    uint32_t* out, hipStream_t s);
int kernel_capacity(int K, Path path, int which, int mode_diskio);
hipError_t launch_k2_topk(int K, Path path, const unsigned char* nodes, uint32_t n_nodes,
                          uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                          const double* rcp, uint32_t n_pods,
                          const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                          uint32_t bs_stride, const uint64_t* blk, uint32_t blk_stride,
                          const Partials& part, double* tk_s, uint32_t* tk_i, int tk,
                          hipStream_t s);
hipError_t launch_topk_merge(const double* tk_s, const uint32_t* tk_i, uint32_t C,
                             uint32_t n_pods, uint32_t node_offset, double* out_s,
                             uint32_t* out_i, int tk, hipStream_t s);
hipError_t launch_k2_topk_block(int K, const unsigned char* nodes, const unsigned char* sum2,
                                const uint64_t* blk, uint32_t blk_stride, uint32_t n_nodes,
                                uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                                const double* rcp, uint32_t n_pods,
                                const uint64_t* bm, uint32_t bm_stride, const BlockMask* bs,
                                uint32_t bs_stride, const uint32_t* counts, uint64_t* keys,
                                uint32_t ib, int tk, hipStream_t s);
hipError_t launch_topk_merge_deep(const uint64_t* keys, uint32_t C, uint32_t n_pods, uint32_t ib,
                                  uint32_t node_offset, double* out_s, uint32_t* out_i, int tk,
                                  int ko, hipStream_t s);
hipError_t launch_topk_merge_keys(const uint64_t* keys, uint32_t C, uint32_t n_pods, uint32_t ib,
                                  uint32_t node_offset, double* out_s, uint32_t* out_i, int tk,
                                  hipStream_t s);
hipError_t launch_set_static(unsigned char* nodes, uint32_t stride, const uint32_t* node,
                             const uint64_t* value, const uint64_t* card_number, uint32_t count,
                             unsigned char* sum, uint32_t sum_stride, unsigned char* sum2,
                             uint32_t sum2_stride, const PermCopy& pc, hipStream_t s);
hipError_t launch_bsum_cn(const unsigned char* sum, uint32_t sum_stride, uint32_t n_nodes,
                          uint32_t* bsum, uint32_t bsw, hipStream_t s);
hipError_t launch_block_ub(int K, const uint32_t* sum2, const uint32_t* tab, uint32_t n_nodes,
                           uint32_t* out, const uint32_t* levels, hipStream_t s);
hipError_t launch_block_dec(int K, const uint32_t* sum2, const uint32_t* mix, uint32_t n_nodes,
                            uint32_t* out, const uint32_t* levels, MemTab mt, hipStream_t s);
hipError_t launch_gtable(int K, const uint32_t* sum2, const uint32_t* mix, uint32_t n_nodes,
                         const uint64_t* g_max,
                         uint32_t* tab, uint32_t* rcp_out, MemTab mt, hipStream_t s);
int topk_k();
int topk_k_capacity();
uint32_t greedy_one_blocks();
hipError_t launch_greedy_one(int K, Path path, const unsigned char* nodes,
                             const unsigned char* sum2, uint32_t n_nodes,
                             const PodParams& pp, const double* rcp,
                             uint32_t n_pods, uint32_t s, const uint64_t* bm, uint32_t bm_stride,
                             const BlockMask* bs, uint32_t bs_stride, const uint64_t* blk,
                             uint32_t blk_stride, double* part_s, uint32_t* part_i, uint32_t* done, uint32_t* out,
                             hipStream_t st);
hipError_t launch_k1_witness(int K, Path path, const unsigned char* nodes, uint32_t n_nodes,
                             uint32_t chunk_nodes, uint32_t C, const PodParams& pp,
                             uint32_t n_pods, uint64_t* pmax, uint32_t* pwit, uint32_t* pcnt,
                             uint64_t* bm, uint32_t bm_stride, hipStream_t s);
hipError_t launch_k1_block_witness(int K, const unsigned char* nodes, const unsigned char* sum,
                                   const unsigned char* sum2, const unsigned char* mix,
                                   uint32_t n_nodes, uint32_t chunk_nodes, uint32_t C,
                                   const PodParams& pp, uint32_t n_pods, uint64_t* pmax,
                                   uint32_t* pwit, uint32_t* pcnt, uint64_t* bm,
                                   uint32_t bm_stride, BlockMask* bs, uint32_t bs_stride,
                                   uint64_t* blk, uint32_t blk_stride, hipStream_t s);
hipError_t launch_reduce_wit(const uint64_t* pmax, const uint32_t* pwit, const uint32_t* pcnt,
                             uint32_t C, uint32_t n_pods, uint32_t node_offset, uint64_t* maxima,
                             uint32_t* counts, uint32_t* wcount, uint32_t* wnode, const MemTab& mt, hipStream_t s);
hipError_t launch_wit_prepare(const uint64_t* gmax, const uint64_t* lmax, uint32_t n_pods,
                              uint32_t* wit, hipStream_t s);
uint32_t one_blocks();
hipError_t launch_one(int K, Path path, const unsigned char* nodes, uint32_t n_nodes,
                      const OnePod& pod, uint64_t* feas, void* part, uint32_t* done,
                      OneOut* out, const MemTab& mt, hipStream_t s);
hipError_t launch_norm_rows(const int64_t* rows, uint32_t n_nodes, uint32_t n_pods,
                            const int64_t* best, const int64_t* lowest, int64_t* norm,
                            hipStream_t s);
hipError_t launch_pack_rec(const int64_t* best, const uint32_t* idx, const uint32_t* ties,
                           const int64_t* low, uint32_t n_pods, ShardRec* rec, hipStream_t s);
hipError_t launch_merge_rec(const ShardRec* all, uint32_t n_pods, uint32_t world, int64_t* best,
                            uint32_t* idx, uint32_t* ties, int64_t* low, hipStream_t s);
hipError_t launch_sum_multi_u32(const PtrList& src, uint32_t k, uint64_t n, uint32_t* dst,
                                hipStream_t s);
hipError_t launch_pack_key(const int64_t* best, const uint32_t* idx, uint32_t n_pods, uint32_t ib,
                           uint64_t* key, hipStream_t s);
hipError_t launch_unpack_key(const uint64_t* key, uint32_t n_pods, uint32_t ib, int64_t* best,
                             uint32_t* idx, uint32_t* ties, int64_t* low, hipStream_t s);
hipError_t launch_max_multi(const PtrList& src, uint32_t k, uint64_t n, uint64_t* dst,
                            hipStream_t s);
size_t order_scratch_bytes(uint32_t n_pods);
hipError_t launch_order_pods(const uint64_t* number, const uint64_t* m_u, const uint64_t* c_u,
                             const uint32_t* need_mem, uint32_t n_pods, const uint32_t key_bits[3],
                             const uint64_t* groups, uint32_t n_groups, void* scratch,
                             size_t scratch_bytes, uint32_t* perm, const uint32_t* m32, hipStream_t s);
hipError_t launch_order_count(const OrderMeta& o, const uint64_t* number, const uint32_t* m32,
                              const uint32_t* c32, const uint32_t* need_mem, uint32_t n_pods,
                              uint32_t* hist, uint32_t* bstart, uint32_t* slot, uint32_t* bkt,
                              const PermTable& t, const uint32_t* pad, uint32_t n_pad,
                              uint64_t* zero, uint32_t n_zero, uint32_t* perm, hipStream_t s);
hipError_t launch_permute(const PermTable& t, const uint32_t* perm, uint32_t n_pods, bool scatter,
                          hipStream_t s);
}  // namespace yoda

using namespace yoda;

namespace {

struct Status {
  int code;
  std::string msg;
};

// Grow-only device buffer.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    const size_t alloc = std::max<size_t>(n, 256);
    hipError_t e = hipMalloc(&p, alloc);
    if (e == hipSuccess) bytes = alloc;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Grow-only pinned host buffer (fast async H2D).
struct PinnedBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void* dp = nullptr;  // the same pages as seen by kernels (hipHostMalloc maps them)
  unsigned flags = hipHostMallocDefault;  // hipHostMallocCoherent: polled by the host
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    bytes = 0;
    const size_t alloc = std::max<size_t>(n, 4096);
    hipError_t e = hipHostMalloc(&p, alloc, flags);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
    if (e == hipSuccess) bytes = alloc;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// RCCL entry points, resolved at the first yoda_comm_* call: libyoda itself does not link
// RCCL (a process that already loaded one -- e.g. PyTorch's, same SONAME -- shares it).
struct RcclApi {
  bool tried = false, ok = false;
  std::string err;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool load() {
    if (tried) return ok;
    tried = true;
    void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!so) {
      err = std::string("librccl.so.1 not found: ") + dlerror();
      return false;
    }
    auto sym = [&](const char* name) {
      void* f = dlsym(so, name);
      if (!f) err = std::string("librccl: missing ") + name;
      return f;
    };
    get_unique_id = reinterpret_cast<decltype(get_unique_id)>(sym("ncclGetUniqueId"));
    comm_init_rank = reinterpret_cast<decltype(comm_init_rank)>(sym("ncclCommInitRank"));
    all_reduce = reinterpret_cast<decltype(all_reduce)>(sym("ncclAllReduce"));
    all_gather = reinterpret_cast<decltype(all_gather)>(sym("ncclAllGather"));
    comm_destroy = reinterpret_cast<decltype(comm_destroy)>(sym("ncclCommDestroy"));
    group_start = reinterpret_cast<decltype(group_start)>(sym("ncclGroupStart"));
    group_end = reinterpret_cast<decltype(group_end)>(sym("ncclGroupEnd"));
    error_string = reinterpret_cast<decltype(error_string)>(sym("ncclGetErrorString"));
    ok = get_unique_id && comm_init_rank && all_reduce && all_gather && comm_destroy &&
         group_start && group_end && error_string;
    return ok;
  }
};
RcclApi& rccl() {
  static RcclApi a;
  return a;
}

enum PodArray {
  kPodMF, kPodCF, kPodMU, kPodCU, kPodNumber, kPodAlpha, kPodBeta,
  kPodM32, kPodC32, kPodNeedMem, kPodNeedClk, kPodArrays
};
constexpr size_t kPodArrayBytes[kPodArrays] = {8, 8, 8, 8, 8, 8, 8, 4, 4, 4, 4};
// Placement in the uploaded blob: first the arrays a private run on the block kernels reads (the
// counting order included), then the rest, whose copy waits for the first entry point that
// needs it (pods_complete) -- after the kernels of such a run.
constexpr int kPodCoreArrays = 5;
constexpr int kPodPlace[kPodArrays] = {kPodM32, kPodC32, kPodNumber, kPodNeedMem, kPodNeedClk,
                                       kPodMU, kPodCU, kPodMF, kPodCF, kPodAlpha, kPodBeta};

}  // namespace

struct yoda_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  std::string last_error;

  // node snapshot
  bool has_nodes = false;
  bool generic = false;  // path == Path::U64
  Path path = Path::N32;
  bool nodes_diskio = false;  // node cpu/disk_io present
  bool pods_diskio = false;   // pod rio/rcpu present
  int K = 1;
  uint32_t n_nodes = 0, node_offset = 0;
  DevBuf nodes;     // fast or generic records
  DevBuf nodes_b;   // Mode B records
  DevBuf k1sum;     // K1 node summaries (N32 path, yoda_layout.h K1SumWord)
  DevBuf k2sum;     // K2 node summaries (N32 path, yoda_layout.h K2SumWord)
  DevBuf kmix;      // per-card GPU models in free order (N32 path, yoda_layout.h MixWord)
  DevBuf kx1;       // K1's tile of the mixed-model nodes (N32 path, yoda_layout.h K1MixWord)
  // memory ranks (yoda_layout.h MemTab): the N32 memory fields are ranks; value tables
  bool mem_ranks = false;
  DevBuf memtab;
  MemTab mt = {};
  std::vector<uint64_t> h_frees;  // the distinct card frees, ascending (pod thresholds)
  DevBuf gtab, gtab_aux;  // the G table (yoda_layout.h GTab) + [G maxima | its reciprocals]
  GTab g = {};
  bool has_k1sum = false, has_k2sum = false;
  bool all_one_model = false;  // every node: one GPU model, one TotalMemory (kNodeUniform4|Total)
  // block-grouped node order of the private batch runs (node_perm at upload): copies of the
  // K1 / K2 summaries and the G table in that order, the local id of each position, and each
  // node's position (k_set_static keeps the copies current)
  bool perm_on = false;
  DevBuf k1sum_p, k2sum_p, gtab_p, perm_ids, perm_inv;
  DevBuf kx1_p, kmix_p;  // the mixed-model tiles in that order (immutable card data)
  DevBuf win_inv;        // capacity windows: each window slot's sorted position (k_window_out)
  // 64-node block summaries (yoda_layout.h BlockSumWord) of the snapshot order and of the
  // block-grouped copy's; loose: node-state pushes left their CardNumber bounds valid but not
  // tight (k_set_static's atomics), recomputed before the next private run
  DevBuf blksum, blksum_p;
  bool blksum_loose = false;
  bool greedy_active = false;  // inside a greedy batch (its pushes keep the bounds valid)
  // K2 block bounds (yoda_layout.h kbub_*) of both orders; dirty: static scores changed since
  DevBuf kbub, kbub_p;
  DevBuf kbdec, kbdec_p;     // the non-G block bounds (yoda_layout.h kbdec_*) of both orders
  DevBuf kb_levels;          // the free levels of kbub's lv[] bounds (kKbLevels u32)
  bool seeds_valid = false;  // this run's block K1 cleared and writes the K2 pruning seeds
  bool blk_fresh = false;    // this run cleared the whole block-list buffer (list, seeds, gbest)
  bool kb_levels_ok = false;  // built for the current snapshot
  bool kbub_dirty = true;   // a static score rose above the bounds' own: rebuild before use
  bool kbub_loose = false;  // static scores only fell since the build: valid, rebuilt for runs
  std::vector<uint64_t> ub_stat;  // each node's static score when the bounds were built
  // a pushed static score against the bounds: above -> dirty, else loose
  void note_static(uint32_t n, uint64_t s) {
    if (n < ub_stat.size() && s <= ub_stat[n]) kbub_loose = true; else kbub_dirty = true;
  }
  // the top tenth of the blocks by bound (ub[K]) at upload, per order: K2 visits them first
  DevBuf hot, hot_p;
  bool hot_ok = false;
  PermCopy perm_copy() const {
    PermCopy pc;
    if (perm_on) {
      pc.inv = perm_inv.as<uint32_t>();
      pc.sum = k1sum_p.as<unsigned char>();
      pc.sum2 = k2sum_p.as<unsigned char>();
      pc.bsum_p = blksum_p.p ? blksum_p.as<uint32_t>() : nullptr;
    }
    pc.bsum = blksum.p && path == Path::N32 ? blksum.as<uint32_t>() : nullptr;
    pc.bsum_words = bsum_stride(K) / 4u;
    return pc;
  }
  // this run is block-grouped.  On a snapshot with mixed-model nodes (or per-card TotalMemory)
  // only a large batch takes the grouped order: grouping gathers the nodes that need the
  // per-card pass into a few blocks, so a few (wave, chunk) tasks carry all of it -- on a
  // small batch (config 4: 10k pods x 20k nodes, K1 88 -> 143 us, the last tasks alone)
  // that tail outweighs the whole-block decisions, which win from 32k pods on (the config-4
  // generator at 100k x 100k: K1 0.52 -> 0.20 ms)
  bool perm_run() const {
    return perm_on && count_order && (all_one_model || n_work >= kGroupedMixedMinPods);
  }
  static constexpr uint32_t kGroupedMixedMinPods = 32768;
  bool all_uni4 = false;       // every node: one GPU model (kNodeUniform4)
  std::vector<unsigned char> host_records;  // kept for alloc updates (greedy)
  std::vector<uint32_t> host_k2sum;         // idem (its static score words)
  std::vector<uint64_t> h_total_sum, h_free_sum, h_alloc, h_card_number;
  // bound on any raw score of this snapshot whatever the allocated memory (Basic + the
  // largest Allocate 300 + Actual): the packed top-k keys need score < 2^(64 - index bits)
  uint64_t score_bound = ~0ull;

  // pods: one device blob of per-pod arrays (PodArray order), staged through pinned memory
  bool has_pods = false;
  uint32_t n_pods = 0;
  DevBuf pod_blob;
  PinnedBuf pod_stage;
  hipEvent_t stage_event = nullptr;
  // the deferred pod arrays' copy of a private run goes on a copy stream of its own, alongside
  // the run's kernels (pods_complete_async); rest_event joins it back into `stream`
  hipStream_t copy_stream = nullptr;
  hipEvent_t core_event = nullptr, rest_event = nullptr;
  bool rest_join = false;
  // the staged f64 thresholds and Mode B weights of the last upload are still to be written
  // (pods_pack_rest: derived from the staged u64 ones, after a run's kernel launches)
  bool rest_lazy = false;
  hipEvent_t switch_event = nullptr;  // yoda_set_stream: the old stream's work, waited on
  bool stage_pending = false;
  size_t pod_off[kPodArrays] = {};
  size_t pod_rest_off = 0, pod_rest_bytes = 0;  // the blob's deferred part (pods_complete)
  bool fast_run = false;  // inside a private block-kernel run: the deferred part may wait
  // a deferred private run's kernels are in flight before the non-core pod arrays (m_f, c_f,
  // m_u, c_u, alpha, beta) reach the device: pod_params hands out null pointers for them, so a
  // kernel that read them there would fault instead of reading the last batch's values
  bool core_only = false;
  // batch ordering (yoda_order.hip): when `ordered`, the kernels of this run read the pods
  // from pod_sorted (sorted position i = original pod perm[i]); bitmask/rows stay in sorted
  // order and are un-permuted by their transposes, the per-pod outputs by finalize().
  bool order_enabled = true;
  bool order_pad = true;  // yoda_set_pod_order(h, 1): pad private runs' groups to waves
  bool ordered = false;
  DevBuf pod_sorted, perm, order_scratch;
  uint32_t key_bits[3] = {24, 8, 32};  // widths of the batch's sort-key fields (c, n, m)
  // Counting-sort order (yoda_order.hip, OrderMeta), built at upload: the batch's distinct
  // (clock, number, has-memory) groups ascending, their first sorted positions unpadded and
  // padded to a wave, and the padding slots (dst, src) -- one device blob, host copy kept
  // for the async upload.  n_work: the sorted positions of this run (n_pad when padded).
  bool og_ok = false;
  uint32_t og_groups = 0, og_nb_log2 = 0, og_m_shift = 0, og_n_pad_slots = 0;
  uint32_t n_pad = 0, n_work = 0;
  size_t og_off_start = 0, og_off_start_pad = 0, og_off_pad = 0;
  std::vector<unsigned char> og_host;
  DevBuf order_meta, order_hist, order_bstart, order_slot, order_bkt;
  size_t sorted_off[kPodArrays] = {};

  // state
  DevBuf maxima, counts, rcp, best, idx, ties, lowest, pick, status, ties_out, flagged, n_flagged;
  // scatter targets of unpermute_outputs, swapped with the buffers above after each scatter
  DevBuf pick_alt, status_alt, ties_out_alt, counts_alt, best_alt, maxima_alt;
  DevBuf win_dev;  // a capacity window's outputs on the device, then one DMA copy to win_stage
  DevBuf bitmask, bitmask_t, rows, rows_t, norm;
  DevBuf blk;               // [wave][node block / 64] u64: blocks with a feasible pod (K1 -> K2)
  bool blk_valid = false;   // the last K1 wrote blk (block-classified K1 on this batch)
  bool blk_zeroed = false;  // this run's order already cleared blk (no memset in phase 1)
  bool flagged_dirty = true;  // n_flagged may be nonzero (a generic run since the last clear)
  bool maxima_sorted = false;  // h->maxima still in the last run's sorted order (n_work rows)
  bool rcp_ready = false;      // phase 1 wrote the reciprocals of its (final) maxima
  bool count_order = false;    // this run orders by the counting sort (private runs)
  DevBuf bsum;              // [wave][node block] BlockMask: the block K1's sparse masks
  bool bm_sparse = false;   // the last K1 wrote the sparse form (bsum + partial masks only)
  const BlockMask* bs_ptr() const { return bm_sparse ? bsum.as<BlockMask>() : nullptr; }
  // the sparse masks' block list: a block whose bit is clear has no feasible pod of the wave
  // and its BlockMask was not written this run
  const uint64_t* blk_ptr() const { return bm_sparse ? blk.as<uint64_t>() : nullptr; }
  // greedy
  DevBuf tk_s_part, tk_i_part, tk_s, tk_i, upd_node, upd_val, upd_cn;
  DevBuf g1_part, g1_done;  // k_greedy_one partials + block counter (zeroed once)
  DevBuf p_wit, wit;        // capacity greedy: witness partials [2][6][C][P], merged [2][6][P]
  DevBuf one_feas, one_part, one_done, one_out;  // k_one_*: a pod against the current state
  PinnedBuf upd_stage, pick_stage, win_stage;
  PinnedBuf poll_stage;  // coherent: the greedy fallback's pick, polled by the host
  uint32_t greedy_restarts = 0;
  uint32_t greedy_refreshes = 0;  // flags-0 mid-window list refreshes (last yoda_greedy)
  hipEvent_t upd_event = nullptr;
  bool upd_pending = false;
  std::vector<uint32_t> h_pos;  // yoda_shard_topk: caller pod index -> sorted position
  bool topk_ready = false;      // the bitmask / reciprocals of that batch are still valid
  uint32_t greedy_windows = 0, greedy_fallbacks = 0;
  double greedy_window_ms = 0, greedy_fallback_ms = 0, greedy_resolve_ms = 0;
  double greedy_prep_ms = 0;  // (YODA_GREEDY_DEBUG) the host part of the windows: state push,
                              // window gather + pod upload + order launches
  DevBuf p_max_u, p_cnt, p_best_f, p_best_i, p_idx, p_ties, p_low_f, p_low_i, p_err;
  uint32_t C1 = 1, chunk1 = 32;  // K1 node chunking (partial chunks; chunk1: nodes per K1 wave)
  uint32_t k1_sub = 1;
  bool pack16 = true;            // N32: the small card fields fit 16 bits (packed K1 partials)
  bool q32 = true;               // ... and <= kF32SmallMax (the block K2's f32 quotients)
  uint64_t small_max = 0;        // the largest bandwidth / clock / core / power (any path)
  // heaviest-first pod blocks for the argmax block K2 (k_lpt_order): this run uses them,
  // the per-wave weights K1 adds to (zero between runs), the order (valid once sorted)
  bool lpt_active = false, lpt_sorted = false;
  DevBuf lpt_w, lpt_order;           // K1 waves per chunk (4: k1_block_n32's SUB, chunk1 = a quarter)
  // the block K1's own heaviest-first order (k1_probe's weights, ranked before the K1): valid
  // for this run once k1_sorted
  bool k1_sorted = false;
  DevBuf k1_w, k1_order;
  uint32_t C2 = 1, chunk2 = 32;  // K2 / K3 node chunking
  int cap[2][3][2] = {};         // resident workgroups per (kernel, path, mode), cached
  int last_mode = -1;
  bool ran = false;
  bool ran_bitmask = false;
  bool phase1_done = false;
  bool phase1_wit = false;  // the last shard phase 1 was the witness one (capacity windows)

  // class counters of the block kernels (yoda_class_stats_*): device [8] u64 + host totals
  bool class_stats = false;
  DevBuf stats_dev;
  uint64_t stats_pairs1 = 0, stats_pairs2 = 0;
  unsigned long long* stats_ptr() const {
    return class_stats ? stats_dev.as<unsigned long long>() : nullptr;
  }
  // yoda_comm_*: this rank's RCCL communicator and the two exchange buffers of a step
  ncclComm_t comm = nullptr;
  int comm_rank = 0, comm_world = 1;
  DevBuf ex1, rec, rec_all;  // [maxima 6P | count slots world x P] u64; ShardRec [P], [world][P]
  // Caller-order exchange (xo): a node-shard evaluation whose exchanged buffers are in the
  // caller's pod order, so that each shard runs its private order -- the padded counting sort
  // and the block-grouped node order of yoda_run -- instead of the reproducible radix order
  // every shard must otherwise share (5.7x slower at one shard of config 3: no node grouping,
  // no padded waves).  yoda_comm_run does it on the fast record paths; the yoda_shard_* calls
  // after yoda_shard_exchange_order(h, 1).  xcnt, xbest, ... : the caller-order copies.
  bool xo_enabled = false, xo = false;
  DevBuf xcnt, xbest, xidx, xties, xlow;
  DevBuf cg_max, cg_cnt, cg_wit, cg_gather;  // yoda_comm_greedy: exchange buffers
  uint32_t comm_greedy_stats[5] = {};          // yoda_comm_greedy_stats
  // sharded exact normalize (K3 over a shard): per-pod records of the flagged pods, pending
  // until the shards' records are merged (yoda_shard_exact_merge)
  DevBuf k3rec, k3all;
  bool k3_pending = false;
  // Mode B batch path: the batch's pod classes (distinct (alpha, beta) bit pairs), built on
  // the first Mode B run after an upload: device [2][D] f64 (alpha, beta) + [P] u32 class
  // of each pod; chunk partials [2][C][D] u32
  bool b_cls_ready = false;
  uint32_t b_ncls = 0;
  DevBuf b_cab, b_cls, b_part;
  uint32_t k3_nfl = 0;
  // profiling: event pairs around K1 / K2
  bool profiling = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_k1, ev_k2;
  size_t ev_used = 0;

  hipEvent_t next_event() {
    if (ev_used == ev_pool.size()) {
      hipEvent_t e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      ev_pool.push_back(e);
    }
    return ev_pool[ev_used++];
  }

  ~yoda_handle() {
    if (comm && rccl().ok) (void)rccl().comm_destroy(comm);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    DevBuf* all[] = {&kx1_p, &kmix_p, &win_inv, &nodes,     &nodes_b,   &k1sum,     &k2sum,    &kmix,    &kx1,     &memtab,    &k1sum_p,   &k2sum_p,   &gtab_p, &blksum, &blksum_p, &kbub, &kbub_p, &kbdec, &kbdec_p, &kb_levels, &hot, &hot_p,    &perm_ids,  &perm_inv,    &pod_blob,   &maxima,       &counts,
                     &pod_sorted, &perm,     &order_scratch, &order_meta, &order_hist,
                     &order_bstart, &order_slot, &order_bkt,
                     &rcp,       &best,       &idx,          &ties,
                     &lowest,    &pick,      &status,     &ties_out,     &flagged,
                     &n_flagged, &bitmask,   &bitmask_t,  &blk,  &bsum, &p_max_u,      &p_cnt, &lpt_w, &lpt_order, &k1_w, &k1_order,
                     &rows,      &rows_t,    &norm,      &tk_s_part,  &tk_i_part,    &tk_s,
                     &tk_i,      &upd_node,  &upd_val,    &upd_cn,    &g1_part,   &g1_done,
                     &p_best_f,  &p_best_i,  &p_idx,      &p_ties,       &p_low_f,
                     &p_low_i,   &p_err,     &pick_alt,   &status_alt,   &ties_out_alt,
                     &p_wit,     &wit,       &stats_dev, &one_feas,  &one_part,  &one_done,
                     &ex1,       &rec,       &rec_all,   &cg_max,    &cg_cnt,    &cg_wit,    &cg_gather, &k3rec,     &k3all,
                     &one_out,   &b_cab,     &b_cls,     &b_part,
                     &counts_alt, &best_alt, &maxima_alt, &win_dev,
                     &xcnt,      &xbest,     &xidx,      &xties,     &xlow};
    for (DevBuf* b : all) b->release();
    pod_stage.release();
    upd_stage.release();
    pick_stage.release();
    poll_stage.release();
    win_stage.release();
    if (stage_event) (void)hipEventDestroy(stage_event);
    if (switch_event) (void)hipEventDestroy(switch_event);
    if (upd_event) (void)hipEventDestroy(upd_event);
    if (core_event) (void)hipEventDestroy(core_event);
    if (rest_event) (void)hipEventDestroy(rest_event);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }
};

namespace {

int fail(yoda_t* h, int code, const std::string& msg) {
  if (h) h->last_error = msg;
  return code;
}

#define HIP_TRY(h, expr)                                                                \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(h, YODA_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

int pow2_cards(uint32_t kmax) {
  int k = 1;
  while ((uint32_t)k < kmax) k <<= 1;
  return k;
}

// CalculateAllocateScore + CalculateActualScore (algorithm.go:293-310), uint64 wrap.
// zero_total: TotalMemorySum == 0, where the reference divides by zero.
uint64_t static_score(uint64_t free_sum, uint64_t total_sum, uint64_t alloc, bool* zero_total) {
  *zero_total = total_sum == 0;
  if (total_sum == 0) return 0;
  const uint64_t allocate = total_sum < alloc ? 0 : (total_sum - alloc) * 100u / total_sum * 3u;
  const uint64_t actual = (free_sum * 100u / total_sum) * 2u;
  return allocate + actual;
}

// Node chunking of one kernel: C chunks x ceil(P/256) pod blocks = B workgroups.  B is sized
// to ~8 full "rounds" of the kernel's resident capacity (occupancy API), so the last round is
// nearly full (efficiency >= 1 - pod_blocks / (8 cap)) and chunks stay small enough to
// balance data-dependent work (K2 skips infeasible nodes).
// Tuning knobs for A/B runs (tools/ab.sh): YODA_CHUNK_ROUNDS1 / 2 (K1 / K2; defaults 6 / 8;
// both at once, config 3: 3 1.92 ms, 4 1.87, 6 1.81, 8 1.78, 10 2.02 per step) and
// YODA_MIN_CHUNK_NODES (default 0 = no floor; a floor keeps the per-(wave, chunk) set-up of
// the block-classified kernels amortised when few pod blocks would otherwise mean many
// small chunks, e.g. one rank's pod shard).  Read once per process.
// Host worker pool for the packing loops (pod upload): threads created once per process and
// parked on a condition variable between calls -- spawning 15 threads per upload cost more
// than the packing itself.  run(n, fn) calls fn(0..n-1) once each, the caller taking part;
// calls are serialised (one batch at a time).
uint32_t pool_spin_us();  // (below, after the knobs)

// After a batch the workers spin for a short while before parking: a scheduler uploads its
// batches back to back, and a parked thread's wake-up is what a late range costs the pack.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool pool;
    return pool;
  }
  uint32_t size() const { return (uint32_t)threads_.size() + 1u; }
  void run(uint32_t n, const std::function<void(uint32_t)>& fn) {
    if (n == 0) return;
    if (n == 1 || threads_.empty()) {
      for (uint32_t i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> serial(call_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      last_n_.store(n, std::memory_order_relaxed);
      next_.store(0);
      left_ = n;
      gen_.fetch_add(1);  // (after the batch's fields: a spinning worker reads them next)
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return left_ == 0; });
    fn_ = nullptr;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }

 private:
  HostPool() {
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t n = std::min(16u, hw) - 1u;  // + the calling thread
    for (uint32_t i = 0; i < n; ++i) threads_.emplace_back([this, i] { loop(i); });
  }
  void work() {
    for (;;) {
      const uint32_t i = next_.fetch_add(1);
      if (i >= n_) return;
      (*fn_)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--left_ == 0) done_cv_.notify_one();
    }
  }
  void loop(uint32_t self) {
    uint64_t seen = 0;
    const uint32_t spin_us = pool_spin_us();
    for (;;) {
      // only the workers the last batch used spin (a small batch leaves the rest parked), and
      // they pause between polls so a sibling hyperthread keeps its issue slots
      if (spin_us && self + 1u < last_n_.load(std::memory_order_relaxed)) {
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t it = 0;
        while (gen_.load() == seen && !stop_.load()) {
          __builtin_ia32_pause();
          if ((++it & 63u) == 0u &&
              std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us))
            break;
        }
      }
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_.load() || gen_.load() != seen; });
        if (stop_.load()) return;
        seen = gen_.load();
      }
      work();
    }
  }
  std::vector<std::thread> threads_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(uint32_t)>* fn_ = nullptr;
  uint32_t n_ = 0, left_ = 0;
  std::atomic<uint32_t> next_{0}, last_n_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

// Tuning knobs of the A/B harness (tools/ab_lib.sh).  Only the A/B build reads them from
// the environment (`make ab` -> libyoda_ab.so, -DYODA_AB_KNOBS); in the release library
// YODA_KNOB(name, default) is the default itself and the name is not even in the binary, so
// a scheduler process's environment cannot change kernel choice, chunking or greedy policy.
#ifdef YODA_AB_KNOBS
static uint32_t knob_env(const char* name, uint32_t dflt) {
  const char* s = std::getenv(name);
  return (s && *s) ? (uint32_t)std::strtoul(s, nullptr, 10) : dflt;
}
#define YODA_KNOB(name, dflt) knob_env(name, dflt)
#else
#define YODA_KNOB(name, dflt) ((uint32_t)(dflt))
#endif
uint32_t pool_spin_us() {
  // how long a HostPool worker spins for the next batch before parking (YODA_POOL_SPIN_US,
  // A/B knob; 0 parks at once).  1 ms covers a batch-to-batch gap of the e2e loop (~0.9 ms);
  // a scheduler that uploads less often parks its workers after that.
  static const uint32_t v = YODA_KNOB("YODA_POOL_SPIN_US", 1000);
  return v;
}
// Diagnostics (*_TRACE, *_DEBUG): counters, timings and traces only, never results or policy.
static uint32_t diag_env(const char* name, uint32_t dflt) {
  const char* s = std::getenv(name);
  return (s && *s) ? (uint32_t)std::strtoul(s, nullptr, 10) : dflt;
}

constexpr uint32_t kMinChunkNodes = 1536;
// the reduces read the chunk partials one thread per pod up to this many chunks (the chunk
// masks' limit too); beyond, one wave per pod (yoda_kernels.hip kWaveReduceChunks)
constexpr uint32_t kPlainReduceChunks = 48;

void plan_chunks_for(uint32_t cap, uint32_t rounds, uint32_t n_pods, uint32_t n_nodes,
                     uint32_t* C_out, uint32_t* chunk_out) {
  static const uint32_t min_chunk = YODA_KNOB("YODA_MIN_CHUNK_NODES", 0);
  const uint32_t pod_blocks = std::max<uint32_t>(1, (n_pods + kBlock - 1) / kBlock);
  const uint32_t max_chunks = std::max<uint32_t>(1, (n_nodes + kChunkAlign - 1) / kChunkAlign);
  if (cap == 0) cap = 2048;
  uint32_t C = std::max<uint32_t>(1, (uint32_t)(((uint64_t)rounds * cap) / pod_blocks));
  C = std::min(C, max_chunks);
  if (min_chunk) {
    C = std::min(C, std::max<uint32_t>(1, (n_nodes + min_chunk - 1) / min_chunk));
  } else if (pod_blocks >= 64) {
    // a large pod batch over few nodes (one rank of a node-sharded batch): chunks of at least
    // kMinChunkNodes amortise the per-(wave, chunk) set-up of the block kernels, as long as
    // the grid keeps two rounds of resident workgroups (A/B in profiles/r02/final/)
    const uint32_t c_nodes = (n_nodes + kMinChunkNodes - 1) / kMinChunkNodes;
    const uint32_t c_rounds = (uint32_t)((2ull * cap + pod_blocks - 1) / pod_blocks);
    C = std::min(C, std::max<uint32_t>({1u, c_nodes, c_rounds}));
  }
  // a multiple of 8 chunks lets the kernels give each XCD whole chunks (tile() in
  // yoda_kernels.hip); trailing chunks may then be empty (they write identity partials)
  const bool xcd = C >= 8;
  if (xcd) C = (C + 7) / 8 * 8;
  uint32_t chunk = (n_nodes + C - 1) / C;
  chunk = std::max<uint32_t>(kChunkAlign, (chunk + kChunkAlign - 1) / kChunkAlign * kChunkAlign);
  *chunk_out = chunk;
  *C_out = xcd ? C : std::max<uint32_t>(1, (n_nodes + chunk - 1) / chunk);
}

int capacity(yoda_t* h, int which, int mode) {
  int& c = h->cap[which - 1][(int)h->path][mode == YODA_MODE_DISKIO ? 1 : 0];
  if (c == 0) c = kernel_capacity(h->K, h->path, which, mode == YODA_MODE_DISKIO);
  return c;
}

void plan_chunks(yoda_t* h, int mode, uint32_t n_pods, uint32_t n_nodes) {
  // K1's partials are 24 B a (pod, chunk) and its reduce reads them all, but with the
  // heaviest-first pod blocks and the lane = block pass a K1 task is short and the tail is
  // set by the task size: 8 rounds while the chunks stay few enough for the chunk masks
  // (C1 <= kPlainReduceChunks; config 3 K1 0.199 -> 0.182 ms, mixed50 / bytes / greedy neutral
  // or better; 10: 0.185, 12: 0.201, 16: 0.241 ms), else 6 (a 50k / 25k / 12.5k-pod batch,
  // one pod-sharded rank: K1 0.137 / 0.139 / 0.138 ms at 6 against 0.155 / 0.140 / 0.157 at
  // 8); profiles/r06/rounds1/.  YODA_CHUNK_ROUNDS1 (A/B knob) fixes the rounds.
  static const uint32_t r1_knob = YODA_KNOB("YODA_CHUNK_ROUNDS1", YODA_KNOB("YODA_CHUNK_ROUNDS", 0));
  static const uint32_t r2 = std::max<uint32_t>(1, YODA_KNOB("YODA_CHUNK_ROUNDS2",
                                                           YODA_KNOB("YODA_CHUNK_ROUNDS", 8)));
  const uint32_t cap1 = (uint32_t)capacity(h, 1, mode);
  plan_chunks_for(cap1, r1_knob ? r1_knob : 8u, n_pods, n_nodes, &h->C1, &h->chunk1);
  if (!r1_knob && h->C1 > kPlainReduceChunks)
    plan_chunks_for(cap1, 6u, n_pods, n_nodes, &h->C1, &h->chunk1);
  // YODA_K1_MAX_CHUNKS (A/B knob, default off): at most that many K1 chunks, so that small
  // batches keep their partials (and k_reduce1's reads) few
  static const uint32_t c1_max = YODA_KNOB("YODA_K1_MAX_CHUNKS", 0);
  if (c1_max && h->C1 > c1_max) {
    h->chunk1 = ((n_nodes + c1_max - 1) / c1_max + kChunkAlign - 1) / kChunkAlign * kChunkAlign;
    h->C1 = std::max<uint32_t>(1, (n_nodes + h->chunk1 - 1) / h->chunk1);
    if (h->C1 >= 8) {  // keep a multiple of 8 (XCD tiling); trailing chunks may be empty
      h->C1 = (h->C1 + 7) / 8 * 8;
    }
  }
  // YODA_K1_SUB=4 (A/B knob, off): the block K1 with SUB = 4 -- the same (pod wave, node range)
  // tasks, the four waves of a workgroup on quarters of one chunk merging their partials in
  // LDS: a quarter of the partial bytes, but K1 0.284-0.289 against 0.230-0.235 ms (the four
  // waves no longer share the node tiles in L1).  C1 becomes the chunk count, chunk1 the quarter.
  static const bool k1_split = YODA_KNOB("YODA_K1_SUB", 1) == 4;
  h->k1_sub = 1;
  if (k1_split && h->path == Path::N32 && h->has_k1sum && mode != YODA_MODE_DISKIO &&
      h->C1 >= 4) {
    uint32_t C = (h->C1 + 3) / 4;
    if (C >= 8) C = (C + 7) / 8 * 8;
    const uint32_t q = (n_nodes + 4 * C - 1) / (4 * C);
    h->chunk1 = std::max<uint32_t>(kChunkAlign, (q + kChunkAlign - 1) / kChunkAlign * kChunkAlign);
    h->C1 = C >= 8 ? C : std::max<uint32_t>(1, (n_nodes + 4 * h->chunk1 - 1) / (4 * h->chunk1));
    h->k1_sub = 4;
  }
  plan_chunks_for((uint32_t)capacity(h, 2, mode), r2, n_pods, n_nodes, &h->C2, &h->chunk2);
}

// u64 words of the block-list buffer: the list, the seeds, the shared best (ensure_state)
size_t blk_words(const yoda_t* h, uint32_t P) {
  const size_t nw = (P + 63) / 64;
  return nw * (blk_row(h->n_nodes) + 1) + P + 2 * nw;  // + the two chunk masks per wave
}

int ensure_state(yoda_t* h, uint32_t P) {
  const size_t CP = (size_t)std::max(h->C1 * h->k1_sub, h->C2) * P;
  HIP_TRY(h, h->maxima.ensure(6 * (size_t)P * 8));
  HIP_TRY(h, h->counts.ensure(2 * (size_t)P * 4));
  HIP_TRY(h, h->rcp.ensure(5 * (size_t)P * 8));
  HIP_TRY(h, h->best.ensure((size_t)P * 8));
  HIP_TRY(h, h->idx.ensure((size_t)P * 4));
  HIP_TRY(h, h->ties.ensure((size_t)P * 4));
  HIP_TRY(h, h->lowest.ensure((size_t)P * 8));
  HIP_TRY(h, h->pick.ensure((size_t)P * 4));
  HIP_TRY(h, h->status.ensure((size_t)P * 4));
  HIP_TRY(h, h->ties_out.ensure((size_t)P * 4));
  HIP_TRY(h, h->flagged.ensure((size_t)P * 4));
  HIP_TRY(h, h->n_flagged.ensure(16));
  // [wave][node] u64 masks (yoda_layout.h), +8 words: K2 reads masks in groups of 8
  HIP_TRY(h, h->bitmask.ensure(((size_t)(P + 63) / 64 * bm_row(h->n_nodes) + 8) * 8));
  // the block list [waves][blk_row], the K2 pruning seeds [waves] (PodParams::seed), the shared
  // per-pod best [P] (PodParams::gbest): blk_words(P) u64, all cleared before each block K1
  HIP_TRY(h, h->blk.ensure(blk_words(h, P) * 8));
  HIP_TRY(h, h->bsum.ensure((size_t)(P + 63) / 64 * bs_row(h->n_nodes) * sizeof(BlockMask)));
  HIP_TRY(h, h->p_max_u.ensure(6 * CP * 8));
  if (h->generic) {
    HIP_TRY(h, h->p_best_i.ensure(CP * 8));
    HIP_TRY(h, h->p_low_i.ensure(CP * 8));
    HIP_TRY(h, h->p_err.ensure(CP * 4));
  }
  HIP_TRY(h, h->p_best_f.ensure(CP * 8));
  HIP_TRY(h, h->p_low_f.ensure(CP * 8));
  HIP_TRY(h, h->p_cnt.ensure(2 * CP * 4));
  HIP_TRY(h, h->p_idx.ensure(CP * 4));
  HIP_TRY(h, h->p_ties.ensure(CP * 4));
  return YODA_OK;
}

// gtab_aux: [G maxima 6 x u64 | G reciprocals 5 x f64]
constexpr size_t kGTabAuxBytes = 48 + 40;

PodParams pod_params(yoda_t* h) {
  unsigned char* b = (h->ordered ? h->pod_sorted : h->pod_blob).as<unsigned char>();
  const size_t* off = h->ordered ? h->sorted_off : h->pod_off;
  PodParams pp;
  pp.m_f = reinterpret_cast<double*>(b + off[kPodMF]);
  pp.c_f = reinterpret_cast<double*>(b + off[kPodCF]);
  pp.m_u = reinterpret_cast<uint64_t*>(b + off[kPodMU]);
  pp.c_u = reinterpret_cast<uint64_t*>(b + off[kPodCU]);
  pp.m_32 = reinterpret_cast<uint32_t*>(b + off[kPodM32]);
  pp.c_32 = reinterpret_cast<uint32_t*>(b + off[kPodC32]);
  pp.number = reinterpret_cast<uint64_t*>(b + off[kPodNumber]);
  pp.need_mem = reinterpret_cast<uint32_t*>(b + off[kPodNeedMem]);
  pp.need_clk = reinterpret_cast<uint32_t*>(b + off[kPodNeedClk]);
  pp.alpha = reinterpret_cast<double*>(b + off[kPodAlpha]);
  pp.beta = reinterpret_cast<double*>(b + off[kPodBeta]);
  if (h->core_only) pp.m_f = pp.c_f = pp.alpha = pp.beta = nullptr, pp.m_u = pp.c_u = nullptr;
  pp.g = h->has_k2sum ? h->g : GTab{};
  pp.mix = h->path == Path::N32 ? h->kmix.as<uint32_t>() : nullptr;
  pp.x1 = h->path == Path::N32 ? h->kx1.as<uint32_t>() : nullptr;
  pp.one_model = h->path == Path::N32 && h->all_one_model;
  pp.all_uni4 = h->path == Path::N32 && h->all_uni4;
  if (h->path == Path::N32 && h->has_k1sum && h->blksum.p) pp.bsum = h->blksum.as<uint32_t>();
  const bool ub_ok = h->path == Path::N32 && pp.g.tab && !h->kbub_dirty && h->kbub.p;
  if (ub_ok) pp.kbub = h->kbub.as<uint32_t>();
  pp.kbub_exact = ub_ok && !h->kbub_loose;
  // (A/B knobs: YODA_KB_LEVELS=0 / YODA_SEEDS=0 turn the level bounds / the seeds off)
  static const bool lv_env = YODA_KNOB("YODA_KB_LEVELS", 1) != 0;
  static const bool seeds_env = YODA_KNOB("YODA_SEEDS", 1) != 0;
  if (ub_ok && h->kb_levels_ok && lv_env) pp.kb_levels = h->kb_levels.as<uint32_t>();
  // the K2 pruning seeds live after the block list (cleared with it); the block K1 of this run
  // writes them, the argmax K2 of the same run reads them
  // (A/B knobs: YODA_KB_DEC=0 / YODA_GBEST=0 turn the non-G bounds / the shared best off)
  static const bool dec_env = YODA_KNOB("YODA_KB_DEC", 1) != 0;
  static const bool gbest_env = YODA_KNOB("YODA_GBEST", 1) != 0;
  // (the non-G bounds pay on one-model snapshots at K <= 8: config 3's K2 0.32 -> 0.21 ms;
  // on mixed-model nodes and at K = 16 their per-block cost exceeds what they prune -- mixed50
  // K2 1.52 vs 1.29 ms, the config-4 generator 0.64 vs 0.48 ms, profiles/r05/y/ab.txt)
  // (YODA_KB_DEC_GROUPED, A/B knob: 1 = also on mixed fleets in the block-grouped order, whose
  // one-model blocks are whole again; 2 = there at K = 16 too)
  static const uint32_t dec_grouped = YODA_KNOB("YODA_KB_DEC_GROUPED", 1);
  const bool dec_ok = dec_env && (h->all_one_model ? h->K <= 8
                                                    : h->perm_run() && dec_grouped != 0 &&
                                                          (h->K <= 8 || dec_grouped == 2));
  if (ub_ok && dec_ok && h->kbdec.p) pp.kbdec = h->kbdec.as<uint32_t>();
  {
    const size_t nw = (h->n_work + 63) / 64;
    uint64_t* sd = h->blk.as<uint64_t>() + nw * blk_row(h->n_nodes);
    if (seeds_env && ub_ok && h->seeds_valid && h->blk_valid && h->bm_sparse && pp.g.tab)
      pp.seed = sd;
    if (gbest_env && ub_ok && h->blk_fresh) pp.gbest = sd + nw;  // [n_work] after the seeds
    // the chunk masks after the shared best (A/B knob YODA_CMASK=0: every chunk writes)
    static const bool cmask_env = YODA_KNOB("YODA_CMASK", 1) != 0;
    uint64_t* cm = sd + nw + h->n_work;
    if (cmask_env && h->blk_fresh && h->path == Path::N32) {
      if (h->has_k1sum && h->C1 <= kPlainReduceChunks && h->k1_sub == 1) pp.cmask1 = cm;
      if (h->has_k2sum && h->C2 <= kPlainReduceChunks) pp.cmask2 = cm + nw;
    }
  }
  if (ub_ok && h->hot_ok) pp.hot = h->hot.as<uint64_t>();
  if (h->perm_run()) {
    pp.ids = h->perm_ids.as<uint32_t>();
    pp.mix = h->kmix_p.as<uint32_t>();
    pp.x1 = h->kx1_p.as<uint32_t>();
    if (pp.g.tab) pp.g.tab = h->gtab_p.as<uint32_t>();
    pp.bsum = h->blksum_p.p ? h->blksum_p.as<uint32_t>() : nullptr;
    pp.kbub = ub_ok && h->kbub_p.p ? h->kbub_p.as<uint32_t>() : nullptr;
    pp.kbdec = pp.kbub && dec_ok && h->kbdec_p.p ? h->kbdec_p.as<uint32_t>() : nullptr;
    pp.hot = pp.kbub && h->hot_ok ? h->hot_p.as<uint64_t>() : nullptr;
  }
  pp.mt = h->mem_ranks ? h->mt : MemTab{};
  pp.nwords = h->pack16 ? kNarrowWords : kWideWords;
  pp.q32 = h->q32;
  if (h->lpt_active) {
    pp.lpt_w = h->lpt_w.as<uint32_t>();
    if (h->lpt_sorted) pp.lpt_order = h->lpt_order.as<uint32_t>();
    if (h->k1_sorted) pp.k1_order = h->k1_order.as<uint32_t>();
  }
  return pp;
}

Partials partials(yoda_t* h) {
  Partials p;
  p.max_u = h->p_max_u.as<uint64_t>();
  p.cnt = h->p_cnt.as<uint32_t>();
  p.best_f = h->p_best_f.as<double>();
  p.best_i = h->p_best_i.as<int64_t>();
  p.idx = h->p_idx.as<uint32_t>();
  p.ties = h->p_ties.as<uint32_t>();
  p.low_f = h->p_low_f.as<double>();
  p.low_i = h->p_low_i.as<int64_t>();
  p.err = h->p_err.as<uint32_t>();
  return p;
}

// The deferred part of the last pod upload (the arrays past kPodCoreArrays) to the device, on
// the handle's stream, from the pinned staging copy (reused only after stage_event).
constexpr uint64_t kPodF64Clamp = 1ull << 53;  // > every F64-path card field (<= 2^44)

// The staged arrays an upload left for later (rest_lazy): mf / cf from the staged mu / cu,
// alpha = beta = 0 (a batch without Mode B inputs).  Host work on the pool; a private run
// does it after launching its kernels.
void pods_pack_rest(yoda_t* h) {
  if (!h->rest_lazy) return;
  h->rest_lazy = false;
  const uint32_t P = h->n_pods;
  unsigned char* st = static_cast<unsigned char*>(h->pod_stage.p);
  const uint64_t* mu = reinterpret_cast<const uint64_t*>(st + h->pod_off[kPodMU]);
  const uint64_t* cu = reinterpret_cast<const uint64_t*>(st + h->pod_off[kPodCU]);
  double* mf = reinterpret_cast<double*>(st + h->pod_off[kPodMF]);
  double* cf = reinterpret_cast<double*>(st + h->pod_off[kPodCF]);
  double* al = reinterpret_cast<double*>(st + h->pod_off[kPodAlpha]);
  double* be = reinterpret_cast<double*>(st + h->pod_off[kPodBeta]);
  const uint32_t n_thr = std::min<uint32_t>(HostPool::get().size(), std::max(1u, P / 4096));
  const uint32_t per = (P + n_thr - 1) / n_thr;
  auto range = [&](uint32_t t) {
    for (uint32_t p = std::min(P, t * per), e = std::min(P, (t + 1) * per); p < e; ++p) {
      mf[p] = (double)std::min(mu[p], kPodF64Clamp);
      cf[p] = (double)std::min(cu[p], kPodF64Clamp);
      al[p] = be[p] = 0.0;
    }
  };
  if (n_thr > 1) HostPool::get().run(n_thr, range); else range(0);
}

// Make `stream` wait for a copy pods_complete_async issued (every reader of the deferred
// arrays comes through pods_complete).
int pods_join(yoda_t* h) {
  if (!h->rest_join) return YODA_OK;
  h->rest_join = false;
  HIP_TRY(h, hipStreamWaitEvent(h->stream, h->rest_event, 0));
  return YODA_OK;
}

// The deferred part on the copy stream, after what `stream` holds so far (the core copy of
// the upload: the run's kernels do not wait for it); pods_join after the run's launches.
int ensure_copy_stream(yoda_t* h) {
  if (h->copy_stream) return YODA_OK;
  HIP_TRY(h, hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
  HIP_TRY(h, hipEventCreateWithFlags(&h->core_event, hipEventDisableTiming));
  HIP_TRY(h, hipEventCreateWithFlags(&h->rest_event, hipEventDisableTiming));
  return YODA_OK;
}

int pods_complete_async(yoda_t* h) {
  if (h->pod_rest_bytes == 0) return YODA_OK;
  if (!h->copy_stream) return fail(h, YODA_ERR_STATE, "pods_complete_async: no copy stream");
  pods_pack_rest(h);
  unsigned char* st = static_cast<unsigned char*>(h->pod_stage.p);
  // (core_event: recorded after the upload's copy -- the run's kernels are queued since)
  HIP_TRY(h, hipStreamWaitEvent(h->copy_stream, h->core_event, 0));
  HIP_TRY(h, hipMemcpyAsync(h->pod_blob.as<unsigned char>() + h->pod_rest_off, st + h->pod_rest_off,
                            h->pod_rest_bytes, hipMemcpyHostToDevice, h->copy_stream));
  HIP_TRY(h, hipEventRecord(h->stage_event, h->copy_stream));
  HIP_TRY(h, hipEventRecord(h->rest_event, h->copy_stream));
  h->stage_pending = true;
  h->rest_join = true;
  h->pod_rest_bytes = 0;
  return YODA_OK;
}

int pods_complete(yoda_t* h) {
  if (int rc = pods_join(h)) return rc;
  if (h->pod_rest_bytes == 0) return YODA_OK;
  pods_pack_rest(h);
  unsigned char* st = static_cast<unsigned char*>(h->pod_stage.p);
  HIP_TRY(h, hipMemcpyAsync(h->pod_blob.as<unsigned char>() + h->pod_rest_off, st + h->pod_rest_off,
                            h->pod_rest_bytes, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(h, hipEventRecord(h->stage_event, h->stream));
  h->stage_pending = true;
  h->pod_rest_bytes = 0;
  return YODA_OK;
}

int check_ready(yoda_t* h, int mode) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (mode != YODA_MODE_SCV && mode != YODA_MODE_DISKIO)
    return fail(h, YODA_ERR_INVALID_ARG, "mode must be YODA_MODE_SCV or YODA_MODE_DISKIO");
  if (!h->has_nodes) return fail(h, YODA_ERR_NO_NODES, "no node snapshot uploaded");
  if (!h->has_pods) return fail(h, YODA_ERR_NO_PODS, "no pods uploaded");
  if (mode == YODA_MODE_DISKIO && !(h->nodes_diskio && h->pods_diskio))
    return fail(h, YODA_ERR_INVALID_ARG, "Mode B needs node cpu/disk_io and pod rio/rcpu");
  HIP_TRY(h, hipSetDevice(h->device));
  return h->fast_run ? YODA_OK : pods_complete(h);
}

// Batches above this size are sorted (below it a batch fills at most one wave).
constexpr uint32_t kOrderMinPods = 2 * kWave;
// Groups x memory buckets of the counting-sort order (its LDS histogram: 64 KiB); a batch
// with more (clock, number, has-memory) groups takes the radix sort without padding.
constexpr uint32_t kOrderMaxGroups = 16384;

// Sort the batch by its Filter inputs and gather the pod arrays (yoda_order.hip).  Runs on
// the device inside every run, so its cost is part of the measured step.  The counting
// sort (groups built at upload) fills h->n_work sorted positions: n_pad when the run pads
// its groups to whole waves (prepare_run), else n_pods; the radix sort is the fallback for
// batches with too many groups.
int order_pods(yoda_t* h, int mode) {
  const uint32_t P = h->n_pods, W = h->n_work;
  h->ordered = false;
  h->blk_zeroed = false;
  h->maxima_sorted = false;
  if (!h->order_enabled || mode != YODA_MODE_SCV || P < kOrderMinPods || h->n_nodes == 0)
    return YODA_OK;
  const unsigned char* b = h->pod_blob.as<unsigned char>();
  HIP_TRY(h, h->perm.ensure((size_t)W * 4));
  size_t total = 0;
  for (int a = 0; a < kPodArrays; ++a) {
    h->sorted_off[a] = total;
    total += ((size_t)W * kPodArrayBytes[a] + 255) / 256 * 256;
  }
  HIP_TRY(h, h->pod_sorted.ensure(total));
  PermTable t{};
  for (int a = 0; a < kPodArrays; ++a) {
    t.src[t.n] = b + h->pod_off[a];
    t.dst[t.n] = h->pod_sorted.as<unsigned char>() + h->sorted_off[a];
    t.bytes[t.n] = (uint32_t)kPodArrayBytes[a];
    ++t.n;
  }
  // The counting sort's order inside a bucket follows its atomics (not reproducible from
  // one run to the next): only the padded single-handle run uses it.  Every other entry
  // point takes the radix sort, whose order is a function of the batch alone -- shards of
  // one batch on several GPUs must agree on it.
  if (h->count_order) {
    const bool padded = W != P;
    // the block kernels (N32 with both summaries) read 5 of the pod arrays; the rest of the
    // sorted blob is left unwritten and unread
    if (h->path == Path::N32 && h->has_k1sum && h->has_k2sum) {
      const int fast[] = {kPodM32, kPodC32, kPodNumber, kPodNeedMem, kPodNeedClk};
      t.n = 0;
      for (int a : fast) {
        t.src[t.n] = b + h->pod_off[a];
        t.dst[t.n] = h->pod_sorted.as<unsigned char>() + h->sorted_off[a];
        t.bytes[t.n] = (uint32_t)kPodArrayBytes[a];
        ++t.n;
      }
    }
    // the K1 block list is cleared here rather than by a memset in phase 1
    const uint32_t n_zero = h->has_k1sum ? (uint32_t)blk_words(h, W) : 0u;
    h->blk_zeroed = n_zero != 0;
    HIP_TRY(h, h->order_slot.ensure((size_t)P * 4));
    HIP_TRY(h, h->order_bkt.ensure((size_t)P * 4));
    const unsigned char* meta = h->order_meta.as<unsigned char>();
    OrderMeta o;
    o.groups = reinterpret_cast<const uint64_t*>(meta);
    o.gstart = reinterpret_cast<const uint32_t*>(meta + (padded ? h->og_off_start_pad
                                                                : h->og_off_start));
    o.n_groups = h->og_groups;
    o.nb_log2 = h->og_nb_log2;
    o.m_shift = h->og_m_shift;
    if (h->mem_ranks) {  // bucket the rank thresholds (< nf + 3) instead of the values
      uint32_t bits = 0;
      while (bits < 32 && ((uint64_t)(h->mt.nf + 2) >> bits)) ++bits;
      o.m_shift = bits > h->og_nb_log2 ? bits - h->og_nb_log2 : 0;
      o.m32 = reinterpret_cast<const uint32_t*>(b + h->pod_off[kPodM32]);
    }
    HIP_TRY(h, launch_order_count(o, reinterpret_cast<const uint64_t*>(b + h->pod_off[kPodNumber]),
                                  reinterpret_cast<const uint32_t*>(b + h->pod_off[kPodM32]),
                                  reinterpret_cast<const uint32_t*>(b + h->pod_off[kPodC32]),
                                  reinterpret_cast<const uint32_t*>(b + h->pod_off[kPodNeedMem]),
                                  P, h->order_hist.as<uint32_t>(), h->order_bstart.as<uint32_t>(),
                                  h->order_slot.as<uint32_t>(), h->order_bkt.as<uint32_t>(), t,
                                  reinterpret_cast<const uint32_t*>(meta + h->og_off_pad),
                                  padded ? h->og_n_pad_slots : 0u, h->blk.as<uint64_t>(), n_zero,
                                  h->perm.as<uint32_t>(), h->stream));
    h->ordered = true;
    return YODA_OK;
  }
  if (W != P) return fail(h, YODA_ERR_STATE, "padded order without its groups");
  uint32_t kb[3] = {h->key_bits[0], h->key_bits[1], h->key_bits[2]};
  if (h->mem_ranks) {  // the rank thresholds' width (< nf + 3)
    kb[2] = 0;
    while (kb[2] < 32 && ((uint64_t)(h->mt.nf + 2) >> kb[2])) ++kb[2];
  }
  const size_t scratch = order_scratch_bytes(P);
  HIP_TRY(h, h->order_scratch.ensure(scratch));
  HIP_TRY(h, launch_order_pods(reinterpret_cast<const uint64_t*>(b + h->pod_off[kPodNumber]),
                               reinterpret_cast<const uint64_t*>(b + h->pod_off[kPodMU]),
                               reinterpret_cast<const uint64_t*>(b + h->pod_off[kPodCU]),
                               reinterpret_cast<const uint32_t*>(b + h->pod_off[kPodNeedMem]), P,
                               kb,
                               h->og_ok ? reinterpret_cast<const uint64_t*>(
                                              h->order_meta.as<unsigned char>())
                                        : nullptr,
                               h->og_ok ? h->og_groups : 0u, h->order_scratch.p,
                               h->order_scratch.bytes, h->perm.as<uint32_t>(),
                               h->mem_ranks ? reinterpret_cast<const uint32_t*>(
                                                  b + h->pod_off[kPodM32])
                                            : nullptr,
                               h->stream));
  HIP_TRY(h, launch_permute(t, h->perm.as<uint32_t>(), P, false, h->stream));
  h->ordered = true;
  return YODA_OK;
}

// Scatter the per-pod outputs of an ordered run back to the caller's pod order.
int unpermute_outputs(yoda_t* h) {
  const uint32_t P = h->n_pods, W = h->n_work;  // W sorted positions (copies: same values)
  if (!h->ordered || P == 0) return YODA_OK;
  // Scatter every row into a second buffer of the same shape, then swap the two: no copy
  // back (the swapped-out buffers become the next scatter's targets).
  struct Arr {
    DevBuf* buf;
    DevBuf* alt;
    uint32_t rows;
    uint32_t bytes;
  };
  const Arr arrs[] = {{&h->pick, &h->pick_alt, 1, 4},         {&h->status, &h->status_alt, 1, 4},
                      {&h->ties_out, &h->ties_out_alt, 1, 4}, {&h->counts, &h->counts_alt, 2, 4},
                      {&h->best, &h->best_alt, 1, 8},         {&h->maxima, &h->maxima_alt, 6, 8}};
  PermTable t{};
  for (const Arr& a : arrs) {
    // sized like the buffer it is swapped with (no reallocation from one run to the next)
    HIP_TRY(h, a.alt->ensure(std::max(a.buf->bytes, (size_t)a.rows * W * a.bytes)));
    for (uint32_t r = 0; r < a.rows; ++r) {
      t.src[t.n] = a.buf->as<unsigned char>() + (size_t)r * W * a.bytes;
      t.dst[t.n] = a.alt->as<unsigned char>() + (size_t)r * P * a.bytes;
      t.bytes[t.n] = a.bytes;
      ++t.n;
    }
  }
  HIP_TRY(h, launch_permute(t, h->perm.as<uint32_t>(), W, true, h->stream));
  for (const Arr& a : arrs) std::swap(*a.buf, *a.alt);
  return YODA_OK;
}

// Caller-order exchange (yoda_t::xo): rows of a run's sorted-order arrays (n_work positions)
// to the caller's pod order (n_pods) or back.  A sorted position that pads a group is a copy
// of its pod (the same values), so the scatter writes some caller slots twice, identically.
// A run left unordered is already in caller order: plain copies.
struct XArr {
  void* sorted;  // [rows][n_work]
  void* caller;  // [rows][n_pods]
  uint32_t rows, bytes;
};
int xfer(yoda_t* h, bool to_caller, std::initializer_list<XArr> arrs) {
  const uint32_t P = h->n_pods, W = h->n_work;
  if (P == 0) return YODA_OK;
  PermTable t{};
  for (const XArr& a : arrs)
    for (uint32_t r = 0; r < a.rows; ++r) {
      unsigned char* sp = static_cast<unsigned char*>(a.sorted) + (size_t)r * W * a.bytes;
      unsigned char* cp = static_cast<unsigned char*>(a.caller) + (size_t)r * P * a.bytes;
      if (!h->ordered) {
        if (sp != cp)
          HIP_TRY(h, hipMemcpyAsync(to_caller ? cp : sp, to_caller ? sp : cp, (size_t)P * a.bytes,
                                    hipMemcpyDeviceToDevice, h->stream));
        continue;
      }
      if (t.n == kPermArrays) {
        HIP_TRY(h, launch_permute(t, h->perm.as<uint32_t>(), W, to_caller, h->stream));
        t = PermTable{};
      }
      t.src[t.n] = to_caller ? sp : cp;
      t.dst[t.n] = to_caller ? cp : sp;
      t.bytes[t.n] = a.bytes;
      ++t.n;
    }
  if (t.n) HIP_TRY(h, launch_permute(t, h->perm.as<uint32_t>(), W, to_caller, h->stream));
  return YODA_OK;
}

int xo_ensure(yoda_t* h) {
  if (!h->xo) return YODA_OK;
  const size_t P = std::max<uint32_t>(h->n_pods, 1);
  HIP_TRY(h, h->xcnt.ensure(2 * P * 4));
  HIP_TRY(h, h->xbest.ensure(P * 8));
  HIP_TRY(h, h->xidx.ensure(P * 4));
  HIP_TRY(h, h->xties.ensure(P * 4));
  HIP_TRY(h, h->xlow.ensure(P * 8));
  return YODA_OK;
}

// Mode B score levels (yoda_layout.h DiskLevels): t[k] = the largest |d| >= 0 whose score
// trunc(10 - 10*|d|) (algorithm.go:110-111, no FMA: this file builds with -ffp-contract=off)
// is >= k, by bisection over the bit patterns of the non-negative doubles (ordered like their
// values); the score is non-increasing in |d|, so the set is [0, t[k]].
static double diskio_score(double l) {
  volatile double t = 10.0 * l;
  volatile double s = 10.0 - t;
  return s >= 1.0 ? std::trunc((double)s) : 0.0;
}

static const DiskLevels& diskio_levels() {
  static const DiskLevels lv = [] {
    DiskLevels d{};
    d.t[0] = HUGE_VAL;
    d.t[11] = -1.0;
    for (int k = 1; k <= 10; ++k) {
      uint64_t lo = 0, hi = 0x7ff0000000000000ull;  // score(+0) = 10 >= k, score(inf) = 0 < k
      while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        double x;
        std::memcpy(&x, &mid, 8);
        if (diskio_score(x) >= (double)k) lo = mid; else hi = mid;
      }
      std::memcpy(&d.t[k], &lo, 8);
    }
    return d;
  }();
  return lv;
}

// The batch's Mode B pod classes, from the staged (alpha, beta) of the last upload: pods with
// bit-identical (alpha, beta) score every node alike (algorithm.go:105-111).
int ensure_diskio_classes(yoda_t* h) {
  if (h->b_cls_ready) return YODA_OK;
  pods_pack_rest(h);
  const uint32_t P = h->n_pods;
  const unsigned char* st = static_cast<const unsigned char*>(h->pod_stage.p);
  const uint64_t* al = reinterpret_cast<const uint64_t*>(st + h->pod_off[kPodAlpha]);
  const uint64_t* be = reinterpret_cast<const uint64_t*>(st + h->pod_off[kPodBeta]);
  size_t cap = 64;
  while (cap < 2 * (size_t)P) cap <<= 1;
  std::vector<uint32_t> slot(cap, 0xffffffffu);  // class id, or empty
  std::vector<uint64_t> ca, cb;
  std::vector<uint32_t> cls(P);
  for (uint32_t p = 0; p < P; ++p) {
    const uint64_t a = al[p], b = be[p];
    size_t i = (size_t)((a * 0x9e3779b97f4a7c15ull ^ b * 0xc2b2ae3d27d4eb4full) >> 20) & (cap - 1);
    while (slot[i] != 0xffffffffu && !(ca[slot[i]] == a && cb[slot[i]] == b)) i = (i + 1) & (cap - 1);
    if (slot[i] == 0xffffffffu) {
      slot[i] = (uint32_t)ca.size();
      ca.push_back(a);
      cb.push_back(b);
    }
    cls[p] = slot[i];
  }
  const uint32_t D = (uint32_t)ca.size();
  std::vector<uint64_t> cab(2 * (size_t)D);
  std::copy(ca.begin(), ca.end(), cab.begin());
  std::copy(cb.begin(), cb.end(), cab.begin() + D);
  HIP_TRY(h, h->b_cab.ensure(std::max<size_t>(cab.size(), 1) * 8));
  HIP_TRY(h, h->b_cls.ensure(std::max<size_t>(P, 1) * 4));
  HIP_TRY(h, hipMemcpyAsync(h->b_cab.p, cab.data(), cab.size() * 8, hipMemcpyHostToDevice,
                            h->stream));
  HIP_TRY(h, hipMemcpyAsync(h->b_cls.p, cls.data(), (size_t)P * 4, hipMemcpyHostToDevice,
                            h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));  // the host vectors go out of scope
  h->b_ncls = D;
  h->b_cls_ready = true;
  return YODA_OK;
}

// The free levels t_0 = 0 < ... < t_{L-1} = 0xFFFFFFFF of the kbub lv[] bounds (yoda_layout.h):
// the quantiles of the snapshot's real card frees (K2 summary words: values, or memory ranks),
// so that a wave's scv/memory range falls between close levels wherever the cards are.
hipError_t build_kb_levels(yoda_t* h) {
  const uint32_t N = h->n_nodes, K = (uint32_t)h->K, S2 = k2sum_stride(h->K);
  std::vector<uint32_t> f;
  f.reserve((size_t)N * K);
  for (uint32_t n = 0; n < N; ++n) {
    const uint32_t cnt = std::min<uint32_t>((h->host_k2sum[sum_index(n, kS2Meta, S2)] >> 8) & 0xffu, K);
    for (uint32_t t = 0; t < cnt; ++t) f.push_back(h->host_k2sum[sum_index(n, kS2Fs + t, S2)]);
  }
  std::vector<uint32_t> lv(kKbLevels, 0u);
  lv[kKbLevels - 1] = 0xffffffffu;
  if (!f.empty()) {
    for (uint32_t l = 1; l + 1 < kKbLevels; ++l) {  // interior levels: quantiles l / (L - 1)
      const size_t at = (size_t)((double)l / (kKbLevels - 1) * (double)(f.size() - 1));
      std::nth_element(f.begin(), f.begin() + at, f.end());
      lv[l] = f[at];
    }
    std::sort(lv.begin() + 1, lv.end() - 1);
    for (uint32_t l = 1; l + 1 < kKbLevels; ++l)  // strictly increasing above t_0 = 0
      lv[l] = std::max(lv[l], lv[l - 1] + 1u);
  }
  hipError_t e = h->kb_levels.ensure(kKbLevels * 4);
  if (e == hipSuccess)
    e = hipMemcpyAsync(h->kb_levels.p, lv.data(), kKbLevels * 4, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);  // (lv goes out of scope)
  if (e == hipSuccess) h->kb_levels_ok = true;
  return e;
}

// The K2 block bounds of both orders from the current K2 summaries and G tables.
hipError_t build_block_ub(yoda_t* h) {
  hipError_t e = hipSuccess;
  if (!(h->path == Path::N32 && h->has_k2sum && h->gtab.p)) return e;
  if (!h->kb_levels_ok && (e = build_kb_levels(h)) != hipSuccess) return e;
  const size_t bytes = sum_words(std::max<uint32_t>((h->n_nodes + 63) / 64, 1),
                                 kbub_stride(h->K)) * 4;  // tiles of 64 blocks
  const size_t dbytes = sum_words(std::max<uint32_t>((h->n_nodes + 63) / 64, 1),
                                  kbdec_stride()) * 4;
  const MemTab mt = h->mem_ranks ? h->mt : MemTab{};
  e = h->kbub.ensure(bytes);
  if (e == hipSuccess) e = h->kbdec.ensure(dbytes);
  if (e == hipSuccess)
    e = launch_block_ub(h->K, h->k2sum.as<uint32_t>(), h->gtab.as<uint32_t>(), h->n_nodes,
                        h->kbub.as<uint32_t>(), h->kb_levels.as<uint32_t>(), h->stream);
  if (e == hipSuccess)
    e = launch_block_dec(h->K, h->k2sum.as<uint32_t>(), h->kmix.as<uint32_t>(), h->n_nodes,
                         h->kbdec.as<uint32_t>(),
                         h->kb_levels.as<uint32_t>(), mt, h->stream);
  if (e == hipSuccess && h->perm_on) {
    e = h->kbub_p.ensure(bytes);
    if (e == hipSuccess) e = h->kbdec_p.ensure(dbytes);
    if (e == hipSuccess)
      e = launch_block_ub(h->K, h->k2sum_p.as<uint32_t>(), h->gtab_p.as<uint32_t>(), h->n_nodes,
                          h->kbub_p.as<uint32_t>(), h->kb_levels.as<uint32_t>(), h->stream);
    if (e == hipSuccess)
      e = launch_block_dec(h->K, h->k2sum_p.as<uint32_t>(), h->kmix_p.as<uint32_t>(), h->n_nodes,
                           h->kbdec_p.as<uint32_t>(),
                           h->kb_levels.as<uint32_t>(), mt, h->stream);
  }
  if (e == hipSuccess) {
    h->kbub_dirty = h->kbub_loose = false;
    // the static scores the bounds hold (the host copy of the K2 summaries' static words)
    const uint32_t N = h->n_nodes, S2 = k2sum_stride(h->K);
    h->ub_stat.resize(N);
    for (uint32_t n = 0; n < N; ++n) {
      const uint64_t b = (uint64_t)h->host_k2sum[sum_index(n, kS2Static, S2)] |
                         ((uint64_t)h->host_k2sum[sum_index(n, kS2Static + 1, S2)] << 32);
      double d;
      std::memcpy(&d, &b, 8);
      h->ub_stat[n] = (uint64_t)d;
    }
  }
  return e;
}

// Inside a greedy batch: its node-state pushes leave the block summaries' bounds valid (the
// atomics of k_set_static), so its windows do not tighten them; the next private run does.
struct GreedyScope {
  yoda_t* h;
  bool prev;
  explicit GreedyScope(yoda_t* x) : h(x), prev(x->greedy_active) { h->greedy_active = true; }
  ~GreedyScope() { h->greedy_active = prev; }
};

// The block summaries' CardNumber bounds, tight again after node-state pushes.
hipError_t tighten_block_sums(yoda_t* h) {
  hipError_t e = hipSuccess;
  const uint32_t bsw = bsum_stride(h->K) / 4u;
  if (h->path == Path::N32 && h->has_k1sum && h->blksum.p)
    e = launch_bsum_cn(h->k1sum.as<unsigned char>(), k1sum_stride(h->K), h->n_nodes,
                       h->blksum.as<uint32_t>(), bsw, h->stream);
  if (e == hipSuccess && h->perm_on && h->blksum_p.p)
    e = launch_bsum_cn(h->k1sum_p.as<unsigned char>(), k1sum_stride(h->K), h->n_nodes,
                       h->blksum_p.as<uint32_t>(), bsw, h->stream);
  if (e == hipSuccess) h->blksum_loose = false;
  return e;
}

// Whose PreScore maxima a phase 1 produces.  (The K2 pruning seeds are scores under this
// handle's G table, lower bounds only for pods whose maxima are at most G's: exchanged maxima
// can exceed a shard's G, so the argmax K2 checks each wave's reciprocals against G's before
// it takes a seed -- tests/test_gpu_shard_seeds.py.)
enum class Maxima {
  Exchanged,  // a node shard: the maxima are reduced across shards after this phase
  Own,        // this handle's maxima are the run's (score rows, greedy windows)
  OwnFinal,   // ... and the reduce writes the reciprocals too (yoda_run)
};

// Phase 1: Filter + PreScore maxima (Mode A), or the all-feasible state (Mode B).
int phase1(yoda_t* h, int mode, uint64_t* maxima, uint32_t* counts,
           Maxima whose = Maxima::Exchanged) {
  const bool final_maxima = whose == Maxima::OwnFinal;
  h->seeds_valid = false;  // (set again below when this run's block K1 writes them)
  h->rcp_ready = false;
  const uint32_t P = h->n_work;  // sorted positions of this run
  if (P == 0) return YODA_OK;
  if (mode == YODA_MODE_DISKIO) {
    HIP_TRY(h, launch_fill_diskio_state(P, h->n_nodes, maxima, counts, h->stream));
    return YODA_OK;
  }
  if (h->n_nodes == 0) {
    HIP_TRY(h, hipMemsetAsync(counts, 0, 2 * (size_t)P * 4, h->stream));
    std::vector<uint64_t> ones(6 * (size_t)P, 1);
    HIP_TRY(h, hipMemcpyAsync(maxima, ones.data(), ones.size() * 8, hipMemcpyHostToDevice,
                              h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return YODA_OK;
  }
  Partials part = partials(h);
  hipEvent_t e0 = h->profiling ? h->next_event() : nullptr;
  hipEvent_t e1 = h->profiling ? h->next_event() : nullptr;
  h->blk_valid = h->has_k1sum;
  h->bm_sparse = h->has_k1sum;  // the block K1 writes the sparse form
  h->seeds_valid = h->has_k1sum && mode == YODA_MODE_SCV;
  h->blk_fresh = h->has_k1sum;  // (the memset below or the order scatter clears it whole)
  if (h->blk_valid && !h->blk_zeroed)  // (the list and the seeds after it)
    HIP_TRY(h, hipMemsetAsync(h->blk.p, 0, blk_words(h, P) * 8, h->stream));
  h->blk_zeroed = false;
  const bool pr = h->perm_run();  // block-grouped node order (upload's node_perm)
  // current block bounds for the K1's seeds (loose ones -- static scores fell since the build --
  // are upper bounds only): a private run (yoda_run) rebuilds them here rather than in phase 2;
  // the other entry points (shards, greedy windows) keep phase 2's rule
  if (mode == YODA_MODE_SCV && h->count_order && !h->greedy_active &&
      (h->kbub_dirty || h->kbub_loose) && h->path == Path::N32 && h->has_k2sum && h->g.tab)
    HIP_TRY(h, build_block_ub(h));
  if (h->blksum_loose && !h->greedy_active) HIP_TRY(h, tighten_block_sums(h));
  // the block K1 visits its pod blocks heaviest first too (k1_probe: the per-node work its
  // whole-block decisions leave each wave on a sample of blocks; YODA_K1_LPT=0: launch order)
  static const bool k1_lpt_env = YODA_KNOB("YODA_K1_LPT", 1) != 0;
  h->k1_sorted = false;
  if (k1_lpt_env && h->lpt_active && h->k1_sub == 1u && mode == YODA_MODE_SCV) {
    const PodParams pp0 = pod_params(h);
    if (pp0.bsum != nullptr) {
      const uint32_t n_pb = (P + kBlock - 1) / kBlock;
      HIP_TRY(h, h->k1_w.ensure((size_t)((P + 63) / 64) * 4));
      HIP_TRY(h, h->k1_order.ensure((size_t)n_pb * 4));
      HIP_TRY(h, launch_k1_order(h->K, pp0, P, h->n_nodes, h->k1_w.as<uint32_t>(),
                                 h->k1_order.as<uint32_t>(), h->stream));
      h->k1_sorted = true;
    }
  }
  // (the K1 profile events bracket the K1 launch alone, as rocprofv3's kernel trace does)
  if (e0) HIP_TRY(h, hipEventRecord(e0, h->stream));
  HIP_TRY(h, launch_k1(h->K, h->path, h->nodes.as<unsigned char>(),
                       h->has_k1sum ? (pr ? h->k1sum_p : h->k1sum).as<unsigned char>() : nullptr,
                       (pr ? h->k2sum_p : h->k2sum).as<unsigned char>(),
                       (pr ? h->kmix_p : h->kmix).as<unsigned char>(), h->n_nodes,
                       h->chunk1, h->C1, pod_params(h), P, part, h->bitmask.as<uint64_t>(),
                       bm_row(h->n_nodes), h->bsum.as<BlockMask>(), bs_row(h->n_nodes),
                       h->blk.as<uint64_t>(), blk_row(h->n_nodes), h->stats_ptr(), h->stream,
                       h->k1_sub));
  if (h->class_stats && h->has_k1sum) h->stats_pairs1 += (uint64_t)(P + 63) / 64 * h->n_nodes;
  if (e1) {
    HIP_TRY(h, hipEventRecord(e1, h->stream));
    h->ev_k1.emplace_back(e0, e1);
  }
  // the block-classified K1 (N32) writes u32 maxima partials; a single-handle run's maxima
  // are final, so the reduce writes the reciprocals too (phase 2 then skips k_prep2)
  const bool rcp = final_maxima && !h->generic;
  HIP_TRY(h, launch_reduce1(part, h->C1, P, h->has_k1sum ? pod_params(h).nwords : 0u, maxima,
                            counts,
                            rcp ? h->rcp.as<double>() : nullptr, pod_params(h).mt, h->stream,
                            h->lpt_active ? h->lpt_w.as<uint32_t>() : nullptr,
                            h->lpt_active ? h->lpt_order.as<uint32_t>() : nullptr,
                            h->has_k1sum ? pod_params(h).cmask1 : nullptr));
  h->lpt_sorted = h->lpt_active;  // (the order of this run's pod blocks, for phase 2)
  h->rcp_ready = rcp;
  return YODA_OK;
}

// Phase 1 of a capacity-decrement greedy window: Filter + PreScore maxima with their
// witnesses (k1_witness), dense masks.  Outputs maxima [6][P], counts [2][P] and
// wit [2][6][P] (witness count, lowest witness node + node_offset), in the run's pod order.
int phase1_witness(yoda_t* h, uint64_t* maxima, uint32_t* counts, uint32_t* wit,
                   uint32_t node_offset) {
  const uint32_t P = h->n_pods, N = h->n_nodes;
  if (P == 0) return YODA_OK;
  h->bm_sparse = false;
  h->blk_valid = false;
  h->seeds_valid = false;
  h->blk_fresh = false;
  if (N == 0) {
    HIP_TRY(h, hipMemsetAsync(counts, 0, 2 * (size_t)P * 4, h->stream));
    HIP_TRY(h, hipMemsetAsync(wit, 0, 6 * (size_t)P * 4, h->stream));
    HIP_TRY(h, hipMemsetAsync(wit + 6 * (size_t)P, 0xff, 6 * (size_t)P * 4, h->stream));
    std::vector<uint64_t> ones(6 * (size_t)P, 1);
    HIP_TRY(h, hipMemcpyAsync(maxima, ones.data(), ones.size() * 8, hipMemcpyHostToDevice,
                              h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return YODA_OK;
  }
  // (the witness K1s run one wave per node range: chunk1 nodes each, C1 * k1_sub of them)
  uint32_t C = h->C1 * h->k1_sub;
  HIP_TRY(h, h->p_wit.ensure(12 * (size_t)C * P * 4));
  Partials part = partials(h);
  static const bool block_wit = YODA_KNOB("YODA_BLOCK_WITNESS", 1) != 0;
  if (block_wit && h->path == Path::N32 && h->has_k1sum && h->has_k2sum && h->all_one_model) {
    // block-classified, like phase 1's K1: sparse masks and the block list for the window's K2.
    // Its per-(wave, chunk) epilogue (18 wave reductions, 104 B of partials a pod) is the
    // cost that grows with the chunk count: chunks of >= YODA_WIT_CHUNK_NODES nodes
    static const uint32_t wit_chunk = std::max<uint32_t>(
        kChunkAlign, YODA_KNOB("YODA_WIT_CHUNK_NODES", 64) / kChunkAlign * kChunkAlign);
    uint32_t chunk = h->chunk1;
    if (chunk < wit_chunk) {
      chunk = wit_chunk;
      C = std::max<uint32_t>(1, (N + chunk - 1) / chunk);
      if (C >= 8) C = (C + 7) / 8 * 8;  // XCD tiling; trailing chunks may be empty
    }
    h->bm_sparse = true;
    h->blk_valid = true;
    h->blk_fresh = true;
    HIP_TRY(h, hipMemsetAsync(h->blk.p, 0, blk_words(h, P) * 8, h->stream));
    HIP_TRY(h, launch_k1_block_witness(h->K, h->nodes.as<unsigned char>(),
                                       h->k1sum.as<unsigned char>(), h->k2sum.as<unsigned char>(),
                                       h->kmix.as<unsigned char>(), N, chunk, C,
                                       pod_params(h), P, part.max_u, h->p_wit.as<uint32_t>(),
                                       part.cnt, h->bitmask.as<uint64_t>(), bm_row(N),
                                       h->bsum.as<BlockMask>(), bs_row(N), h->blk.as<uint64_t>(),
                                       blk_row(N), h->stream));
  } else {
    HIP_TRY(h, launch_k1_witness(h->K, h->path, h->nodes.as<unsigned char>(), N, h->chunk1, C,
                                 pod_params(h), P, part.max_u, h->p_wit.as<uint32_t>(), part.cnt,
                                 h->bitmask.as<uint64_t>(), bm_row(N), h->stream));
  }
  HIP_TRY(h, launch_reduce_wit(part.max_u, h->p_wit.as<uint32_t>(), part.cnt, C, P,
                               node_offset, maxima, counts, wit, wit + 6 * (size_t)P, pod_params(h).mt, h->stream));
  return YODA_OK;
}

// Phase 2: Score over the feasible nodes with the (globally reduced) maxima.
// counts: the pods' feasible-node counts ([P] prefix of phase 1's [2][P], local or reduced;
// NULL: unknown): a pod with none takes no part in the block K2's wave bounds.
int phase2(yoda_t* h, int mode, const uint64_t* maxima, const uint32_t* counts, int64_t* best,
           uint32_t* idx, uint32_t* ties, int64_t* low, int64_t* rows = nullptr) {
  const uint32_t P = h->n_work;  // sorted positions of this run
  if (P == 0) return YODA_OK;
  const uint64_t* cmask2 = nullptr;
  if (h->n_nodes == 0) {
    std::vector<int64_t> neg(P, -1), big(P, INT64_MAX);
    std::vector<uint32_t> none(P, 0xffffffffu);
    HIP_TRY(h, hipMemcpyAsync(best, neg.data(), (size_t)P * 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(h, hipMemcpyAsync(low, big.data(), (size_t)P * 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(h, hipMemcpyAsync(idx, none.data(), (size_t)P * 4, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(h, hipMemsetAsync(ties, 0, (size_t)P * 4, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return YODA_OK;
  }
  Partials part = partials(h);
  bool is_f64 = true;
  hipEvent_t e0 = h->profiling ? h->next_event() : nullptr;
  hipEvent_t e1 = h->profiling ? h->next_event() : nullptr;
  if (mode == YODA_MODE_SCV && !h->generic && !h->rcp_ready)
    HIP_TRY(h, launch_prep2(maxima, P, h->rcp.as<double>(),  h->stream));
  h->rcp_ready = false;
  if (mode == YODA_MODE_DISKIO && !rows) {
    // batch path: over the batch's pod classes, then each pod takes its class's outcome
    // (Mode B runs are never reordered: P == n_pods, caller order)
    int rc = ensure_diskio_classes(h);
    if (rc) return rc;
    if ((uint64_t)h->n_nodes >> kDiskCountBits)
      return fail(h, YODA_ERR_INVALID_ARG, "Mode B batch: more than 2^28 nodes");
    const uint32_t D = h->b_ncls;
    const DiskPlan pl = diskio_plan(h->n_nodes, D);
    HIP_TRY(h, h->b_part.ensure(2 * (size_t)pl.C * D * 4));
    uint32_t* plc = h->b_part.as<uint32_t>();
    uint32_t* pix = plc + (size_t)pl.C * D;
    if (e0) HIP_TRY(h, hipEventRecord(e0, h->stream));
    HIP_TRY(h, launch_k2b(h->nodes_b.as<NodeRecB>(), h->n_nodes, h->b_cab.as<double>(), D,
                          diskio_levels(), pl, plc, pix, h->stream));
    if (e1) {
      HIP_TRY(h, hipEventRecord(e1, h->stream));
      h->ev_k2.emplace_back(e0, e1);
    }
    HIP_TRY(h, launch_reduce2b(plc, pix, pl.C, D, h->b_cls.as<uint32_t>(), P, h->node_offset,
                               best, idx, ties, low, h->stream));
    return YODA_OK;
  }
  if (mode == YODA_MODE_SCV && !rows && (h->kbub_dirty || (h->kbub_loose && !h->greedy_active)) &&
      h->path == Path::N32 && h->has_k2sum && h->g.tab)
    HIP_TRY(h, build_block_ub(h));
  if (e0) HIP_TRY(h, hipEventRecord(e0, h->stream));
  uint32_t C2 = h->C2;
  if (mode == YODA_MODE_DISKIO) {
    // score rows (the plugin's row per cycle, small P): lane = node over 256-node chunks
    C2 = (h->n_nodes + kBlock - 1) / kBlock;
    const size_t cp = (size_t)C2 * P;
    HIP_TRY(h, h->p_best_f.ensure(cp * 8));
    HIP_TRY(h, h->p_low_f.ensure(cp * 8));
    HIP_TRY(h, h->p_idx.ensure(cp * 4));
    HIP_TRY(h, h->p_ties.ensure(cp * 4));
    part = partials(h);
    HIP_TRY(h, launch_k2b_rows(h->nodes_b.as<NodeRecB>(), h->n_nodes, pod_params(h), P, part,
                               rows, h->stream));
  } else {
    // the block argmax K2 (N32 with summaries) marks the chunks it wrote (PodParams::cmask2)
    if (h->path == Path::N32 && h->has_k2sum && !rows) cmask2 = pod_params(h).cmask2;
    HIP_TRY(h, launch_k2(h->K, h->path, h->nodes.as<unsigned char>(),
                         h->has_k2sum ? (h->perm_run() ? h->k2sum_p : h->k2sum)
                                            .as<unsigned char>()
                                      : nullptr,
                         h->blk_valid ? h->blk.as<uint64_t>() : nullptr, blk_row(h->n_nodes),
                         h->n_nodes,
                         h->chunk2, h->C2, pod_params(h), maxima, h->rcp.as<double>(),
                          P, h->bitmask.as<uint64_t>(), bm_row(h->n_nodes),
                         h->bs_ptr(), bs_row(h->n_nodes), part, rows, h->stats_ptr(), counts,
                         h->stream));
    if (h->class_stats && h->has_k2sum && !rows)
      h->stats_pairs2 += (uint64_t)(P + 63) / 64 * h->n_nodes;
    is_f64 = !h->generic;
    // the shared best and the chunk masks hold this K2's scores: a later phase 2 on the same
    // phase 1 (other maxima) must not read them
    if (!rows) h->blk_fresh = false;
  }
  if (e1) {
    HIP_TRY(h, hipEventRecord(e1, h->stream));
    h->ev_k2.emplace_back(e0, e1);
  }
  // the block K2 (N32 with summaries, argmax) writes no lowest scores: the
  // merge reports each pod's best in their place
  Partials pr = part;
  if (mode == YODA_MODE_SCV && h->path == Path::N32 && h->has_k2sum && !rows) pr.low_f = nullptr;
  HIP_TRY(h, launch_reduce2(pr, C2, P, is_f64, h->node_offset, best, idx, ties, low,
                            h->stream, cmask2));
  return YODA_OK;
}

// Finalize into the handle's pick/status/ties; runs K3 for generic-path overflow pods.
int finalize(yoda_t* h, int mode, const uint32_t* counts, const int64_t* best,
             const uint32_t* idx, const uint32_t* ties, const int64_t* low, bool sharded) {
  const uint32_t P = h->n_work;  // sorted positions of this run
  h->k3_pending = false;
  if (P == 0) return YODA_OK;
  const bool generic = h->generic && mode == YODA_MODE_SCV;
  // the overflow count is written by the generic path only: clear it for those runs, and
  // once after one (yoda_shard_overflow_count reads it)
  if (generic || h->flagged_dirty) HIP_TRY(h, hipMemsetAsync(h->n_flagged.p, 0, 4, h->stream));
  h->flagged_dirty = generic;
  if (h->ordered && !generic) {
    // one kernel: the outputs computed and scattered to the caller's pod order into the
    // *_alt buffers, then swapped in (as unpermute_outputs would)
    const uint32_t Pc = h->n_pods;
    // (the maxima -- 48 B a pod, read only by yoda_download -- stay in sorted order until a
    // download asks for them: h->maxima_sorted)
    DevBuf* pairs[][2] = {{&h->pick, &h->pick_alt},         {&h->status, &h->status_alt},
                          {&h->ties_out, &h->ties_out_alt}, {&h->counts, &h->counts_alt},
                          {&h->best, &h->best_alt}};
    for (auto& pr : pairs) HIP_TRY(h, pr[1]->ensure(pr[0]->bytes));
    FinalScatter sc{h->perm.as<uint32_t>(), Pc, h->counts_alt.as<uint32_t>(),
                    h->best_alt.as<int64_t>(), nullptr, nullptr};
    HIP_TRY(h, launch_finalize(counts, best, idx, ties, low, P, false, h->pick_alt.as<int32_t>(),
                               h->status_alt.as<int32_t>(), h->ties_out_alt.as<uint32_t>(),
                               h->flagged.as<uint32_t>(), h->n_flagged.as<uint32_t>(), sc,
                               h->stream));
    for (auto& pr : pairs) std::swap(*pr[0], *pr[1]);
    h->maxima_sorted = true;
    return YODA_OK;
  }
  const FinalScatter none{};
  HIP_TRY(h, launch_finalize(counts, best, idx, ties, low, P, generic, h->pick.as<int32_t>(),
                             h->status.as<int32_t>(), h->ties_out.as<uint32_t>(),
                             h->flagged.as<uint32_t>(), h->n_flagged.as<uint32_t>(), none,
                             h->stream));
  if (generic) {
    uint32_t nfl = 0;
    HIP_TRY(h, hipMemcpyAsync(&nfl, h->n_flagged.p, 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (nfl > 0) {
      Partials part = partials(h);
      HIP_TRY(h, launch_k3(h->K, h->nodes.as<unsigned char>(), h->n_nodes, h->chunk2, h->C2,
                           pod_params(h), h->maxima.as<uint64_t>(), P, h->bitmask.as<uint64_t>(),
                           bm_row(h->n_nodes),
                           h->flagged.as<uint32_t>(), h->n_flagged.as<uint32_t>(), best, low,
                           part, nfl, h->stream));
      if (sharded) {
        // over this shard's nodes only: per-pod records, merged across the shards by
        // yoda_shard_exact_merge (the flagged set is the same on every shard: it depends on
        // the reduced counts, best and lowest only)
        HIP_TRY(h, h->k3rec.ensure((size_t)P * sizeof(ShardRec)));
        HIP_TRY(h, launch_reduce3_rec(part, h->C2, h->flagged.as<uint32_t>(),
                                      h->n_flagged.as<uint32_t>(), nfl, h->node_offset,
                                      h->k3rec.as<ShardRec>(), h->stream));
        h->k3_pending = true;
        h->k3_nfl = nfl;
        return YODA_OK;  // outputs stay in sorted order until the merge
      }
      HIP_TRY(h, launch_reduce3(part, h->C2, h->flagged.as<uint32_t>(), h->n_flagged.as<uint32_t>(),
                                nfl, h->node_offset, h->pick.as<int32_t>(), h->status.as<int32_t>(),
                                h->ties_out.as<uint32_t>(), h->stream));
    }
  }
  return unpermute_outputs(h);
}

// Top-k candidate lists of the run's P sorted pods (greedy windows, yoda_shard_topk) into
// h->tk_s / h->tk_i ([KT][P], scores and global node ids, (score desc, node asc)), after
// phase 1 and the reciprocals.  The block-classified K2 with packed keys whenever the record
// path and the score bound allow it (its own chunking: one round of workgroups, so that the
// [C][P][KT] lists stay small); else the per-pair K2 (k2_score OUT_TOPK).
// YODA_TOPK_PER_PAIR=1 forces the per-pair kernels (A/B, tests).
// The block-classified top-k K2 with packed keys serves this snapshot (else the per-pair one).
bool topk_block_ok(const yoda_t* h) {
  static const bool per_pair = YODA_KNOB("YODA_TOPK_PER_PAIR", 0) == 1;
  uint32_t ib = 1;
  while ((1ull << ib) <= h->n_nodes) ++ib;
  return !per_pair && h->path == Path::N32 && h->has_k2sum && h->K <= 8 && ib <= 40 &&
         h->score_bound < (1ull << (64 - ib));
}

// deep > KT (the capacity windows, block kernels only): the chunks' KT-deep lists merged into
// `deep`-deep lists exact as far as they reach (k_topk_merge_deep; entries past that empty);
// *depth_out: the depth written (deep, or KT where the block kernels do not run).
int topk_lists(yoda_t* h, uint32_t P, uint32_t KT, const uint32_t* d_counts, uint32_t deep = 0,
               uint32_t* depth_out = nullptr) {
  const uint32_t N = h->n_nodes;
  if (depth_out) *depth_out = KT;
  const uint32_t KD = std::max(KT, deep);
  HIP_TRY(h, h->tk_s.ensure((size_t)KD * P * 8));
  HIP_TRY(h, h->tk_i.ensure((size_t)KD * P * 4));
  if (P == 0 || N == 0) return YODA_OK;
  uint32_t ib = 1;
  while ((1ull << ib) <= N) ++ib;  // node ids < 2^ib - 1: a real key is never 0
  const bool block = topk_block_ok(h);
  if (block) {
    uint32_t Ct = 1, cht = 64;
    // rounds of resident workgroups: 4 for window-sized batches (more, shorter per-(wave,
    // chunk) lists balance better), 1 below 2048 pods (the capacity windows, where the merge's
    // reads dominate); A/B in profiles/r02/greedy_topk/
    static const uint32_t rt_env = YODA_KNOB("YODA_TOPK_ROUNDS", 0);
    const uint32_t rt = rt_env ? rt_env : (P >= 2048 ? 4u : 1u);
    plan_chunks_for((uint32_t)capacity(h, 2, YODA_MODE_SCV), rt, P, N, &Ct, &cht);
    // YODA_TOPK_MIN_CHUNK (A/B knob): chunks of at least that many nodes -- fewer per-(wave,
    // chunk) lists to write and merge in small windows
    static const uint32_t tk_min = YODA_KNOB("YODA_TOPK_MIN_CHUNK", 0);
    if (tk_min && cht < tk_min) {
      cht = (tk_min + kChunkAlign - 1) / kChunkAlign * kChunkAlign;
      Ct = std::max<uint32_t>(1, (N + cht - 1) / cht);
      if (Ct >= 8) Ct = (Ct + 7) / 8 * 8;
    }
    HIP_TRY(h, h->tk_s_part.ensure((size_t)Ct * P * KT * 8));
    // the chunks' shared k-th keys start empty at every list pass (a mid-window refresh scores
    // a later node state, whose keys are lower: the last pass's would be too high)
    PodParams pp = pod_params(h);
    // (A/B knobs: YODA_TOPK_GBEST=0 / YODA_TOPK_DEC=0 -- the shared k-th keys / the non-G
    // bounds in the list passes)
    // (both off by default: the capacity windows ran 1.51 s without them, 1.58 s with them,
    // profiles/r05/g)
    static const bool tk_gbest = YODA_KNOB("YODA_TOPK_GBEST", 0) != 0;
    static const bool tk_dec = YODA_KNOB("YODA_TOPK_DEC", 0) != 0;
    if (!tk_gbest) pp.gbest = nullptr;
    if (!tk_dec) pp.kbdec = nullptr;
    if (pp.gbest) HIP_TRY(h, hipMemsetAsync(pp.gbest, 0, (size_t)P * 8, h->stream));
    HIP_TRY(h, launch_k2_topk_block(h->K, h->nodes.as<unsigned char>(),
                                    h->k2sum.as<unsigned char>(),
                                    h->blk_valid ? h->blk.as<uint64_t>() : nullptr, blk_row(N), N,
                                    cht, Ct, pp, h->rcp.as<double>(),
                                     P, h->bitmask.as<uint64_t>(), bm_row(N),
                                    h->bs_ptr(), bs_row(N), d_counts,
                                    h->tk_s_part.as<uint64_t>(), ib, (int)KT, h->stream));
    if (deep > KT) {
      HIP_TRY(h, launch_topk_merge_deep(h->tk_s_part.as<uint64_t>(), Ct, P, ib, h->node_offset,
                                        h->tk_s.as<double>(), h->tk_i.as<uint32_t>(), (int)KT,
                                        (int)deep, h->stream));
      if (depth_out) *depth_out = deep;
      return YODA_OK;
    }
    HIP_TRY(h, launch_topk_merge_keys(h->tk_s_part.as<uint64_t>(), Ct, P, ib, h->node_offset,
                                      h->tk_s.as<double>(), h->tk_i.as<uint32_t>(), (int)KT,
                                      h->stream));
    return YODA_OK;
  }
  const size_t CPk = (size_t)h->C2 * KT * P;
  HIP_TRY(h, h->tk_s_part.ensure(CPk * 8));
  HIP_TRY(h, h->tk_i_part.ensure(CPk * 4));
  HIP_TRY(h, launch_k2_topk(h->K, h->path, h->nodes.as<unsigned char>(), N, h->chunk2, h->C2,
                            pod_params(h), h->rcp.as<double>(),  P,
                            h->bitmask.as<uint64_t>(), bm_row(N), h->bs_ptr(), bs_row(N),
                            h->blk_ptr(), blk_row(N), partials(h), h->tk_s_part.as<double>(), h->tk_i_part.as<uint32_t>(),
                            (int)KT, h->stream));
  HIP_TRY(h, launch_topk_merge(h->tk_s_part.as<double>(), h->tk_i_part.as<uint32_t>(), h->C2, P,
                               h->node_offset, h->tk_s.as<double>(), h->tk_i.as<uint32_t>(),
                               (int)KT, h->stream));
  return YODA_OK;
}

bool is_pow2_le16(uint32_t k) { return k == 1 || k == 2 || k == 4 || k == 8 || k == 16; }

}  // namespace

// ======================================================================================
extern "C" {

int yoda_abi_version(void) { return YODA_ABI_VERSION; }

int yoda_create(int device, yoda_t** out) {
  if (!out) return YODA_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return YODA_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return YODA_ERR_NO_DEVICE;
  yoda_t* h = new (std::nothrow) yoda_t();
  if (!h) return YODA_ERR_INVALID_ARG;
  h->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return YODA_ERR_HIP;
  }
  h->stream = h->own_stream;
  if (hipEventCreateWithFlags(&h->stage_event, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->upd_event, hipEventDisableTiming) != hipSuccess) {
    delete h;
    return YODA_ERR_HIP;
  }
  *out = h;
  return YODA_OK;
}

int yoda_destroy(yoda_t* h) {
  if (!h) return YODA_ERR_INVALID_ARG;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  delete h;
  return YODA_OK;
}

const char* yoda_last_error(const yoda_t* h) {
  return h ? h->last_error.c_str() : "null handle";
}

// Switch the handle's stream: work already queued on the old stream (an upload's copies and
// kernels) is ordered before anything queued on the new one (an event wait, no host sync).
static int switch_stream(yoda_t* h, hipStream_t ns) {
  if (ns == h->stream) return YODA_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  if (!h->switch_event)
    HIP_TRY(h, hipEventCreateWithFlags(&h->switch_event, hipEventDisableTiming));
  HIP_TRY(h, hipEventRecord(h->switch_event, h->stream));
  HIP_TRY(h, hipStreamWaitEvent(ns, h->switch_event, 0));
  h->stream = ns;
  return YODA_OK;
}

int yoda_set_stream(yoda_t* h, void* hip_stream) {
  if (!h) return YODA_ERR_INVALID_ARG;
  return switch_stream(h, static_cast<hipStream_t>(hip_stream));
}

int yoda_use_own_stream(yoda_t* h) {
  if (!h) return YODA_ERR_INVALID_ARG;
  return switch_stream(h, h->own_stream);
}

int yoda_synchronize(yoda_t* h) {
  if (!h) return YODA_ERR_INVALID_ARG;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return YODA_OK;
}

int yoda_upload_nodes(yoda_t* h, const yoda_node_soa* nd, uint32_t node_offset, uint32_t flags) {
  if (!h) return YODA_ERR_INVALID_ARG;
  try {
    if (!nd) return fail(h, YODA_ERR_INVALID_ARG, "nodes is NULL");
    const uint32_t N = nd->n_nodes, KS = nd->max_cards;
    h->topk_ready = false;
    if (KS < 1 || KS > YODA_MAX_CARDS)
      return fail(h, YODA_ERR_INVALID_ARG, "max_cards must be in 1..16");
    if (N > 0 && (!nd->card_number || !nd->card_count || !nd->free_memory_sum ||
                  !nd->total_memory_sum || !nd->card_free_memory || !nd->card_total_memory ||
                  !nd->card_clock || !nd->card_bandwidth || !nd->card_core || !nd->card_power ||
                  !nd->card_healthy))
      return fail(h, YODA_ERR_INVALID_ARG, "a required node array is NULL");
    if ((uint64_t)node_offset + N > 0x7fffffffull)
      return fail(h, YODA_ERR_RANGE, "node index exceeds int32");
    HIP_TRY(h, hipSetDevice(h->device));
    uint32_t kmax = 1;
    for (uint32_t i = 0; i < N; ++i) {
      if (nd->card_count[i] > KS) return fail(h, YODA_ERR_INVALID_ARG, "card_count > max_cards");
      kmax = std::max(kmax, nd->card_count[i]);
    }
    const int K = pow2_cards(kmax);
    // Record format: the narrowest exact one.
    std::vector<uint64_t> stat(N);
    std::vector<uint8_t> zt(N);
    uint64_t max_field = 0, max_small = 0, max_clock = 0, max_static = 0, max_mem = 0;
    uint64_t max_ckq = 0;  // the largest clock quotient a card can score
    bool all_one = true;   // every node one GPU model with one TotalMemory
    for (uint32_t i = 0; i < N; ++i) {
      bool z = false;
      const uint64_t alloc = nd->alloc_memory ? nd->alloc_memory[i] : 0;
      stat[i] = static_score(nd->free_memory_sum[i], nd->total_memory_sum[i], alloc, &z);
      zt[i] = z;
      max_static = std::max(max_static, stat[i]);
      for (uint32_t j = 0; j < nd->card_count[i]; ++j) {
        const size_t k = (size_t)i * KS + j;
        max_field = std::max({max_field, nd->card_free_memory[k], nd->card_total_memory[k],
                              nd->card_clock[k], nd->card_bandwidth[k], nd->card_core[k],
                              nd->card_power[k]});
        max_small = std::max({max_small, nd->card_bandwidth[k], nd->card_core[k],
                              nd->card_power[k], nd->card_clock[k]});
        max_mem = std::max({max_mem, nd->card_free_memory[k], nd->card_total_memory[k]});
        max_clock = std::max(max_clock, nd->card_clock[k]);
        // clock / MaxBandwidth (algorithm.go:283): a scored card qualifies, so MaxBandwidth is
        // at least its own bandwidth (and 1)
        if (nd->card_clock[k] <= kN32FieldMax)
          max_ckq = std::max(max_ckq, nd->card_clock[k] * 100u /
                                          std::max<uint64_t>(1, nd->card_bandwidth[k]));
      }
      // one GPU model with one TotalMemory (the mixed-model K1 tiles pack small fields in 16 bits)
      const size_t a = (size_t)i * KS;
      bool one = nd->card_count[i] > 0 && !(flags & YODA_UPLOAD_NO_UNIFORM);
      for (uint32_t j = 1; j < nd->card_count[i] && one; ++j)
        one = nd->card_clock[a + j] == nd->card_clock[a] &&
              nd->card_bandwidth[a + j] == nd->card_bandwidth[a] &&
              nd->card_core[a + j] == nd->card_core[a] && nd->card_power[a + j] == nd->card_power[a] &&
              nd->card_total_memory[a + j] == nd->card_total_memory[a];
      all_one = all_one && one;
    }
    // per-card score <= 800 + 100*clock (five quotients <= 100, clock/MaxBandwidth <= 100*clock)
    const long double score_bound =
        (long double)K * (800.0L + 100.0L * (long double)max_clock) + (long double)max_static;
    const bool f64_ok = max_field <= kFastFieldMax && score_bound < (long double)kFastScoreMax;
    {
      uint64_t max_actual = 0;  // Actual does not depend on the allocated memory
      for (uint32_t i = 0; i < N; ++i)
        if (nd->total_memory_sum[i] != 0)
          max_actual = std::max(max_actual,
                                nd->free_memory_sum[i] * 100u / nd->total_memory_sum[i] * 2u);
      const long double b = (long double)K * (800.0L + 100.0L * (long double)max_clock) + 300.0L +
                            (long double)max_actual;
      h->score_bound = b < 9.0e18L ? (uint64_t)b + 1u : ~0ull;
    }
    // N32: every small card field in u32, every quotient exact in f64 (x, M < 2^32: 300 x + M
    // < 2^53) -- the block K2 keeps the small-field quotients in f32 while those fields are
    // <= kF32SmallMax (q32) -- the card score summed in u32: per card at most 800 + the clock
    // quotient.  Small fields beyond that need one-model nodes (the mixed-model K1 tiles pack
    // them in 16 bits, and the f64 block K2 is instantiated without the mixed-model rows); beyond
    // 16 bits the K1 writes unpacked partial words (kWideWords).  Memory fields beyond 32 bits (e.g.
    // bytes) keep the N32 path with memory RANKS in the u32 fields (yoda_layout.h MemTab):
    // every compare and max is unchanged, the values come back for the quotients and the
    // maxima (all <= 2^44: exact in f64).
    const bool pack16 = max_small <= kPack16Max;
    const bool q32 = max_small <= kF32SmallMax && !(flags & YODA_UPLOAD_F64_QUOTIENTS);
    const bool n32_ok = f64_ok && max_small <= kN32FieldMax && (q32 || all_one) &&
                        (uint64_t)K * (800u + max_ckq) < (1ull << 32);
    Path path = n32_ok ? Path::N32 : (f64_ok ? Path::F64 : Path::U64);
    if ((flags & YODA_UPLOAD_FORCE_F64) && path == Path::N32) path = Path::F64;
    if (flags & YODA_UPLOAD_FORCE_GENERIC) path = Path::U64;
    const bool ranks = path == Path::N32 &&
                       (max_mem > kN32FieldMax || (flags & YODA_UPLOAD_MEM_RANKS) != 0u);
    std::vector<uint64_t> frees, totals;  // distinct values, ascending (ranks)
    if (ranks) {
      for (uint32_t i = 0; i < N; ++i)
        for (uint32_t j = 0; j < nd->card_count[i]; ++j) {
          frees.push_back(nd->card_free_memory[(size_t)i * KS + j]);
          totals.push_back(nd->card_total_memory[(size_t)i * KS + j]);
        }
      for (auto* v : {&frees, &totals}) {
        std::sort(v->begin(), v->end());
        v->erase(std::unique(v->begin(), v->end()), v->end());
      }
    }
    // the u32 code of a card's FreeMemory / TotalMemory: its value, or 2 + its rank
    auto code_f = [&](uint64_t x) -> uint32_t {
      if (!ranks) return (uint32_t)x;
      return 2u + (uint32_t)(std::lower_bound(frees.begin(), frees.end(), x) - frees.begin());
    };
    auto code_t = [&](uint64_t x) -> uint32_t {
      if (!ranks) return (uint32_t)x;
      return 2u + (uint32_t)(std::lower_bound(totals.begin(), totals.end(), x) - totals.begin());
    };
    // Build records.
    const size_t stride = path == Path::N32 ? n32_stride(K) : node_stride(K);
    std::vector<unsigned char> rec((size_t)std::max<uint32_t>(N, 1) * stride, 0);
    // K1 node summaries (N32 path): the facts the block-classified K1 reads per node
    const bool want_sum = path == Path::N32;
    uint32_t g_rcp[10] = {};  // the G table's reciprocals, read back from the device
    const size_t sstride = k1sum_stride(K);
    std::vector<uint32_t> sum(want_sum ? (size_t)std::max<uint32_t>(N, 1) * sstride / 4 : 0, 0);
    const size_t s2stride = k2sum_stride(K);
    std::vector<uint32_t> sum2(want_sum ? (size_t)std::max<uint32_t>(N, 1) * s2stride / 4 : 0, 0);
    const size_t mstride = mix_stride(K);
    std::vector<uint32_t> mix(want_sum ? (size_t)std::max<uint32_t>(N, 1) * mstride / 4 : 0, 0);
    uint32_t n_one_model = 0, n_uni4 = 0;
    // per node: the clocks of its real cards and of its healthy cards, min / max (block sums)
    std::vector<uint32_t> clk_rng(want_sum ? 4 * (size_t)N : 0);
    const size_t xstride = x1_stride(K);
    std::vector<uint32_t> x1m(want_sum ? (size_t)std::max<uint32_t>(N, 1) * xstride / 4 : 0, 0);
    for (uint32_t i = 0; i < N; ++i) {
      unsigned char* r = rec.data() + (size_t)i * stride;
      uint32_t hm = 0;
      for (uint32_t j = 0; j < nd->card_count[i]; ++j)
        if (nd->card_healthy[(size_t)i * KS + j]) hm |= 1u << j;
      NodeHdrG hd{};  // NodeHdrF has the same layout; static_score's bits set below
      hd.card_number = nd->card_number[i];
      hd.healthy_mask = hm;
      hd.zero_total = zt[i];
      const uint32_t cnt = nd->card_count[i];
      hd.real_mask = cnt >= 32 ? 0xffffffffu : ((1u << cnt) - 1u);
      bool uni = cnt > 0;
      for (uint32_t j = 1; j < cnt; ++j) {
        const size_t a = (size_t)i * KS, b = a + j;
        uni = uni && nd->card_clock[b] == nd->card_clock[a] &&
              nd->card_bandwidth[b] == nd->card_bandwidth[a] &&
              nd->card_core[b] == nd->card_core[a] && nd->card_power[b] == nd->card_power[a];
      }
      bool uni_total = uni;
      for (uint32_t j = 1; j < cnt; ++j)
        uni_total = uni_total && nd->card_total_memory[(size_t)i * KS + j] ==
                                     nd->card_total_memory[(size_t)i * KS];
      hd.flags = 0u;
      if (uni && !(flags & YODA_UPLOAD_NO_UNIFORM))
        hd.flags = kNodeUniform4 | (uni_total ? kNodeUniformTotal : 0u);
      n_one_model += (hd.flags & (kNodeUniform4 | kNodeUniformTotal)) ==
                     (kNodeUniform4 | kNodeUniformTotal);
      n_uni4 += (hd.flags & kNodeUniform4) != 0u;
      if (path == Path::U64) {
        hd.static_score = stat[i];
      } else {
        const double sd = (double)stat[i];
        std::memcpy(&hd.static_score, &sd, 8);
      }
      std::memcpy(r, &hd, sizeof(hd));
      if (want_sum) {
        uint32_t* s = sum.data() + (size_t)i * sstride / 4;
        const size_t a = (size_t)i * KS;
        s[kSumCnLo] = (uint32_t)hd.card_number;
        s[kSumCnHi] = (uint32_t)(hd.card_number >> 32);
        s[kSumMeta] = ((hd.flags & kNodeUniform4) ? kSumUni4 : 0u) |
                      ((hd.flags & kNodeUniformTotal) ? kSumUniTotal : 0u) |
                      (zt[i] ? kSumZeroTotal : 0u) | ((uint32_t)__builtin_popcount(hm) << 8);
        if (cnt > 0) {  // the model values of card 0 (all cards under kSumUni4)
          s[kSumClock] = (uint32_t)nd->card_clock[a];
          s[kSumTotal] = code_t(nd->card_total_memory[a]);
          s[kSumBw] = (uint32_t)nd->card_bandwidth[a];
          s[kSumCore] = (uint32_t)nd->card_core[a];
          s[kSumPower] = (uint32_t)nd->card_power[a];
        }
        uint32_t mrf1 = 0, nhf = 0;
        uint32_t hfs[YODA_MAX_CARDS];
        for (uint32_t j = 0; j < cnt; ++j) {  // N32: free <= 0xFFFFFFFE, so free + 1 fits
          const uint32_t f1 = code_f(nd->card_free_memory[a + j]) + 1u;
          mrf1 = std::max(mrf1, f1);
          if (nd->card_healthy[a + j]) hfs[nhf++] = f1;
        }
        std::sort(hfs, hfs + nhf, [](uint32_t x, uint32_t y) { return x > y; });
        s[kSumMrf1] = mrf1;
        for (uint32_t j = 0; j < nhf; ++j) s[kSumHfs + j] = hfs[j];
        // K2 summary: real cards in descending free order (stable: ties keep card order)
        uint32_t* s2 = sum2.data() + (size_t)i * s2stride / 4;
        std::memcpy(s2 + kS2Static, &hd.static_score, 8);  // f64 bits (set above)
        s2[kS2Clock] = s[kSumClock];
        s2[kS2Meta] = ((hd.flags & kNodeUniform4) ? kSumUni4 : 0u) | (cnt << 8);
        s2[kS2Bw] = s[kSumBw];
        s2[kS2Core] = s[kSumCore];
        s2[kS2Power] = s[kSumPower];
        uint32_t ord[YODA_MAX_CARDS];
        for (uint32_t j = 0; j < cnt; ++j) ord[j] = j;
        std::stable_sort(ord, ord + cnt, [&](uint32_t x, uint32_t y) {
          return nd->card_free_memory[a + x] > nd->card_free_memory[a + y];
        });
        uint32_t* mx = mix.data() + (size_t)i * mstride / 4;
        uint32_t minclk = 0xffffffffu, hmf = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
          const size_t b = a + ord[j];
          s2[kS2Fs + j] = code_f(nd->card_free_memory[b]);
          s2[kS2Fs + K + j] = code_t(nd->card_total_memory[b]);
          // the per-card models in the same order (nodes without kSumUni4 read them)
          mx[mix_word(kMixCk, (int)j, K)] = (uint32_t)nd->card_clock[b];
          mx[mix_word(kMixBw, (int)j, K)] = (uint32_t)nd->card_bandwidth[b];
          mx[mix_word(kMixCo, (int)j, K)] = (uint32_t)nd->card_core[b];
          mx[mix_word(kMixPw, (int)j, K)] = (uint32_t)nd->card_power[b];
          if (nd->card_healthy[b]) hmf |= 1u << j;
          minclk = std::min(minclk, (uint32_t)nd->card_clock[b]);
        }
        mx[mix_hm(K)] = hmf;
        s2[kS2MinClk] = minclk;
        // K1 tile (K1MixWord): prefix maxima per 16-bit half, their change bits, the cards
        // packed, the healthy-card counts per distinct clock
        uint32_t* x = x1m.data() + (size_t)i * xstride / 4;
        uint32_t pa = 0, pb = 0, pt = 0, chg = 0, nch = 0;
        auto hmax = [](uint32_t u, uint32_t v) {
          return std::max(u & 0xffffu, v & 0xffffu) | (std::max(u >> 16, v >> 16) << 16);
        };
        for (uint32_t j = 0; j < cnt; ++j) {
          const size_t b = a + ord[j];
          const uint32_t ca = (uint32_t)nd->card_clock[b] | ((uint32_t)nd->card_bandwidth[b] << 16);
          const uint32_t cb = (uint32_t)nd->card_core[b] | ((uint32_t)nd->card_power[b] << 16);
          const uint32_t na = hmax(pa, ca), nb2 = hmax(pb, cb);
          const uint32_t nt = std::max(pt, s2[kS2Fs + K + j]);
          if (j == 0 || na != pa || nb2 != pb || nt != pt) chg |= 1u << (j + 1);
          pa = na;
          pb = nb2;
          pt = nt;
          x[x1_pm((int)j, 0)] = pa;
          x[x1_pm((int)j, 1)] = pb;
          x[x1_pm((int)j, 2)] = pt;
          x[x1_cd((int)j, 0, K)] = ca;
          x[x1_cd((int)j, 1, K)] = cb;
          if (nd->card_healthy[b]) {
            const uint32_t ck = (uint32_t)nd->card_clock[b];
            uint32_t e = 0;
            while (e < nch && (x[kX1Ch + e] & 0xffffu) != ck) ++e;
            if (e == nch) {
              if (nch == 4) {
                chg |= kX1ChgMany;
                continue;
              }
              x[kX1Ch + nch++] = ck;
            }
            x[kX1Ch + e] += 1u << 16;
          }
        }
        x[kX1Chg] = chg;
        uint32_t* cr = clk_rng.data() + 4 * (size_t)i;
        cr[0] = cr[2] = 0xffffffffu;
        cr[1] = cr[3] = 0u;
        for (uint32_t j = 0; j < cnt; ++j) {
          const uint32_t ck = (uint32_t)nd->card_clock[a + j];
          cr[0] = std::min(cr[0], ck);
          cr[1] = std::max(cr[1], ck);
          if (nd->card_healthy[a + j]) {
            cr[2] = std::min(cr[2], ck);
            cr[3] = std::max(cr[3], ck);
          }
        }
      }
      for (uint32_t j = 0; j < nd->card_count[i]; ++j) {
        const size_t k = (size_t)i * KS + j;
        const uint64_t v[6] = {nd->card_free_memory[k], nd->card_clock[k],
                               nd->card_total_memory[k], nd->card_bandwidth[k],
                               nd->card_core[k], nd->card_power[k]};  // CardField order
        if (path == Path::N32) {
          uint32_t* u = reinterpret_cast<uint32_t*>(r + 32);
          for (int f = 0; f < kCardFields; ++f) u[f * K + j] = (uint32_t)v[f];
          u[kFree * K + j] = code_f(v[kFree]);
          u[kTotal * K + j] = code_t(v[kTotal]);
          double* d = reinterpret_cast<double*>(r + n32_f64_off(0, K));
          d[kF64Free * K + j] = (double)v[kFree];
          d[kF64Total * K + j] = (double)v[kTotal];
        } else if (path == Path::F64) {
          double* d = reinterpret_cast<double*>(r + 32);
          for (int f = 0; f < kCardFields; ++f) d[f * K + j] = (double)v[f];
        } else {
          uint64_t* u = reinterpret_cast<uint64_t*>(r + 32);
          for (int f = 0; f < kCardFields; ++f) u[f * K + j] = v[f];
        }
      }
    }
    HIP_TRY(h, h->nodes.ensure(rec.size()));
    HIP_TRY(h, hipMemcpyAsync(h->nodes.p, rec.data(), rec.size(), hipMemcpyHostToDevice,
                              h->stream));
    if (want_sum) {  // node-major as built -> 64-node tiles (sum_index, yoda_layout.h)
      auto tiles = [N](const std::vector<uint32_t>& v, uint32_t stride) {
        std::vector<uint32_t> t(sum_words(std::max<uint32_t>(N, 1), stride), 0u);
        const uint32_t W = stride / 4u;
        for (uint32_t i = 0; i < N; ++i)
          for (uint32_t w = 0; w < W; ++w) t[sum_index(i, w, stride)] = v[(size_t)i * W + w];
        return t;
      };
      // Block-grouped node order for the private batch runs (node order): a
      // snapshot of one-model nodes is dealt into 64-node blocks of one clock each (PodFitsClock
      // then rules whole blocks out for a clock-labelled wave, and K2 skips them), whole blocks
      // round-robin in proportion to each clock's block count so that every node chunk keeps
      // the snapshot's mix, the groups' remainders last.  Copies of the K1 / K2 summaries in
      // that order; the kernels compare the nodes' local ids (perm_ids) on score ties.
      h->perm_on = false;
      static const bool perm_env = YODA_KNOB("YODA_NODE_PERM", 1) != 0;
      std::vector<uint32_t> nperm;
      // Mixed-model nodes (cards of several GPU models) form a group of their own, so that
      // the one-model nodes still fill one-model blocks, which the block summaries decide
      // whole (50 % mixed-model nodes: every block mixed without it).  YODA_NODE_PERM_MIXED=0
      // (A/B knob): one-model snapshots only, as in round 5.
      static const bool perm_mixed = YODA_KNOB("YODA_NODE_PERM_MIXED", 1) != 0;
      if (perm_env && path == Path::N32 && (n_one_model == N || perm_mixed) && N >= 4096 &&
          !(flags & YODA_UPLOAD_PER_NODE_K1) && !(flags & YODA_UPLOAD_PER_NODE_K2)) {
        const uint32_t SW = (uint32_t)(sstride / 4);
        std::vector<uint32_t> keys;
        std::vector<std::vector<uint32_t>> grp;
        bool ok = true;
        for (uint32_t i = 0; i < N && ok; ++i) {
          // (a mixed-model node's kSumClock is its first card's: the key of its group is ~0)
          const uint32_t ck = (sum[(size_t)i * SW + kSumMeta] & kSumUni4)
                                  ? sum[(size_t)i * SW + kSumClock] : 0xffffffffu;
          size_t g = 0;
          while (g < keys.size() && keys[g] != ck) ++g;
          if (g == keys.size()) {
            if (keys.size() == 64) ok = false;  // too many clocks to group usefully
            keys.push_back(ck);
            grp.emplace_back();
          }
          if (ok) grp[g].push_back(i);
        }
        const size_t G = grp.size();
        // Inside a clock group the nodes go into blocks by their healthy frees: sorted on a
        // Z-order key of hfs[0], hfs[1], hfs[3], hfs[7] (the frees that PodFitsMemory compares
        // for 1, 2, 4, 8 GPUs; hfs[15] too at K = 16), so that a block's nodes are alike and its
        // bounds decide it for a whole wave (tools: 16 % of (wave, block)s undecided on config 3
        // with the blocks as uploaded, 4 % sorted); the sorted blocks are then taken in
        // bit-reversed order, so that any run of consecutive blocks -- a node chunk -- still
        // samples every free level (the chunks stay even).
        // Not with memory ranks: there the rank-space K2 ran slower on the sorted blocks
        // (memory in bytes: 1.91 vs 1.80 ms, profiles/r05/y/ab.txt).
        static const bool zorder_env = YODA_KNOB("YODA_NODE_ZORDER", 1) != 0;  // A/B knob
        // (YODA_ZORDER_RANKS=1, A/B knob: with memory ranks too)
        static const bool zorder_ranks = YODA_KNOB("YODA_ZORDER_RANKS", 0) != 0;
        if (ok && zorder_env && (!ranks || zorder_ranks)) {
          std::vector<uint32_t> hix;
          for (uint32_t t = 1; t <= (uint32_t)K; t <<= 1) hix.push_back(t - 1);
          const uint32_t nc = (uint32_t)hix.size(), bits = 64 / nc > 16 ? 16 : 64 / nc;
          std::vector<std::pair<uint64_t, uint32_t>> zk;
          for (auto& g : grp) {
            uint32_t mx[8] = {};
            for (uint32_t i : g)
              for (uint32_t c = 0; c < nc; ++c)
                mx[c] = std::max(mx[c], sum[(size_t)i * SW + kSumHfs + hix[c]]);
            zk.clear();
            for (uint32_t i : g) {
              uint64_t z = 0;
              for (uint32_t c = 0; c < nc; ++c) {
                const uint64_t v = sum[(size_t)i * SW + kSumHfs + hix[c]];
                const uint64_t qv = mx[c] ? std::min<uint64_t>((v << bits) / ((uint64_t)mx[c] + 1),
                                                               (1ull << bits) - 1) : 0;
                for (uint32_t b = 0; b < bits; ++b) z |= ((qv >> b) & 1ull) << (b * nc + c);
              }
              zk.emplace_back(z, i);
            }
            std::stable_sort(zk.begin(), zk.end(), [](const std::pair<uint64_t, uint32_t>& a,
                                                      const std::pair<uint64_t, uint32_t>& b) {
              return a.first < b.first;
            });
            const size_t nbg = g.size() / 64;
            size_t lg = 0;
            while (((size_t)1 << lg) < nbg) ++lg;
            std::vector<uint32_t> out;
            out.reserve(g.size());
            for (size_t j = 0; j < ((size_t)1 << lg); ++j) {  // bit-reversed block order
              size_t r = 0;
              for (size_t b = 0; b < lg; ++b) r |= ((j >> b) & 1u) << (lg - 1 - b);
              if (r < nbg)
                for (size_t k = 0; k < 64; ++k) out.push_back(zk[r * 64 + k].second);
            }
            for (size_t k = nbg * 64; k < g.size(); ++k) out.push_back(zk[k].second);
            g.swap(out);
          }
        }
        if (ok && G >= 1) {
          std::vector<size_t> nb(G), done(G, 0);
          size_t total = 0;
          for (size_t g = 0; g < G; ++g) total += (nb[g] = grp[g].size() / 64);
          nperm.reserve(N);
          for (size_t b = 0; b < total; ++b) {
            size_t best = G;
            double bt = 0.0;
            for (size_t g = 0; g < G; ++g) {
              if (done[g] == nb[g]) continue;
              const double t = (done[g] + 0.5) / (double)nb[g];
              if (best == G || t < bt) best = g, bt = t;
            }
            const size_t o = done[best]++ * 64;
            nperm.insert(nperm.end(), grp[best].begin() + o, grp[best].begin() + o + 64);
          }
          for (size_t g = 0; g < G; ++g)
            nperm.insert(nperm.end(), grp[g].begin() + done[g] * 64, grp[g].end());
          h->perm_on = nperm.size() == N;
        }
      }
      if (h->perm_on) {
        const uint32_t SW = (uint32_t)(sstride / 4), S2W = (uint32_t)(s2stride / 4);
        std::vector<uint32_t> sp((size_t)N * SW), s2p((size_t)N * S2W), inv(N);
        const uint32_t MW = (uint32_t)(mstride / 4), XW = (uint32_t)(xstride / 4);
        std::vector<uint32_t> mp((size_t)N * MW), xp((size_t)N * XW);
        for (uint32_t q = 0; q < N; ++q) {
          const uint32_t i = nperm[q];
          std::memcpy(sp.data() + (size_t)q * SW, sum.data() + (size_t)i * SW, SW * 4);
          std::memcpy(s2p.data() + (size_t)q * S2W, sum2.data() + (size_t)i * S2W, S2W * 4);
          std::memcpy(mp.data() + (size_t)q * MW, mix.data() + (size_t)i * MW, MW * 4);
          std::memcpy(xp.data() + (size_t)q * XW, x1m.data() + (size_t)i * XW, XW * 4);
          inv[i] = q;
        }
        sp = tiles(sp, (uint32_t)sstride);
        s2p = tiles(s2p, (uint32_t)s2stride);
        mp = tiles(mp, (uint32_t)mstride);
        xp = tiles(xp, (uint32_t)xstride);
        HIP_TRY(h, h->kmix_p.ensure(mp.size() * 4));
        HIP_TRY(h, h->kx1_p.ensure(xp.size() * 4));
        HIP_TRY(h, hipMemcpyAsync(h->kmix_p.p, mp.data(), mp.size() * 4, hipMemcpyHostToDevice,
                                  h->stream));
        HIP_TRY(h, hipMemcpyAsync(h->kx1_p.p, xp.data(), xp.size() * 4, hipMemcpyHostToDevice,
                                  h->stream));
        HIP_TRY(h, h->k1sum_p.ensure(sp.size() * 4));
        HIP_TRY(h, h->k2sum_p.ensure(s2p.size() * 4));
        HIP_TRY(h, h->perm_ids.ensure((size_t)N * 4));
        HIP_TRY(h, h->perm_inv.ensure((size_t)N * 4));
        HIP_TRY(h, hipMemcpyAsync(h->k1sum_p.p, sp.data(), sp.size() * 4, hipMemcpyHostToDevice,
                                  h->stream));
        HIP_TRY(h, hipMemcpyAsync(h->k2sum_p.p, s2p.data(), s2p.size() * 4,
                                  hipMemcpyHostToDevice, h->stream));
        HIP_TRY(h, hipMemcpyAsync(h->perm_ids.p, nperm.data(), (size_t)N * 4,
                                  hipMemcpyHostToDevice, h->stream));
        HIP_TRY(h, hipMemcpyAsync(h->perm_inv.p, inv.data(), (size_t)N * 4,
                                  hipMemcpyHostToDevice, h->stream));
        HIP_TRY(h, hipStreamSynchronize(h->stream));  // (the host copies go out of scope)
      }
      // block summaries of the snapshot order and of the block-grouped copy's (BlockSumWord)
      {
        const uint32_t SW = (uint32_t)(sstride / 4);
        auto bsums = [&](const uint32_t* order) {
          const uint32_t nb = (N + 63) / 64, BW = bsum_stride(K) / 4;
          std::vector<uint32_t> b(sum_words(std::max<uint32_t>(nb, 1), bsum_stride(K)), 0u);
          std::vector<uint32_t> o(BW);
          for (uint32_t blk = 0; blk < nb; ++blk) {
            std::fill(o.begin(), o.end(), 0u);
            uint64_t cmin = ~0ull, cmax = 0;
            uint32_t fl = kBsOneModel | kBsUni4, ckmin = ~0u, ckmax = 0, hmin = ~0u, hmax = 0;
            uint32_t nhmin = ~0u, nhmax = 0, mrmin = ~0u, mrmax = 0, nreal = 0, nzt = 0;
            uint32_t mx[6] = {0, 0, 0, 0, 0, 0}, wc[6] = {0, 0, 0, 0, 0, 0};
            uint32_t wl[6] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
            uint32_t tmin[YODA_MAX_CARDS], tmax[YODA_MAX_CARDS];
            for (int t = 0; t < K; ++t) tmin[t] = ~0u, tmax[t] = 0;
            uint32_t sat = ~0u;
            // the healthy-card clocks of the block's nodes: clock, min / max count over the
            // nodes seen so far (a node without the clock counts 0: hc_seen tracks it)
            uint32_t hc_clk[4] = {0, 0, 0, 0}, hc_lo[4] = {0, 0, 0, 0}, hc_hi[4] = {0, 0, 0, 0};
            uint32_t n_hc = 0;
            bool hc_ok = true;
            for (uint32_t l = 0; l < 64 && blk * 64 + l < N; ++l) {
              const uint32_t i = order ? order[blk * 64 + l] : blk * 64 + l;
              const uint32_t* w = sum.data() + (size_t)i * SW;
              const uint64_t cn = (uint64_t)w[kSumCnLo] | ((uint64_t)w[kSumCnHi] << 32);
              const uint32_t meta = w[kSumMeta], nh = (meta >> 8) & 0xffu;
              const uint32_t* cr = clk_rng.data() + 4 * (size_t)i;
              const uint32_t* s2n = sum2.data() + (size_t)i * (s2stride / 4);
              const uint32_t* xn = x1m.data() + (size_t)i * (xstride / 4);
              const uint32_t cnt = (s2n[kS2Meta] >> 8) & 0xffu;
              const bool one = (meta & kSumUni4) && (meta & kSumUniTotal);
              // saturation: 1 + the free of the last card (free order) where a prefix maximum
              // changes (K1MixWord chg bits 1..K); one-model nodes of one total: card 0
              uint32_t sat1 = w[kSumMrf1];
              if (!one && cnt > 0) {
                const uint32_t chg = xn[kX1Chg] & ((2u << K) - 2u);
                const uint32_t jl = chg ? 30u - (uint32_t)__builtin_clz(chg) : 0u;  // bit jl+1
                sat1 = s2n[kS2Fs + jl] + 1u;
              }
              sat = std::min(sat, sat1);
              // healthy cards per clock (K1MixWord ch; more than 4 clocks or a clock beyond 16
              // bits: no table)
              if ((xn[kX1Chg] & kX1ChgMany) || (nh > 0 && cr[3] > 0xffffu)) hc_ok = false;
              if (hc_ok) {
                uint32_t mine[4] = {0, 0, 0, 0};  // this node's count per table entry
                for (uint32_t e = 0; e < 4; ++e) {
                  const uint32_t xw = xn[kX1Ch + e];
                  if ((xw >> 16) == 0u) continue;
                  const uint32_t ck = xw & 0xffffu;
                  uint32_t k = 0;
                  while (k < n_hc && hc_clk[k] != ck) ++k;
                  if (k == n_hc) {
                    if (n_hc == 4) { hc_ok = false; break; }
                    hc_clk[k] = ck;
                    hc_lo[k] = nreal == 0 ? ~0u : 0u;  // the nodes before lacked it
                    hc_hi[k] = 0u;
                    ++n_hc;
                  }
                  mine[k] = xw >> 16;
                }
                for (uint32_t k = 0; k < n_hc; ++k) {
                  hc_lo[k] = std::min(hc_lo[k], mine[k]);
                  hc_hi[k] = std::max(hc_hi[k], mine[k]);
                }
              }
              ++nreal;
              cmin = std::min(cmin, cn);
              cmax = std::max(cmax, cn);
              if (!(meta & kSumUni4)) fl &= ~(kBsUni4 | kBsOneModel);
              if (!(meta & kSumUniTotal)) fl &= ~kBsOneModel;
              if (meta & kSumZeroTotal) ++nzt;
              ckmin = std::min(ckmin, cr[0]);
              ckmax = std::max(ckmax, cr[1]);
              hmin = std::min(hmin, cr[2]);
              hmax = std::max(hmax, cr[3]);
              nhmin = std::min(nhmin, nh);
              nhmax = std::max(nhmax, nh);
              mrmin = std::min(mrmin, w[kSumMrf1]);
              mrmax = std::max(mrmax, w[kSumMrf1]);
              const uint32_t mr = w[kSumMrf1];
              uint32_t v[6] = {w[kSumBw], w[kSumClock], w[kSumCore], mr - (mr != 0u ? 1u : 0u),
                               w[kSumPower], w[kSumTotal]};  // kMax* order
              if (!one && cnt > 0) {  // the all-card maxima (K1MixWord pm over every card)
                const uint32_t a = xn[x1_pm((int)cnt - 1, 0)], b = xn[x1_pm((int)cnt - 1, 1)];
                if (!(meta & kSumUni4)) {  // (16-bit halves: such snapshots keep them <= 65535)
                  v[kMaxBw] = a >> 16;
                  v[kMaxClock] = a & 0xffffu;
                  v[kMaxCore] = b & 0xffffu;
                  v[kMaxPower] = b >> 16;
                }
                v[kMaxTotal] = xn[x1_pm((int)cnt - 1, 2)];
              }
              for (int f = 0; f < 6; ++f) {
                if (wc[f] == 0 || v[f] > mx[f]) {
                  mx[f] = v[f];
                  wc[f] = 1;
                  wl[f] = l;
                } else if (v[f] == mx[f]) {
                  ++wc[f];
                }
              }
              for (int t = 0; t < K; ++t) {
                tmin[t] = std::min(tmin[t], w[kSumHfs + t]);
                tmax[t] = std::max(tmax[t], w[kSumHfs + t]);
              }
            }
            if (nreal == 0) continue;
            o[kBsCnMin] = (uint32_t)std::min<uint64_t>(cmin, 0xffffffffull);
            o[kBsCnMax] = (uint32_t)std::min<uint64_t>(cmax, 0xffffffffull);
            o[kBsFlags] = fl;
            o[kBsCkMin] = ckmin;
            o[kBsCkMax] = ckmax;
            o[kBsHckMin] = hmin;
            o[kBsHckMax] = hmax;
            o[kBsNhMin] = nhmin;
            o[kBsNhMax] = nhmax;
            o[kBsMrfMin] = mrmin;
            o[kBsMrfMax] = mrmax;
            o[kBsNReal] = nreal;
            o[kBsNzt] = nzt;
            o[kBsSat] = sat;
            if (hc_ok) {
              o[kBsFlags] |= kBsHcTab | (n_hc << 8);
              for (uint32_t k = 0; k < n_hc; ++k)
                o[kBsHc + k] = hc_clk[k] | (hc_lo[k] << 16) | (hc_hi[k] << 24);
            }
            for (int f = 0; f < 6; ++f) {
              o[kBsMx + f] = mx[f];
              o[kBsWc + f] = wc[f];
              o[kBsWl + f] = wl[f];
            }
            for (int t = 0; t < K; ++t) {
              o[kBsT + t] = tmin[t];
              o[kBsT + K + t] = tmax[t];
            }
            for (uint32_t w = 0; w < BW; ++w) b[sum_index(blk, w, bsum_stride(K))] = o[w];
          }
          return b;
        };
        const std::vector<uint32_t> bo = bsums(nullptr);
        HIP_TRY(h, h->blksum.ensure(bo.size() * 4));
        HIP_TRY(h, hipMemcpyAsync(h->blksum.p, bo.data(), bo.size() * 4, hipMemcpyHostToDevice,
                                  h->stream));
        if (h->perm_on) {
          const std::vector<uint32_t> bp = bsums(nperm.data());
          HIP_TRY(h, h->blksum_p.ensure(bp.size() * 4));
          HIP_TRY(h, hipMemcpyAsync(h->blksum_p.p, bp.data(), bp.size() * 4,
                                    hipMemcpyHostToDevice, h->stream));
        }
        HIP_TRY(h, hipStreamSynchronize(h->stream));  // (the host copies go out of scope)
        h->blksum_loose = false;
      }
      sum = tiles(sum, (uint32_t)sstride);
      sum2 = tiles(sum2, (uint32_t)s2stride);
      mix = tiles(mix, (uint32_t)mstride);
      x1m = tiles(x1m, (uint32_t)xstride);
      HIP_TRY(h, h->kx1.ensure(x1m.size() * 4));
      HIP_TRY(h, hipMemcpyAsync(h->kx1.p, x1m.data(), x1m.size() * 4, hipMemcpyHostToDevice,
                                h->stream));
      HIP_TRY(h, h->kmix.ensure(mix.size() * 4));
      HIP_TRY(h, hipMemcpyAsync(h->kmix.p, mix.data(), mix.size() * 4, hipMemcpyHostToDevice,
                                h->stream));
      HIP_TRY(h, h->k1sum.ensure(sum.size() * 4));
      HIP_TRY(h, hipMemcpyAsync(h->k1sum.p, sum.data(), sum.size() * 4, hipMemcpyHostToDevice,
                                h->stream));
      HIP_TRY(h, h->k2sum.ensure(sum2.size() * 4));
      HIP_TRY(h, hipMemcpyAsync(h->k2sum.p, sum2.data(), sum2.size() * 4, hipMemcpyHostToDevice,
                                h->stream));
      // the G table: per field the max over every real card (floor 1, collection.go:31-38),
      // the CollectMaxValues result of any pod feasible on the maximal cards' nodes
      uint64_t gmax[6] = {1, 1, 1, 1, 1, 1};
      for (uint32_t i = 0; i < N; ++i)
        for (uint32_t j = 0; j < nd->card_count[i]; ++j) {
          const size_t k = (size_t)i * KS + j;
          gmax[kMaxBw] = std::max(gmax[kMaxBw], nd->card_bandwidth[k]);
          gmax[kMaxClock] = std::max(gmax[kMaxClock], nd->card_clock[k]);
          gmax[kMaxCore] = std::max(gmax[kMaxCore], nd->card_core[k]);
          gmax[kMaxFree] = std::max(gmax[kMaxFree], nd->card_free_memory[k]);
          gmax[kMaxPower] = std::max(gmax[kMaxPower], nd->card_power[k]);
          gmax[kMaxTotal] = std::max(gmax[kMaxTotal], nd->card_total_memory[k]);
        }
      HIP_TRY(h, h->gtab.ensure(sum_words(std::max<uint32_t>(N, 1), gtab_stride(K)) * 4));
      HIP_TRY(h, h->gtab_aux.ensure(kGTabAuxBytes));
      HIP_TRY(h, hipMemcpyAsync(h->gtab_aux.p, gmax, sizeof(gmax), hipMemcpyHostToDevice,
                                h->stream));
      uint32_t* rcp_dev = reinterpret_cast<uint32_t*>(h->gtab_aux.as<unsigned char>() + 48);
      MemTab mt{};
      if (ranks) {  // value tables: v[0] = v[1] = 0, v[2 + i] = the i-th distinct value
        std::vector<double> vt(4 + frees.size() + totals.size(), 0.0);
        for (size_t i = 0; i < frees.size(); ++i) vt[2 + i] = (double)frees[i];
        for (size_t i = 0; i < totals.size(); ++i) vt[4 + frees.size() + i] = (double)totals[i];
        HIP_TRY(h, h->memtab.ensure(vt.size() * 8));
        HIP_TRY(h, hipMemcpy(h->memtab.p, vt.data(), vt.size() * 8, hipMemcpyHostToDevice));
        mt.vf = h->memtab.as<double>();
        mt.vt = h->memtab.as<double>() + 2 + frees.size();
        mt.nf = (uint32_t)frees.size();
      }
      h->mt = mt;
      HIP_TRY(h, launch_gtable(K, h->k2sum.as<uint32_t>(), h->kmix.as<uint32_t>(), N,
                               h->gtab_aux.as<uint64_t>(),
                               h->gtab.as<uint32_t>(), rcp_dev, mt, h->stream));
      if (h->perm_on) {  // the G table of the block-grouped copy (the same rows, reordered)
        HIP_TRY(h, h->gtab_p.ensure(sum_words(std::max<uint32_t>(N, 1), gtab_stride(K)) * 4));
        HIP_TRY(h, launch_gtable(K, h->k2sum_p.as<uint32_t>(), h->kmix_p.as<uint32_t>(), N,
                                 h->gtab_aux.as<uint64_t>(), h->gtab_p.as<uint32_t>(), rcp_dev,
                                 mt, h->stream));
      }
      HIP_TRY(h, hipMemcpyAsync(g_rcp, rcp_dev, sizeof(g_rcp), hipMemcpyDeviceToHost, h->stream));
    }
    const bool diskio = nd->cpu && nd->disk_io;
    if (diskio && N > 0) {  // (g_rcp: read back by the synchronize below)
      std::vector<NodeRecB> rb(N);
      for (uint32_t i = 0; i < N; ++i) {
        rb[i].v = nd->cpu[i] / 100.0;     // algorithm.go:73
        rb[i].u = nd->disk_io[i] / 50.0;  // algorithm.go:71
      }
      HIP_TRY(h, h->nodes_b.ensure((size_t)N * sizeof(NodeRecB)));
      HIP_TRY(h, hipMemcpyAsync(h->nodes_b.p, rb.data(), (size_t)N * sizeof(NodeRecB),
                                hipMemcpyHostToDevice, h->stream));
    }
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    h->host_records.swap(rec);
    h->host_k2sum.swap(sum2);
    h->h_total_sum.assign(nd->total_memory_sum, nd->total_memory_sum + N);
    h->h_free_sum.assign(nd->free_memory_sum, nd->free_memory_sum + N);
    h->h_card_number.assign(nd->card_number, nd->card_number + N);
    h->h_alloc.assign(N, 0);
    if (nd->alloc_memory) h->h_alloc.assign(nd->alloc_memory, nd->alloc_memory + N);
    h->nodes_diskio = diskio;
    h->n_nodes = N;
    h->node_offset = node_offset;
    if (h->K != K || h->path != path) std::memset(h->cap, 0, sizeof(h->cap));
    h->K = K;
    h->path = path;
    h->has_k1sum = want_sum && !(flags & YODA_UPLOAD_PER_NODE_K1);
    h->all_one_model = n_one_model == N;
    h->all_uni4 = n_uni4 == N;
    h->has_k2sum = want_sum && !(flags & YODA_UPLOAD_PER_NODE_K2);
    h->g = GTab{};
    static const bool no_gtab = YODA_KNOB("YODA_NO_GTAB", 0) != 0;  // A/B knob
    if (h->has_k2sum && N > 0 && !no_gtab && !(flags & YODA_UPLOAD_NO_GTAB)) {
      h->g.tab = h->gtab.as<uint32_t>();
      std::memcpy(&h->g.r_bw, &g_rcp[0], 8);
      std::memcpy(&h->g.r_core, &g_rcp[2], 8);
      std::memcpy(&h->g.r_pow, &g_rcp[4], 8);
      std::memcpy(&h->g.r_free, &g_rcp[6], 8);
      std::memcpy(&h->g.r_tot, &g_rcp[8], 8);
      auto ru32 = [](double r) {  // the smallest float >= r (yoda_kernels.hip ru32_of)
        float f = (float)r;
        if ((double)f < r) f = std::nextafter(f, INFINITY);
        return f;
      };
      h->g.f_bw = ru32(h->g.r_bw);
      h->g.f_core = ru32(h->g.r_core);
      h->g.f_pow = ru32(h->g.r_pow);
    }
    h->generic = path == Path::U64;
    h->mem_ranks = ranks;
    h->pack16 = pack16;
    h->q32 = q32;
    h->small_max = max_small;
    h->kbub_dirty = true;
    h->kbub_loose = false;
    h->kb_levels_ok = false;
    h->hot_ok = false;
    if (h->has_k2sum && h->g.tab && N > 0) {
      HIP_TRY(h, build_block_ub(h));
      // the blocks whose bound with every card qualifying (ub[K]) is in the top tenth: a
      // static visiting order hint for the argmax K2 (results do not depend on it)
      const uint32_t nb = (N + 63) / 64, KST = kbub_stride(K);
      std::vector<uint32_t> ubw(sum_words(nb, KST));
      std::vector<uint64_t> words((nb + 63) / 64), words_p((nb + 63) / 64);
      auto hot_bits = [&](const DevBuf& src, std::vector<uint64_t>& out) -> int {
        HIP_TRY(h, hipMemcpyAsync(ubw.data(), src.p, ubw.size() * 4, hipMemcpyDeviceToHost,
                                  h->stream));
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        std::vector<double> u(nb);
        for (uint32_t b = 0; b < nb; ++b) {
          const uint64_t bits = (uint64_t)ubw[sum_index(b, 2 * K, KST)] |
                                ((uint64_t)ubw[sum_index(b, 2 * K + 1, KST)] << 32);
          std::memcpy(&u[b], &bits, 8);
        }
        std::vector<double> srt(u);
        const size_t q = srt.size() - 1 - srt.size() / 10;
        std::nth_element(srt.begin(), srt.begin() + q, srt.end());
        const double thr = srt[q];
        std::fill(out.begin(), out.end(), 0ull);
        for (uint32_t b = 0; b < nb; ++b)
          if (u[b] >= thr) out[b >> 6] |= 1ull << (b & 63);
        return YODA_OK;
      };
      int hr = hot_bits(h->kbub, words);
      if (!hr && h->perm_on) hr = hot_bits(h->kbub_p, words_p);
      if (hr) return hr;
      HIP_TRY(h, h->hot.ensure(words.size() * 8));
      HIP_TRY(h, hipMemcpy(h->hot.p, words.data(), words.size() * 8, hipMemcpyHostToDevice));
      if (h->perm_on) {
        HIP_TRY(h, h->hot_p.ensure(words_p.size() * 8));
        HIP_TRY(h, hipMemcpy(h->hot_p.p, words_p.data(), words_p.size() * 8,
                             hipMemcpyHostToDevice));
      }
      h->hot_ok = true;
    }
    if (!ranks) h->mt = MemTab{};
    h->h_frees.swap(frees);
    h->has_nodes = true;
    // the uploaded pods' N32 memory thresholds follow the snapshot (ranks or the clamp)
    if (h->has_pods && path == Path::N32) {
      int rc = pods_complete(h);  // (the rank kernel reads the 64-bit scv/memory)
      if (rc) return rc;
      unsigned char* b = h->pod_blob.as<unsigned char>();
      HIP_TRY(h, launch_mem_rank(reinterpret_cast<const uint64_t*>(b + h->pod_off[kPodMU]),
                                 h->n_pods, pod_params(h).mt,
                                 reinterpret_cast<uint32_t*>(b + h->pod_off[kPodM32]), h->stream));
      HIP_TRY(h, hipStreamSynchronize(h->stream));
    }
    h->ran = false;
    h->phase1_done = false;
    if (!is_pow2_le16((uint32_t)K)) return fail(h, YODA_ERR_INVALID_ARG, "bad K");
    return YODA_OK;
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_uses_generic_path(const yoda_t* h) { return h ? (h->generic ? 1 : 0) : -1; }

int yoda_record_path(const yoda_t* h) { return h ? (int)h->path : -1; }

int yoda_memory_ranks(const yoda_t* h) { return h ? (h->mem_ranks ? 1 : 0) : -1; }
uint64_t yoda_small_field_max(const yoda_t* h) { return h ? h->small_max : 0; }

uint64_t yoda_score_bound(const yoda_t* h) { return h && h->has_nodes ? h->score_bound : ~0ull; }

int yoda_update_alloc(yoda_t* h, const uint64_t* alloc) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!h->has_nodes) return fail(h, YODA_ERR_NO_NODES, "no node snapshot uploaded");
  if (!alloc && h->n_nodes) return fail(h, YODA_ERR_INVALID_ARG, "alloc is NULL");
  try {
    // Every node through the sparse node-state push: the records, the K2 summaries, their
    // block-grouped copies (perm_on) and the host copies (h_alloc, host_records) all change
    // together -- k_set_static is the one writer of a node's static score.
    const uint32_t N = h->n_nodes;
    std::vector<uint32_t> ids(N);
    for (uint32_t i = 0; i < N; ++i) ids[i] = h->node_offset + i;
    const std::vector<uint64_t> cn(h->h_card_number);
    int rc = yoda_set_node_state(h, N, ids.data(), alloc, cn.data());
    if (rc) return rc;
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return YODA_OK;
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_upload_pods(yoda_t* h, const yoda_pod_soa* pd) {
  if (!h) return YODA_ERR_INVALID_ARG;
  try {
    if (!pd) return fail(h, YODA_ERR_INVALID_ARG, "pods is NULL");
    const uint32_t P = pd->n_pods;
    if (P > 0 && (!pd->has_number || !pd->number || !pd->has_memory || !pd->memory ||
                  !pd->has_clock || !pd->clock))
      return fail(h, YODA_ERR_INVALID_ARG, "a required pod array is NULL");
    h->topk_ready = false;
    h->b_cls_ready = false;
    HIP_TRY(h, hipSetDevice(h->device));
    // One blob of per-pod arrays, staged in pinned memory; the arrays a private block-kernel
    // run reads go with one copy now, the rest (kPodPlace) when an entry point needs them.
    size_t off[kPodArrays], total = 0, core_bytes = 0;
    for (int i = 0; i < kPodArrays; ++i) {
      const int a = kPodPlace[i];
      off[a] = total;
      total += ((size_t)std::max<uint32_t>(P, 1) * kPodArrayBytes[a] + 255) / 256 * 256;
      if (i == kPodCoreArrays - 1) core_bytes = total;
    }
    h->pod_rest_bytes = 0;  // (a deferred part of the previous batch is dropped)
    h->rest_lazy = false;
    // (memory ranks: the rank kernel below reads the 64-bit scv/memory now)
    const bool defer = !(h->has_nodes && h->mem_ranks);
    // the f64 thresholds and the Mode B weights (zero without rio / rcpu) are written later,
    // off the upload's critical path (pods_pack_rest)
    const bool lazy = defer && !(pd->rio && pd->rcpu);
    static const bool dbg = std::getenv("YODA_UPLOAD_DEBUG") != nullptr;
    auto now_ms = [] {
      return std::chrono::duration<double, std::milli>(
                 std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double t_start = dbg ? now_ms() : 0.0;
    if (h->stage_pending) HIP_TRY(h, hipEventSynchronize(h->stage_event));  // staging reuse
    HIP_TRY(h, h->pod_stage.ensure(total));
    HIP_TRY(h, h->pod_blob.ensure(total));
    unsigned char* st = static_cast<unsigned char*>(h->pod_stage.p);
    double* mf = reinterpret_cast<double*>(st + off[kPodMF]);
    double* cf = reinterpret_cast<double*>(st + off[kPodCF]);
    uint64_t* mu = reinterpret_cast<uint64_t*>(st + off[kPodMU]);
    uint64_t* cu = reinterpret_cast<uint64_t*>(st + off[kPodCU]);
    uint64_t* num = reinterpret_cast<uint64_t*>(st + off[kPodNumber]);
    double* al = reinterpret_cast<double*>(st + off[kPodAlpha]);
    double* be = reinterpret_cast<double*>(st + off[kPodBeta]);
    uint32_t* m32 = reinterpret_cast<uint32_t*>(st + off[kPodM32]);
    uint32_t* c32 = reinterpret_cast<uint32_t*>(st + off[kPodC32]);
    uint32_t* nm = reinterpret_cast<uint32_t*>(st + off[kPodNeedMem]);
    uint32_t* nc = reinterpret_cast<uint32_t*>(st + off[kPodNeedClk]);
    const uint64_t kClamp = kPodF64Clamp;
    uint64_t key_or[3] = {0, 0, 0};       // OR of the sort key's clamped fields (c, n, m)
    // distinct (clock, number, has-memory) groups with their pod counts and, per group, its
    // pods of the largest and of the smallest memory (the padding copies) as (m << 32 | pod)
    // extremes.  The pods are packed by up to 16 host threads over contiguous ranges, each
    // with its own group table (merged after: counts add, extremes max/min).
    struct GroupTable {
      std::vector<uint64_t> key = std::vector<uint64_t>(64, 0ull);  // key + 1 (0 = empty)
      std::vector<uint32_t> cnt = std::vector<uint32_t>(64, 0u);
      std::vector<uint64_t> mx = std::vector<uint64_t>(64, 0ull), mn = std::vector<uint64_t>(64, ~0ull);
      size_t n = 0;
      size_t slot(uint64_t k1) const {
        size_t i = (size_t)(k1 * 0x9e3779b97f4a7c15ull >> 40) & (key.size() - 1);
        while (key[i] != 0ull && key[i] != k1) i = (i + 1) & (key.size() - 1);
        return i;
      }
      void add(uint64_t g, uint32_t c, uint64_t vmax, uint64_t vmin) {
        size_t i = slot(g + 1);
        if (key[i] == 0ull) {
          if (2 * (n + 1) > key.size()) {  // grow and rehash
            GroupTable o;
            const size_t n2 = key.size() * 2;
            o.key.assign(n2, 0ull);
            o.cnt.assign(n2, 0u);
            o.mx.assign(n2, 0ull);
            o.mn.assign(n2, ~0ull);
            for (size_t j = 0; j < key.size(); ++j)
              if (key[j]) {
                const size_t t = o.slot(key[j]);
                o.key[t] = key[j];
                o.cnt[t] = cnt[j];
                o.mx[t] = mx[j];
                o.mn[t] = mn[j];
              }
            o.n = n;
            *this = std::move(o);
            i = slot(g + 1);
          }
          key[i] = g + 1;
          ++n;
        }
        cnt[i] += c;
        mx[i] = std::max(mx[i], vmax);
        mn[i] = std::min(mn[i], vmin);
      }
    };
    auto pack_range = [&](uint32_t p0, uint32_t p1, GroupTable& gt, uint64_t* kor_out) {
      // (ORs accumulated locally: the per-thread outputs share cache lines)
      uint64_t kor[3] = {0ull, 0ull, 0ull};
      uint64_t g_last = ~0ull;
      uint32_t g_run = 0;
      uint64_t r_max = 0, r_min = ~0ull;  // the current run's extremes
      for (uint32_t p = p0; p < p1; ++p) {
        const uint64_t number = pd->has_number[p] ? pd->number[p] : 1;  // filter.go:12-15
        const uint64_t m = pd->has_memory[p] ? pd->memory[p] : 0;       // filter.go:19,32
        const uint64_t c = pd->has_clock[p] ? pd->clock[p] : 0;         // filter.go:36,49
        const uint32_t need = number > 0xffffffffull ? 0xffffffffu : (uint32_t)number;
        num[p] = number;
        nm[p] = pd->has_memory[p] ? need : 0;
        nc[p] = pd->has_clock[p] ? need : 0;
        mu[p] = m;
        cu[p] = c;
        if (!lazy) {
          mf[p] = (double)std::min(m, kClamp);
          cf[p] = (double)std::min(c, kClamp);
        }
        m32[p] = (uint32_t)std::min<uint64_t>(m, 0xffffffffull);  // > every N32 field
        c32[p] = (uint32_t)std::min<uint64_t>(c, 0xffffffffull);
        kor[0] |= std::min<uint64_t>(c, 0xffffffull);  // the clamps of k_order_keys
        kor[1] |= std::min<uint64_t>(number, 0xffull);
        kor[2] |= std::min<uint64_t>(m, 0xffffffffull);
        const uint64_t g = (std::min<uint64_t>(c, 0xffffffull) << 9) |
                           (std::min<uint64_t>(number, 0xffull) << 1) | (nm[p] != 0u ? 1u : 0u);
        if (g != g_last) {  // consecutive pods of one group (the common case) skip the probe
          if (g_run) gt.add(g_last, g_run, r_max, r_min);
          g_last = g;
          g_run = 0;
          r_max = 0;
          r_min = ~0ull;
        }
        ++g_run;
        const uint64_t mp = (std::min<uint64_t>(m, 0xffffffffull) << 32) | p;
        r_max = std::max(r_max, mp);
        r_min = std::min(r_min, mp);
        if (!lazy) al[p] = be[p] = 0.0;
        if (pd->rio && pd->rcpu) {  // algorithm.go:105-106
          const double beta = 1.0 / (1.0 + (double)pd->rcpu[p] / pd->rio[p]);
          be[p] = beta;
          al[p] = 1 - beta;
        }
      }
      if (g_run) gt.add(g_last, g_run, r_max, r_min);
      for (int f = 0; f < 3; ++f) kor_out[f] = kor[f];
    };
    // ranges of >= YODA_UPLOAD_MIN_RANGE (default 4096) pods over the process's worker pool
    // (HostPool); A/B knob for the greedy windows' 6144-pod uploads
    static const uint32_t thr_cap = YODA_KNOB("YODA_UPLOAD_THREADS", 16);
    static const uint32_t min_range = std::max<uint32_t>(256, YODA_KNOB("YODA_UPLOAD_MIN_RANGE", 4096));
    const uint32_t n_thr = std::min<uint32_t>({HostPool::get().size(), std::max(1u, thr_cap),
                                               std::max(1u, P / min_range)});
    std::vector<GroupTable> tables(n_thr);
    std::vector<std::array<uint64_t, 3>> kors(n_thr, {0ull, 0ull, 0ull});
    {
      std::vector<uint8_t> thr_failed(n_thr, 0);  // a worker's exception (bad_alloc) -> rethrown
      const uint32_t per = (P + n_thr - 1) / n_thr;
      HostPool::get().run(n_thr, [&](uint32_t t) {
        try {
          pack_range(std::min(P, t * per), std::min(P, (t + 1) * per), tables[t], kors[t].data());
        } catch (...) {
          thr_failed[t] = 1;
        }
      });
      for (uint8_t f : thr_failed)
        if (f) throw std::bad_alloc();
    }
    const double t_packed = dbg ? now_ms() : 0.0;
    GroupTable all = std::move(tables[0]);
    for (uint32_t t = 1; t < n_thr; ++t)
      for (size_t j = 0; j < tables[t].key.size(); ++j)
        if (tables[t].key[j])
          all.add(tables[t].key[j] - 1, tables[t].cnt[j], tables[t].mx[j], tables[t].mn[j]);
    for (const auto& k : kors)
      for (int f = 0; f < 3; ++f) key_or[f] |= k[f];
    std::vector<uint64_t>& gkey = all.key;
    std::vector<uint32_t>& gcnt = all.cnt;
    std::vector<uint64_t>& gmax = all.mx;
    std::vector<uint64_t>& gmin = all.mn;
    const size_t g_n = all.n;
    const double t_merged = dbg ? now_ms() : 0.0;
    HIP_TRY(h, hipMemcpyAsync(h->pod_blob.p, st, defer ? core_bytes : total, hipMemcpyHostToDevice,
                              h->stream));
    if (defer) {  // (the deferred copy of a private run starts from here: pods_complete_async)
      if (int rc = ensure_copy_stream(h)) return rc;
      HIP_TRY(h, hipEventRecord(h->core_event, h->stream));
    }
    const double t_copied = dbg ? now_ms() : 0.0;
    if (h->has_nodes && h->mem_ranks)  // scv/memory -> its rank threshold, on the device
      HIP_TRY(h, launch_mem_rank(reinterpret_cast<const uint64_t*>(
                                     h->pod_blob.as<unsigned char>() + off[kPodMU]),
                                 P, h->mt,
                                 reinterpret_cast<uint32_t*>(h->pod_blob.as<unsigned char>() +
                                                             off[kPodM32]),
                                 h->stream));
    {  // the counting-sort order's groups (yoda_order.hip)
      struct Grp {
        uint64_t key;
        uint32_t count, pod_max, pod_min;  // pods of the largest / smallest memory
        bool operator<(const Grp& o) const { return key < o.key; }
      };
      std::vector<Grp> gs;
      gs.reserve(g_n);
      for (size_t i = 0; i < gkey.size(); ++i)
        if (gkey[i])
          gs.push_back({gkey[i] - 1, gcnt[i], (uint32_t)gmax[i], (uint32_t)gmin[i]});
      std::sort(gs.begin(), gs.end());
      const uint32_t G = (uint32_t)gs.size();
      h->og_ok = G > 0 && G <= kOrderMaxGroups;
      h->n_pad = P;
      if (h->og_ok) {
        uint32_t nbl = 10;  // buckets per group: G * NB <= kOrderMaxGroups entries (LDS)
        while (nbl > 0 && ((size_t)G << nbl) > kOrderMaxGroups) --nbl;
        uint32_t bm = 0;
        while (bm < 32 && (key_or[2] >> bm)) ++bm;
        h->og_groups = G;
        h->og_nb_log2 = nbl;
        h->og_m_shift = bm > nbl ? bm - nbl : 0;
        std::vector<uint32_t> st0(G), stp(G), pad;
        uint32_t a0 = 0, ap = 0;
        for (uint32_t g = 0; g < G; ++g) {
          st0[g] = a0;
          stp[g] = ap;
          a0 += gs[g].count;
          const uint32_t padded = (gs[g].count + kWave - 1) / kWave * kWave;
          // copies of the group's last pod in memory order (largest memory in an ascending
          // -- even -- group, smallest in a descending one): the tail wave's neighbour
          const uint32_t last = (g & 1u) ? gs[g].pod_min : gs[g].pod_max;
          for (uint32_t i = gs[g].count; i < padded; ++i) {
            pad.push_back(ap + i);
            pad.push_back(last);
          }
          ap += padded;
        }
        h->n_pad = ap;
        h->og_n_pad_slots = (uint32_t)(pad.size() / 2);
        h->og_off_start = (size_t)G * 8;
        h->og_off_start_pad = h->og_off_start + (size_t)G * 4;
        h->og_off_pad = h->og_off_start_pad + (size_t)G * 4;
        h->og_host.assign(h->og_off_pad + pad.size() * 4, 0);
        for (uint32_t g = 0; g < G; ++g)
          std::memcpy(h->og_host.data() + (size_t)g * 8, &gs[g].key, 8);
        std::memcpy(h->og_host.data() + h->og_off_start, st0.data(), (size_t)G * 4);
        std::memcpy(h->og_host.data() + h->og_off_start_pad, stp.data(), (size_t)G * 4);
        if (!pad.empty())
          std::memcpy(h->og_host.data() + h->og_off_pad, pad.data(), pad.size() * 4);
        HIP_TRY(h, h->order_meta.ensure(h->og_host.size()));
        HIP_TRY(h, hipMemcpyAsync(h->order_meta.p, h->og_host.data(), h->og_host.size(),
                                  hipMemcpyHostToDevice, h->stream));
        const size_t nbk = (size_t)G << nbl;
        if (h->order_hist.bytes < nbk * 4) {  // the scan clears it after each use
          HIP_TRY(h, h->order_hist.ensure(nbk * 4));
          HIP_TRY(h, hipMemsetAsync(h->order_hist.p, 0, h->order_hist.bytes, h->stream));
        }
        HIP_TRY(h, h->order_bstart.ensure(nbk * 4));
      }
    }
    HIP_TRY(h, hipEventRecord(h->stage_event, h->stream));
    h->stage_pending = true;
    for (int a = 0; a < kPodArrays; ++a) h->pod_off[a] = off[a];
    h->pod_rest_off = core_bytes;
    h->pod_rest_bytes = defer ? total - core_bytes : 0;
    h->rest_lazy = lazy;
    for (int f = 0; f < 3; ++f) {
      uint32_t bits = 0;
      while (bits < 64 && (key_or[f] >> bits)) ++bits;
      h->key_bits[f] = bits;
    }
    h->n_pods = P;
    h->n_work = P;
    h->has_pods = true;
    h->ran = false;
    h->phase1_done = false;
    h->ordered = false;
    h->pods_diskio = pd->rio != nullptr && pd->rcpu != nullptr;
    if (dbg)
      std::fprintf(stderr, "yoda_upload_pods: %u pods, %u threads: pack %.3f merge %.3f copy %.3f "
                   "groups %.3f ms\n", P, n_thr, t_packed - t_start, t_merged - t_packed,
                   t_copied - t_merged, now_ms() - t_copied);
    return YODA_OK;
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

// pad: a private run (yoda_run without the bitmask) -- it may take the counting sort and pad
// the order's groups to whole waves; every other entry point keeps the radix order, one
// sorted position per caller pod, reproducible across the shards of a batch.
static int prepare_run(yoda_t* h, int mode, bool pad = false) {
  int rc = check_ready(h, mode);
  if (rc) return rc;
  h->topk_ready = false;  // this run overwrites the bitmask and reciprocals
  const bool ordering = h->order_enabled && mode == YODA_MODE_SCV &&
                        h->n_pods >= kOrderMinPods && h->n_nodes > 0;
  // a private run takes the counting sort, padded when that adds at most 1/8 of the batch
  // (many small groups would otherwise multiply the work)
  h->count_order = pad && ordering && h->og_ok;
  const bool padded = h->count_order && h->order_pad && YODA_KNOB("YODA_ORDER_PAD", 1) &&
                      (uint64_t)h->n_pad * 8 <= (uint64_t)h->n_pods * 9;
  h->n_work = padded ? h->n_pad : h->n_pods;
  plan_chunks(h, mode, h->n_work, h->n_nodes);
  // a run on the block kernels (argmax, or the greedy windows' top-k) visits its pod blocks
  // heaviest first (the weights: K1's PART nodes per pod block; YODA_LPT=0: launch order)
  static const bool lpt_env = YODA_KNOB("YODA_LPT", 1) != 0;
  const uint32_t n_pb = (h->n_work + kBlock - 1) / kBlock;
  h->lpt_sorted = false;
  h->lpt_active = lpt_env && mode == YODA_MODE_SCV && h->path == Path::N32 &&
                  h->has_k1sum && h->has_k2sum && n_pb >= 8 && n_pb <= 4096;
  if (h->lpt_active) {
    const size_t had = h->lpt_w.bytes;
    HIP_TRY(h, h->lpt_w.ensure((size_t)((h->n_work + 63) / 64) * 4));
    HIP_TRY(h, h->lpt_order.ensure((size_t)n_pb * 4));
    if (h->lpt_w.bytes != had)  // fresh weights start at zero (k_lpt_order re-zeroes them)
      HIP_TRY(h, hipMemsetAsync(h->lpt_w.p, 0, h->lpt_w.bytes, h->stream));
  }
  return ensure_state(h, std::max<uint32_t>(h->n_work, 1));
}

// Diagnostic (YODA_SEED_DEBUG): how close the block K1's K2 pruning seeds came to each wave's
// smallest best score (sorted order, before finalize), on stderr.  Never results or policy.
static void seed_report(yoda_t* h) {
  const uint32_t W = h->n_work, nw = (W + 63) / 64;
  std::vector<uint64_t> sd(nw);
  std::vector<int64_t> best(W);
  std::vector<uint32_t> cnt(W);
  const PodParams pp = pod_params(h);
  if (hipMemcpyAsync(sd.data(), pp.seed, nw * 8ull, hipMemcpyDeviceToHost, h->stream) ||
      hipMemcpyAsync(best.data(), h->best.p, W * 8ull, hipMemcpyDeviceToHost, h->stream) ||
      hipMemcpyAsync(cnt.data(), h->counts.p, W * 4ull, hipMemcpyDeviceToHost, h->stream) ||
      hipStreamSynchronize(h->stream))
    return;
  uint32_t zero = 0, bad = 0, act_w = 0, hist[6] = {};
  double gap = 0;
  for (uint32_t w = 0; w < nw; ++w) {
    int64_t mb = INT64_MAX;
    for (uint32_t l = 64 * w; l < std::min(W, 64 * w + 64); ++l)
      if (cnt[l] && best[l] >= 0) mb = std::min(mb, best[l]);
    if (mb == INT64_MAX) continue;
    ++act_w;
    if (sd[w] == 0) { ++zero; continue; }
    if ((int64_t)sd[w] > mb) ++bad;
    const double r = (double)sd[w] / (double)std::max<int64_t>(mb, 1);
    hist[r >= 1.0 ? 5 : r >= 0.99 ? 4 : r >= 0.95 ? 3 : r >= 0.9 ? 2 : r >= 0.75 ? 1 : 0]++;
    gap += (double)(mb - (int64_t)sd[w]);
  }
  std::fprintf(stderr, "seeds: %u waves with a best, %u without a seed, %u ABOVE the best (bug); "
               "seed/best <.75 %u, <.9 %u, <.95 %u, <.99 %u, <1 %u, =1 %u; mean gap %.1f\n",
               act_w, zero, bad, hist[0], hist[1], hist[2], hist[3], hist[4], hist[5],
               gap / std::max<uint32_t>(1, act_w - zero));
}

int yoda_run(yoda_t* h, int mode, uint32_t flags) {
  if (!h) return YODA_ERR_INVALID_ARG;
  // a private run on the block kernels in the counting order reads only the pod arrays the
  // upload copied first; the rest of the batch goes to the device after its kernels
  const bool fast = mode == YODA_MODE_SCV && !(flags & YODA_RUN_BITMASK) &&
                    h->path == Path::N32 && h->has_k1sum && h->has_k2sum && !h->mem_ranks;
  h->fast_run = fast;
  int rc = prepare_run(h, mode, (flags & YODA_RUN_BITMASK) == 0);
  h->fast_run = false;
  if (rc) return rc;
  const bool defer = fast && h->count_order;
  if (!defer && (rc = pods_complete(h))) return rc;
  // (YODA_SIDE_COPY=0, A/B knob: the deferred copy on the run's stream after its kernels)
  static const bool side = YODA_KNOB("YODA_SIDE_COPY", 1) != 0;
  h->core_only = defer;
  try {
    struct Clear {
      bool& f;
      ~Clear() { f = false; }
    } clear{h->core_only};
    if ((rc = order_pods(h, mode))) return rc;
    if ((rc = phase1(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(),
                     Maxima::OwnFinal)))
      return rc;
    if ((rc = phase2(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                     h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>())))
      return rc;
    if (diag_env("YODA_SEED_DEBUG", 0) && pod_params(h).seed) seed_report(h);
    if ((rc = finalize(h, mode, h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                       h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>(),
                       false)))
      return rc;
    // the deferred arrays: packed on the host while the kernels run, copied on the side stream
    // (from the upload's core copy on, so alongside the kernels), joined into the stream
    h->core_only = false;
    if (defer && side && h->copy_stream && (rc = pods_complete_async(h))) return rc;
    if (defer && (rc = pods_complete(h))) return rc;
    h->ran = true;
    h->ran_bitmask = mode == YODA_MODE_SCV && (flags & YODA_RUN_BITMASK);
    h->last_mode = mode;
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_download(yoda_t* h, yoda_eval_out* out) {
  if (!h || !out) return YODA_ERR_INVALID_ARG;
  if (!h->ran) return fail(h, YODA_ERR_STATE, "yoda_download before yoda_run/finalize");
  if (h->k3_pending)  // picks of the flagged pods unresolved, outputs still in sorted order
    return fail(h, YODA_ERR_STATE,
                "exact normalize pending: run yoda_shard_exact_records / yoda_shard_exact_merge");
  try {
    HIP_TRY(h, hipSetDevice(h->device));
    const uint32_t P = h->n_pods;
    if (P == 0) return YODA_OK;
    hipStream_t s = h->stream;
    if (out->pick)
      HIP_TRY(h, hipMemcpyAsync(out->pick, h->pick.p, P * 4ull, hipMemcpyDeviceToHost, s));
    if (out->status)
      HIP_TRY(h, hipMemcpyAsync(out->status, h->status.p, P * 4ull, hipMemcpyDeviceToHost, s));
    if (out->n_feasible)
      HIP_TRY(h, hipMemcpyAsync(out->n_feasible, h->counts.p, P * 4ull, hipMemcpyDeviceToHost, s));
    if (out->n_ties)
      HIP_TRY(h, hipMemcpyAsync(out->n_ties, h->ties_out.p, P * 4ull, hipMemcpyDeviceToHost, s));
    std::vector<int64_t> top;
    std::vector<int32_t> st;
    if (out->top_score) {
      top.resize(P);
      st.resize(P);
      HIP_TRY(h, hipMemcpyAsync(top.data(), h->best.p, P * 8ull, hipMemcpyDeviceToHost, s));
      HIP_TRY(h, hipMemcpyAsync(st.data(), h->status.p, P * 4ull, hipMemcpyDeviceToHost, s));
    }
    std::vector<uint64_t> mx;
    if (out->maxima && h->maxima_sorted) {  // scatter the maxima to the caller's order now
      const uint32_t W = h->n_work;
      HIP_TRY(h, h->maxima_alt.ensure(h->maxima.bytes));
      PermTable t{};
      for (uint32_t r = 0; r < 6; ++r) {
        t.src[t.n] = h->maxima.as<unsigned char>() + (size_t)r * W * 8;
        t.dst[t.n] = h->maxima_alt.as<unsigned char>() + (size_t)r * P * 8;
        t.bytes[t.n] = 8;
        ++t.n;
      }
      HIP_TRY(h, launch_permute(t, h->perm.as<uint32_t>(), W, true, s));
      std::swap(h->maxima, h->maxima_alt);
      h->maxima_sorted = false;
    }
    if (out->maxima) {
      mx.resize(6 * (size_t)P);
      HIP_TRY(h, hipMemcpyAsync(mx.data(), h->maxima.p, mx.size() * 8, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(h, hipStreamSynchronize(s));
    if (out->top_score)
      for (uint32_t p = 0; p < P; ++p) out->top_score[p] = st[p] == YODA_STATUS_OK ? top[p] : 0;
    if (out->maxima)
      for (uint32_t p = 0; p < P; ++p)
        for (int f = 0; f < 6; ++f) out->maxima[(size_t)p * 6 + f] = mx[(size_t)f * P + p];
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_download_bitmask(yoda_t* h, uint32_t* words, uint64_t n_words) {
  if (!h || !words) return YODA_ERR_INVALID_ARG;
  if (!h->ran_bitmask)
    return fail(h, YODA_ERR_STATE, "no bitmask: run Mode A with YODA_RUN_BITMASK first");
  const uint32_t W = (h->n_nodes + 31) / 32;
  const uint64_t need = (uint64_t)W * h->n_pods;
  if (n_words < need) return fail(h, YODA_ERR_INVALID_ARG, "bitmask buffer too small");
  if (need == 0) return YODA_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, h->bitmask_t.ensure(need * 4));
  HIP_TRY(h, launch_bitmask_transpose(h->bitmask.as<uint64_t>(), bm_row(h->n_nodes), h->bs_ptr(),
                                      bs_row(h->n_nodes), h->blk_ptr(), blk_row(h->n_nodes),
                                      h->n_nodes,
                                      W, h->n_pods,
                                      h->ordered ? h->perm.as<uint32_t>() : nullptr,
                                      h->bitmask_t.as<uint32_t>(), h->stream));
  HIP_TRY(h, hipMemcpyAsync(words, h->bitmask_t.p, need * 4, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return YODA_OK;
}

int yoda_score_rows(yoda_t* h, int mode, uint32_t* bitmask_out, uint64_t n_bitmask_words,
                    int64_t* scores_out, uint64_t n_scores) {
  return yoda_score_rows_norm(h, mode, bitmask_out, n_bitmask_words, scores_out, n_scores,
                              nullptr, 0);
}

int yoda_score_rows_norm(yoda_t* h, int mode, uint32_t* bitmask_out, uint64_t n_bitmask_words,
                         int64_t* scores_out, uint64_t n_scores, int64_t* norm_out,
                         uint64_t n_norm) {
  int rc = prepare_run(h, mode);
  if (rc) return rc;
  try {
    const uint32_t P = h->n_pods, N = h->n_nodes;
    const uint64_t W = (N + 31) / 32;
    if (bitmask_out && n_bitmask_words < W * P)
      return fail(h, YODA_ERR_INVALID_ARG, "bitmask buffer too small");
    if (scores_out && n_scores < (uint64_t)N * P)
      return fail(h, YODA_ERR_INVALID_ARG, "scores buffer too small");
    if (norm_out && n_norm < (uint64_t)N * P)
      return fail(h, YODA_ERR_INVALID_ARG, "norm buffer too small");
    if ((uint64_t)N * P > (1ull << 31))
      return fail(h, YODA_ERR_RANGE, "yoda_score_rows is for small pod batches (P*N <= 2^31)");
    int64_t* rows = nullptr;
    if ((scores_out || norm_out) && (uint64_t)N * P > 0) {
      HIP_TRY(h, h->rows.ensure((size_t)N * P * 8));
      HIP_TRY(h, h->rows_t.ensure((size_t)N * P * 8));
      HIP_TRY(h, hipMemsetAsync(h->rows.p, 0xff, (size_t)N * P * 8, h->stream));  // -1
      rows = h->rows.as<int64_t>();
    }
    if ((rc = order_pods(h, mode))) return rc;
    if ((rc = phase1(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(), Maxima::Own)))
      return rc;
    if ((rc = phase2(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                     h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>(),
                     rows)))
      return rc;
    if (norm_out && rows) {  // before finalize: best / lowest still in the rows' pod order
      HIP_TRY(h, h->norm.ensure((size_t)N * P * 8));
      HIP_TRY(h, launch_norm_rows(rows, N, P, h->best.as<int64_t>(), h->lowest.as<int64_t>(),
                                  h->norm.as<int64_t>(), h->stream));
    }
    if ((rc = finalize(h, mode, h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                       h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>(),
                       false)))
      return rc;
    h->ran = true;
    h->ran_bitmask = mode == YODA_MODE_SCV;
    h->last_mode = mode;
    if (rows && scores_out) {
      HIP_TRY(h, launch_rows_transpose(rows, N, P, h->ordered ? h->perm.as<uint32_t>() : nullptr,
                                       h->rows_t.as<int64_t>(), h->stream));
      HIP_TRY(h, hipMemcpyAsync(scores_out, h->rows_t.p, (size_t)N * P * 8,
                                hipMemcpyDeviceToHost, h->stream));
      if (norm_out) HIP_TRY(h, hipStreamSynchronize(h->stream));  // rows_t is reused below
    }
    if (rows && norm_out) {
      HIP_TRY(h, launch_rows_transpose(h->norm.as<int64_t>(), N, P,
                                       h->ordered ? h->perm.as<uint32_t>() : nullptr,
                                       h->rows_t.as<int64_t>(), h->stream));
      HIP_TRY(h, hipMemcpyAsync(norm_out, h->rows_t.p, (size_t)N * P * 8, hipMemcpyDeviceToHost,
                                h->stream));
    }
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (bitmask_out && W * P > 0) {
      if (mode == YODA_MODE_DISKIO) {  // Filter is a pass-through: every node feasible
        for (uint64_t p = 0; p < P; ++p)
          for (uint64_t w = 0; w < W; ++w) {
            const uint32_t bits = (w + 1) * 32 <= N ? 0xffffffffu : ((1u << (N % 32)) - 1);
            bitmask_out[p * W + w] = bits;
          }
      } else if ((rc = yoda_download_bitmask(h, bitmask_out, n_bitmask_words))) {
        return rc;
      }
    }
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_eval(yoda_t* h, const yoda_pod_soa* pods, int mode, yoda_eval_out* out) {
  int rc = yoda_upload_pods(h, pods);
  if (rc) return rc;
  if ((rc = yoda_run(h, mode, 0))) return rc;
  return yoda_download(h, out);
}

// ---- sharded entry points -------------------------------------------------------------
int yoda_shard_exchange_order(yoda_t* h, int caller_order) {
  if (!h || (caller_order != 0 && caller_order != 1)) return YODA_ERR_INVALID_ARG;
  h->xo_enabled = caller_order == 1;
  return YODA_OK;
}

int yoda_shard_phase1(yoda_t* h, int mode, uint64_t* d_maxima, uint32_t* d_counts) {
  if (!h) return YODA_ERR_INVALID_ARG;
  // caller-order exchange (yoda_shard_exchange_order): each shard its private order; not on the
  // U64 path (its exact-normalize records are per sorted position)
  h->xo = h->xo_enabled && !h->generic;
  int rc = prepare_run(h, mode, h->xo);
  if (rc) return rc;
  if (!d_maxima || !d_counts) return fail(h, YODA_ERR_INVALID_ARG, "NULL exchange buffer");
  try {
    if ((rc = order_pods(h, mode))) return rc;
    if (h->xo) {
      if ((rc = phase1(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>()))) return rc;
      if ((rc = xfer(h, true, {{h->maxima.p, d_maxima, 6, 8}, {h->counts.p, d_counts, 2, 4}})))
        return rc;
    } else if ((rc = phase1(h, mode, d_maxima, d_counts))) {
      return rc;
    }
    h->phase1_done = true;
    h->phase1_wit = false;
    h->ran = false;
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_phase2(yoda_t* h, int mode, const uint64_t* d_maxima, const uint32_t* d_counts,
                      int64_t* d_best, uint32_t* d_idx, uint32_t* d_ties, int64_t* d_lowest) {
  int rc = check_ready(h, mode);
  if (rc) return rc;
  if (!h->phase1_done) return fail(h, YODA_ERR_STATE, "yoda_shard_phase2 before phase1");
  if (!d_maxima || !d_counts || !d_best || !d_idx || !d_ties || !d_lowest)
    return fail(h, YODA_ERR_INVALID_ARG, "NULL exchange buffer");
  try {
    const uint32_t P = h->n_pods;
    if (h->xo) {  // the reduced caller-order buffers into this run's order, and back
      int rc2 = xfer(h, false, {{h->maxima.p, const_cast<uint64_t*>(d_maxima), 6, 8},
                                {h->counts.p, const_cast<uint32_t*>(d_counts), 2, 4}});
      if (rc2) return rc2;
      if ((rc2 = phase2(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(),
                        h->best.as<int64_t>(), h->idx.as<uint32_t>(), h->ties.as<uint32_t>(),
                        h->lowest.as<int64_t>())))
        return rc2;
      return xfer(h, true, {{h->best.p, d_best, 1, 8}, {h->idx.p, d_idx, 1, 4},
                            {h->ties.p, d_ties, 1, 4}, {h->lowest.p, d_lowest, 1, 8}});
    }
    // keep the reduced maxima for download and the generic exact-normalize pass
    if (P) HIP_TRY(h, hipMemcpyAsync(h->maxima.p, d_maxima, 6ull * P * 8, hipMemcpyDeviceToDevice,
                                     h->stream));
    return phase2(h, mode, h->maxima.as<uint64_t>(), d_counts, d_best, d_idx, d_ties, d_lowest);
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_prepare_merge(yoda_t* h, const int64_t* d_best_global, const int64_t* d_best_local,
                             uint32_t* d_idx, uint32_t* d_ties) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!d_best_global || !d_best_local || !d_idx || !d_ties)
    return fail(h, YODA_ERR_INVALID_ARG, "NULL exchange buffer");
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->n_pods == 0) return YODA_OK;
  HIP_TRY(h, launch_merge_prepare(d_best_global, d_best_local, h->n_pods, d_idx, d_ties,
                                  h->stream));
  return YODA_OK;
}

int yoda_shard_finalize(yoda_t* h, int mode, const uint32_t* d_counts, const int64_t* d_best,
                        const uint32_t* d_idx, const uint32_t* d_ties, const int64_t* d_lowest) {
  int rc = check_ready(h, mode);
  if (rc) return rc;
  if (!d_counts || !d_best || !d_idx || !d_ties || !d_lowest)
    return fail(h, YODA_ERR_INVALID_ARG, "NULL exchange buffer");
  try {
    const uint32_t P = h->n_pods;
    if (h->xo) {  // the merged caller-order buffers into this run's order
      if ((rc = xfer(h, false, {{h->counts.p, const_cast<uint32_t*>(d_counts), 2, 4},
                                {h->best.p, const_cast<int64_t*>(d_best), 1, 8},
                                {h->idx.p, const_cast<uint32_t*>(d_idx), 1, 4},
                                {h->ties.p, const_cast<uint32_t*>(d_ties), 1, 4},
                                {h->lowest.p, const_cast<int64_t*>(d_lowest), 1, 8}})))
        return rc;
      if ((rc = finalize(h, mode, h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                         h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>(),
                         true)))
        return rc;
    } else {
      if (P) {
        HIP_TRY(h, hipMemcpyAsync(h->counts.p, d_counts, 2ull * P * 4, hipMemcpyDeviceToDevice,
                                  h->stream));
        HIP_TRY(h, hipMemcpyAsync(h->best.p, d_best, P * 8ull, hipMemcpyDeviceToDevice, h->stream));
      }
      if ((rc = finalize(h, mode, h->counts.as<uint32_t>(), h->best.as<int64_t>(), d_idx, d_ties,
                         d_lowest, true)))
        return rc;
    }
    h->ran = true;
    h->ran_bitmask = false;
    h->last_mode = mode;
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_exact_records(yoda_t* h, void* d_rec) {
  if (!h || !d_rec) return YODA_ERR_INVALID_ARG;
  if (!h->k3_pending) return fail(h, YODA_ERR_STATE, "no exact-normalize pods pending");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemcpyAsync(d_rec, h->k3rec.p, (size_t)h->n_work * sizeof(ShardRec),
                            hipMemcpyDeviceToDevice, h->stream));
  return YODA_OK;
}

int yoda_shard_exact_merge(yoda_t* h, const void* d_all, int world) {
  if (!h || !d_all || world < 1) return YODA_ERR_INVALID_ARG;
  if (!h->k3_pending) return fail(h, YODA_ERR_STATE, "no exact-normalize pods pending");
  try {
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, launch_merge3(static_cast<const ShardRec*>(d_all), h->n_work, (uint32_t)world,
                             h->flagged.as<uint32_t>(), h->n_flagged.as<uint32_t>(), h->k3_nfl,
                             h->pick.as<int32_t>(), h->status.as<int32_t>(),
                             h->ties_out.as<uint32_t>(), h->stream));
    h->k3_pending = false;
    return unpermute_outputs(h);
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_overflow_count(yoda_t* h, uint32_t* n_pods) {
  if (!h || !n_pods) return YODA_ERR_INVALID_ARG;
  *n_pods = 0;
  if (!h->generic || !h->n_flagged.p) return YODA_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemcpyAsync(n_pods, h->n_flagged.p, 4, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return YODA_OK;
}

int yoda_order_info(const yoda_t* h, uint32_t* out) {
  if (!h || !out) return YODA_ERR_INVALID_ARG;
  out[0] = h->og_ok ? h->og_groups : 0u;
  out[1] = h->n_pad;
  out[2] = h->n_work;
  out[3] = h->ordered ? (h->count_order ? 2u : 1u) : 0u;
  return YODA_OK;
}

int yoda_node_order(const yoda_t* h, uint32_t* grouped) {
  if (!h || !grouped) return YODA_ERR_INVALID_ARG;
  *grouped = h->perm_on ? 1u : 0u;
  return YODA_OK;
}

int yoda_set_pod_order(yoda_t* h, int enable) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (enable < 0 || enable > 2) return fail(h, YODA_ERR_INVALID_ARG, "enable must be 0, 1 or 2");
  h->order_enabled = enable != 0;
  h->order_pad = enable == 1;
  return YODA_OK;
}

int yoda_class_stats_enable(yoda_t* h, int enable) {
  if (!h) return YODA_ERR_INVALID_ARG;
  HIP_TRY(h, hipSetDevice(h->device));
  if (enable && !h->class_stats) {
    // YODA_K2_TRACE=<(wave, chunk) slots>: K2 also records per-(wave, chunk) timings
    const uint32_t tr = diag_env("YODA_K2_TRACE", 0);
    const size_t bytes = (16 + 4 * (size_t)tr) * 8;
    HIP_TRY(h, h->stats_dev.ensure(bytes));
    HIP_TRY(h, hipMemsetAsync(h->stats_dev.p, 0, bytes, h->stream));
    if (tr) {  // YODA_K1_TRACE set: the K1 records it instead of the K2
      // low byte: which kernel traces; above it the slot count (the kernels bound the index)
      const uint64_t one = (diag_env("YODA_K1_TRACE", 0) ? 2 : 1) | ((uint64_t)tr << 8);
      HIP_TRY(h, hipMemcpyAsync(h->stats_dev.as<uint64_t>() + 15, &one, 8,
                                hipMemcpyHostToDevice, h->stream));
      HIP_TRY(h, hipStreamSynchronize(h->stream));
    }
    h->stats_pairs1 = h->stats_pairs2 = 0;
  }
  h->class_stats = enable != 0;
  return YODA_OK;
}

int yoda_class_stats_read(yoda_t* h, uint64_t* out) {
  if (!h || !out) return YODA_ERR_INVALID_ARG;
  for (int i = 0; i < 18; ++i) out[i] = 0;
  if (!h->stats_dev.p) return YODA_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  uint64_t d[16] = {};
  HIP_TRY(h, hipMemcpyAsync(d, h->stats_dev.p, 16 * 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  out[0] = d[0];                                                   // K1 ALL
  out[1] = d[1];                                                   // K1 NONE
  out[2] = h->stats_pairs1 - std::min(h->stats_pairs1, d[0] + d[1]);  // K1 PART
  out[3] = d[2];                                                   // K2 U
  out[4] = d[3];                                                   // K2 FAST
  out[5] = d[4];                                                   // K2 EXACT
  out[6] = h->stats_pairs2 - std::min(h->stats_pairs2, d[2] + d[3] + d[4]);  // K2 skipped
  out[7] = d[5];                                                   // K2 (wave, chunk)s, uniform
  out[8] = d[6];                                                   // K2 (wave, chunk)s
  out[9] = h->stats_pairs1;
  out[10] = d[7];                                                  // K2 FAST via node records
  out[11] = d[8];                                                  // K2 per-pod, non-uniform
  out[12] = d[9];                                                  // max per-pod nodes/(w, c)
  out[13] = d[10];                                                 // K1 (w, block)s all NONE
  out[14] = d[11];                                                 // K1 (w, block)s all ALL
  out[15] = d[12];                                                 // K1 (w, block)s
  out[16] = d[13];                                                 // K2 (w, block)s pruned
  out[17] = d[14];                                                 // K2 (w, block)s worked
  HIP_TRY(h, hipMemsetAsync(h->stats_dev.p, 0, 15 * 8, h->stream));
  h->stats_pairs1 = h->stats_pairs2 = 0;
  return YODA_OK;
}

int yoda_k2_trace_read(yoda_t* h, uint64_t* out, uint64_t n_slots) {
  if (!h || !out) return YODA_ERR_INVALID_ARG;
  if (!h->stats_dev.p || h->stats_dev.bytes < (16 + 4 * n_slots) * 8) return YODA_ERR_INVALID_ARG;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemcpyAsync(out, h->stats_dev.as<uint64_t>() + 16, 4 * n_slots * 8,
                            hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return YODA_OK;
}

int yoda_profile(yoda_t* h, int enable) {
  if (!h) return YODA_ERR_INVALID_ARG;
  h->profiling = enable != 0;
  return YODA_OK;
}

int yoda_profile_read(yoda_t* h, double* k1_ms, double* k2_ms, uint32_t* n_launches) {
  if (!h) return YODA_ERR_INVALID_ARG;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  double t1 = 0, t2 = 0;
  for (auto& pr : h->ev_k1) {
    float ms = 0;
    HIP_TRY(h, hipEventElapsedTime(&ms, pr.first, pr.second));
    t1 += ms;
  }
  for (auto& pr : h->ev_k2) {
    float ms = 0;
    HIP_TRY(h, hipEventElapsedTime(&ms, pr.first, pr.second));
    t2 += ms;
  }
  if (k1_ms) *k1_ms = t1;
  if (k2_ms) *k2_ms = t2;
  if (n_launches) *n_launches = (uint32_t)h->ev_k2.size();
  h->ev_k1.clear();
  h->ev_k2.clear();
  h->ev_used = 0;
  return YODA_OK;
}

namespace {

// Device-side node state for the greedy resolve: the static score (Allocate + Actual) and
// CardNumber of the nodes picked so far, pushed in small batches (k_set_static).
struct GreedyState {
  yoda_t* h;
  std::vector<uint64_t> alloc, card_number, stat;    // current, per node
  std::vector<uint64_t> stat_w;                       // static at window start
  std::vector<uint8_t> touched_w, dirty;
  std::vector<uint32_t> touched_list, dirty_list;

  uint64_t stat_bits(uint64_t v) const {  // header word: f64 bits on the fast paths
    if (h->generic) return v;
    const double d = (double)v;
    uint64_t b;
    std::memcpy(&b, &d, 8);
    return b;
  }
  void touch(uint32_t n) {
    if (!touched_w[n]) {
      touched_w[n] = 1;
      stat_w[n] = stat[n];
      touched_list.push_back(n);
    }
    if (!dirty[n]) {
      dirty[n] = 1;
      dirty_list.push_back(n);
    }
  }
  int push(std::vector<uint32_t>& list, std::vector<uint8_t>* marks) {
    if (list.empty()) return YODA_OK;
    // one pinned staging copy: [node u32 x cnt | pad | static u64 x cnt | CardNumber u64 x cnt]
    const uint32_t cnt = (uint32_t)list.size();
    const size_t o_val = ((size_t)cnt * 4 + 15) / 16 * 16, o_cn = o_val + (size_t)cnt * 8;
    const size_t bytes = o_cn + (size_t)cnt * 8;
    if (h->upd_pending) HIP_TRY(h, hipEventSynchronize(h->upd_event));
    HIP_TRY(h, h->upd_stage.ensure(bytes));
    unsigned char* st = static_cast<unsigned char*>(h->upd_stage.p);
    uint32_t* nd = reinterpret_cast<uint32_t*>(st);
    uint64_t* val = reinterpret_cast<uint64_t*>(st + o_val);
    uint64_t* cn = reinterpret_cast<uint64_t*>(st + o_cn);
    for (uint32_t i = 0; i < cnt; ++i) {
      nd[i] = list[i];
      val[i] = stat_bits(stat[list[i]]);
      cn[i] = card_number[list[i]];
    }
    // k_set_static reads the (mapped) staging pages itself: no copy; the event marks the
    // end of that read, before which the pages are not rewritten
    const unsigned char* d = static_cast<const unsigned char*>(h->upd_stage.dp);
    const uint32_t stride = h->path == Path::N32 ? n32_stride(h->K) : node_stride(h->K);
    h->blksum_loose = true;  // (the atomics keep the block bounds valid, not tight)
    for (uint32_t i = 0; i < cnt; ++i) h->note_static(list[i], stat[list[i]]);
    HIP_TRY(h, launch_set_static(h->nodes.as<unsigned char>(), stride,
                                 reinterpret_cast<const uint32_t*>(d),
                                 reinterpret_cast<const uint64_t*>(d + o_val),
                                 reinterpret_cast<const uint64_t*>(d + o_cn), cnt,
                                 h->has_k1sum ? h->k1sum.as<unsigned char>() : nullptr,
                                 k1sum_stride(h->K),
                                 h->has_k2sum ? h->k2sum.as<unsigned char>() : nullptr,
                                 k2sum_stride(h->K), h->perm_copy(), h->stream));
    HIP_TRY(h, hipEventRecord(h->upd_event, h->stream));
    h->upd_pending = true;
    if (marks)
      for (uint32_t n : list) (*marks)[n] = 0;
    list.clear();
    return YODA_OK;
  }
  int push_dirty() { return push(dirty_list, &dirty); }
};

// A pod SoA holding the pods `idx` of `src` (in that order).
struct PodGather {
  std::vector<uint8_t> hn, hm, hc;
  std::vector<uint64_t> n, m, c;
  std::vector<int64_t> prio, rcpu;
  std::vector<double> rio;
  yoda_pod_soa soa{};
  void build(const yoda_pod_soa* src, const uint32_t* idx, uint32_t cnt) {
    hn.resize(cnt), hm.resize(cnt), hc.resize(cnt), n.resize(cnt), m.resize(cnt), c.resize(cnt);
    prio.assign(cnt, 0), rcpu.assign(cnt, 0), rio.assign(cnt, 0.0);
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint32_t p = idx[i];
      hn[i] = src->has_number[p], n[i] = src->number[p];
      hm[i] = src->has_memory[p], m[i] = src->memory[p];
      hc[i] = src->has_clock[p], c[i] = src->clock[p];
      if (src->priority) prio[i] = src->priority[p];
      if (src->rio) rio[i] = src->rio[p];
      if (src->rcpu) rcpu[i] = src->rcpu[p];
    }
    soa.n_pods = cnt;
    soa.has_number = hn.data(), soa.number = n.data();
    soa.has_memory = hm.data(), soa.memory = m.data();
    soa.has_clock = hc.data(), soa.clock = c.data();
    soa.priority = prio.data();
    soa.rio = src->rio ? rio.data() : nullptr;
    soa.rcpu = src->rcpu ? rcpu.data() : nullptr;
  }
};

// Queue order (sort.go:8-10): scv/priority descending, then input index.  A counting sort
// when the priorities span < 2^16 values (the usual small integers), else a stable sort.
void queue_order(const int64_t* prio, uint32_t P, std::vector<uint32_t>& order) {
  order.resize(P);
  if (!prio || P == 0) {
    for (uint32_t i = 0; i < P; ++i) order[i] = i;
    return;
  }
  int64_t lo = prio[0], hi = prio[0];
  for (uint32_t i = 1; i < P; ++i) {
    lo = std::min(lo, prio[i]);
    hi = std::max(hi, prio[i]);
  }
  if ((uint64_t)hi - (uint64_t)lo < (1u << 16)) {
    const uint32_t R = (uint32_t)((uint64_t)hi - (uint64_t)lo) + 1;
    std::vector<uint32_t> start(R + 1, 0);
    for (uint32_t i = 0; i < P; ++i) ++start[(uint32_t)((uint64_t)hi - (uint64_t)prio[i]) + 1];
    for (uint32_t r = 0; r < R; ++r) start[r + 1] += start[r];
    for (uint32_t i = 0; i < P; ++i) order[start[(uint32_t)((uint64_t)hi - (uint64_t)prio[i])]++] = i;
    return;
  }
  for (uint32_t i = 0; i < P; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [prio](uint32_t a, uint32_t b) { return prio[a] > prio[b]; });
}

// 6144 pods: larger windows cost fewer, longer GPU windows but more exact fallbacks (touched
// nodes invalidate more candidate lists); profiles/r02/final/greedy_window_ab.txt
constexpr uint32_t kGreedyWindow = 6144;
// A/B knob: YODA_GREEDY_WINDOW overrides the window size (pods per GPU window).
uint32_t greedy_window() {
  static const uint32_t w = [] {
    const uint32_t v = YODA_KNOB("YODA_GREEDY_WINDOW", 0);
    return v >= 64 && v <= (1u << 20) ? v : kGreedyWindow;
  }();
  return w;
}

// Exact evaluation of ONE pod against the current device state (pushes pending updates).
int greedy_eval_one(GreedyState& g, const yoda_pod_soa* pods, uint32_t p, int mode,
                    int32_t* pick_out) {
  yoda_t* h = g.h;
  int rc = g.push_dirty();
  if (rc) return rc;
  PodGather one;
  one.build(pods, &p, 1);
  if ((rc = yoda_upload_pods(h, &one.soa))) return rc;
  if ((rc = yoda_run(h, mode, 0))) return rc;
  HIP_TRY(h, h->pick_stage.ensure(16));
  HIP_TRY(h, hipMemcpyAsync(h->pick_stage.p, h->pick.p, 4, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  *pick_out = *static_cast<int32_t*>(h->pick_stage.p);
  return YODA_OK;
}

// Exact evaluation of the window pod at sorted position s against the current node state,
// reusing the window's feasibility bits and maxima (only static scores change inside a
// window, and push_dirty makes them current): one launch + an 4-byte copy.
int greedy_eval_fast(GreedyState& g, uint32_t s, int32_t* pick_out) {
  yoda_t* h = g.h;
  int rc = g.push_dirty();
  if (rc) return rc;
  const uint32_t nb = greedy_one_blocks();
  if (h->g1_done.bytes == 0) {
    HIP_TRY(h, h->g1_done.ensure(16));
    HIP_TRY(h, hipMemsetAsync(h->g1_done.p, 0, 16, h->stream));
  }
  HIP_TRY(h, h->g1_part.ensure((size_t)nb * 12 + 16));
  double* ps = h->g1_part.as<double>();
  uint32_t* pi = reinterpret_cast<uint32_t*>(ps + nb);
  uint32_t* done = h->g1_done.as<uint32_t>();
  // the last block writes the pick straight into mapped (coherent) pinned memory: no copy,
  // and the host polls the node word instead of synchronising the stream (the next device
  // work is stream-ordered after this kernel anyway)
  h->poll_stage.flags = hipHostMallocCoherent;
  HIP_TRY(h, h->poll_stage.ensure(16));
  volatile uint32_t* res = static_cast<volatile uint32_t*>(h->poll_stage.p) + 1;
  constexpr uint32_t kPending = 0xfffffffeu;  // never a node index (N < 2^31)
  *res = kPending;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  HIP_TRY(h, launch_greedy_one(h->K, h->path, h->nodes.as<unsigned char>(),
                               h->has_k2sum ? h->k2sum.as<unsigned char>() : nullptr, h->n_nodes,
                               pod_params(h), h->rcp.as<double>(), 
                               h->n_pods, s, h->bitmask.as<uint64_t>(), bm_row(h->n_nodes),
                               h->bs_ptr(), bs_row(h->n_nodes), h->blk_ptr(),
                               blk_row(h->n_nodes), ps, pi, done,
                               static_cast<uint32_t*>(h->poll_stage.dp) + 1, h->stream));
  {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; *res == kPending; ++spin) {
      // past a generous bound (a stalled device, or memory the device cannot reach coherently
      // on this system) the stream synchronisation decides
      if ((spin & 1023u) == 0u &&
          std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
        HIP_TRY(h, hipStreamSynchronize(h->stream));
        break;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  // (word 1: the kernel's out[0]; its f64 score follows 8-byte aligned at word 2)
  const uint32_t n = *res;
  if (n == kPending) return fail(h, YODA_ERR_STATE, "greedy: the fallback's result never arrived");
  if (n == 0xffffffffu) return fail(h, YODA_ERR_INVALID_ARG, "greedy: no feasible node found");
  *pick_out = (int32_t)(n + h->node_offset);
  return YODA_OK;
}

}  // namespace

}  // extern "C"
static int greedy_capacity(yoda_t* h, const yoda_pod_soa* pods, int32_t* pick);
extern "C" {

int yoda_greedy(yoda_t* h, const yoda_pod_soa* pods, int mode, uint32_t flags, int32_t* pick) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!pods || !pick) return fail(h, YODA_ERR_INVALID_ARG, "NULL pods or pick");
  if (!h->has_nodes) return fail(h, YODA_ERR_NO_NODES, "no node snapshot uploaded");
  try {
    HIP_TRY(h, hipSetDevice(h->device));
    GreedyScope scope(h);
    const uint32_t P = pods->n_pods, N = h->n_nodes;
    h->greedy_windows = 0;
    h->greedy_fallbacks = 0;
    h->greedy_restarts = 0;
    h->greedy_refreshes = 0;
    h->greedy_window_ms = h->greedy_fallback_ms = h->greedy_resolve_ms = 0;
    h->greedy_prep_ms = 0;
    using Clock = std::chrono::steady_clock;
    auto ms_since = [](Clock::time_point t0) {
      return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    };
    if (P == 0) return YODA_OK;
    int rc;
    // Queue order: sort.Less (sort.go:8-10) -- scv/priority descending, then input index.
    std::vector<uint32_t> order;
    queue_order(pods->priority, P, order);
    if (mode == YODA_MODE_DISKIO) {  // Mode B reads no assumed-pod state: independent cycles
      PodGather all;
      all.build(pods, order.data(), P);
      if ((rc = yoda_upload_pods(h, &all.soa)) || (rc = yoda_run(h, mode, 0))) return rc;
      std::vector<int32_t> pk(P);
      // the handle's stream may be non-blocking: copy and wait on it, not on the null stream
      HIP_TRY(h, hipMemcpyAsync(pk.data(), h->pick.p, P * 4ull, hipMemcpyDeviceToHost, h->stream));
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      for (uint32_t i = 0; i < P; ++i) pick[order[i]] = pk[i];
      return YODA_OK;
    }
    if ((flags & YODA_GREEDY_CARD_CAPACITY) && !h->generic) return greedy_capacity(h, pods, pick);
    GreedyState g;
    g.h = h;
    g.alloc = h->h_alloc;
    g.card_number = h->h_card_number;
    g.stat.resize(N);
    g.stat_w.resize(N);
    g.touched_w.assign(N, 0);
    g.dirty.assign(N, 0);
    for (uint32_t n = 0; n < N; ++n) {
      bool z;
      g.stat[n] = static_score(h->h_free_sum[n], h->h_total_sum[n], g.alloc[n], &z);
    }
    const std::vector<uint64_t> stat0 = g.stat;
    std::vector<uint32_t> all_touched;
    std::vector<uint8_t> ever(N, 0);
    auto apply_pick = [&](uint32_t p, int32_t node) {
      if (node < 0) return;
      const uint32_t n = (uint32_t)node - h->node_offset;
      g.touch(n);  // snapshots the window-start static before it changes
      if (pods->has_memory[p]) g.alloc[n] += pods->memory[p];  // uint64 wrap (algorithm.go:301)
      if (flags & YODA_GREEDY_CARD_CAPACITY) {
        const uint64_t num = pods->has_number[p] ? pods->number[p] : 1;
        g.card_number[n] = g.card_number[n] >= num ? g.card_number[n] - num : 0;
      }
      bool z;
      g.stat[n] = static_score(h->h_free_sum[n], h->h_total_sum[n], g.alloc[n], &z);
      if (!ever[n]) {
        ever[n] = 1;
        all_touched.push_back(n);
      }
    };
    const bool exact_seq = (flags & YODA_GREEDY_CARD_CAPACITY) || h->generic;
    if (exact_seq) {
      // Feasibility (CardNumber) or the U64 normalize check can change after every pick:
      // evaluate each pod exactly against the current state.
      for (uint32_t i = 0; i < P; ++i) {
        const uint32_t p = order[i];
        int32_t pk = -1;
        if ((rc = greedy_eval_one(g, pods, p, mode, &pk))) return rc;
        pick[p] = pk;
        apply_pick(p, pk);
        ++h->greedy_fallbacks;
      }
    } else {
      // Windowed top-k + certified sequential resolve (greedy).  Within a
      // window only the Allocate term of picked nodes changes, and it never increases
      // (unless alloc wraps around 2^64: then the rest of the window is evaluated exactly).
      // YODA_GREEDY_TOPK=16 (A/B knob): the capacity mode's deeper lists for this mode too
      static const uint32_t kt_env = YODA_KNOB("YODA_GREEDY_TOPK", 0);
      const uint32_t KT = kt_env == (uint32_t)topk_k_capacity() ? kt_env : (uint32_t)topk_k();
      // Small windows: the GPU work is the same P x N in total, while fewer nodes are
      // touched per window, so fewer candidate lists lose certification.
      const uint32_t W = std::min<uint32_t>(P, greedy_window());
      PodGather win;
      std::vector<uint32_t> counts(2 * (size_t)W);
      std::vector<double> ts((size_t)KT * W);
      std::vector<uint32_t> ti((size_t)KT * W);
      std::vector<uint32_t> perm(W), pos(W), Tidx, ti2;
      std::vector<double> Tw, ts2;
      for (uint32_t ws = 0; ws < P; ws += W) {
        const uint32_t wn = std::min(W, P - ws);
        const auto tw = Clock::now();
        if ((rc = g.push_dirty())) return rc;
        for (uint32_t n : g.touched_list) g.touched_w[n] = 0;
        g.touched_list.clear();
        win.build(pods, order.data() + ws, wn);
        if ((rc = yoda_upload_pods(h, &win.soa))) return rc;
        if ((rc = prepare_run(h, YODA_MODE_SCV))) return rc;
        // sort the window like any batch (whole waves skip nodes); outputs stay in sorted
        // order and are read through pos[i] = sorted position of window pod i
        if ((rc = order_pods(h, YODA_MODE_SCV))) return rc;
        h->greedy_prep_ms += ms_since(tw);
        if (N > 0) {
          if ((rc = phase1(h, YODA_MODE_SCV, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(),
                           Maxima::Own)))
            return rc;
          HIP_TRY(h, launch_prep2(h->maxima.as<uint64_t>(), wn, h->rcp.as<double>(),
                                   h->stream));
          if ((rc = topk_lists(h, wn, KT, h->counts.as<uint32_t>()))) return rc;
          HIP_TRY(h, hipMemcpyAsync(counts.data(), h->counts.p, 2ull * wn * 4,
                                    hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(h, hipMemcpyAsync(ts.data(), h->tk_s.p, (size_t)KT * wn * 8,
                                    hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(h, hipMemcpyAsync(ti.data(), h->tk_i.p, (size_t)KT * wn * 4,
                                    hipMemcpyDeviceToHost, h->stream));
          if (h->ordered)
            HIP_TRY(h, hipMemcpyAsync(perm.data(), h->perm.p, (size_t)wn * 4,
                                      hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(h, hipStreamSynchronize(h->stream));
        } else {
          std::fill(counts.begin(), counts.end(), 0u);
        }
        for (uint32_t i = 0; i < wn; ++i) pos[i] = i;
        if (h->ordered)
          for (uint32_t q = 0; q < wn; ++q) pos[perm[q]] = q;
        // each list's certificate threshold: its last entry's window-start (or refresh-time)
        // score and node
        Tw.resize(wn), Tidx.resize(wn);
        auto set_thresholds = [&](uint32_t q) {
          const uint32_t len = std::max<uint32_t>(1, std::min<uint32_t>(counts[q], KT));
          Tw[q] = ts[(size_t)(len - 1) * wn + q];
          Tidx[q] = ti[(size_t)(len - 1) * wn + q];
        };
        for (uint32_t q = 0; q < wn; ++q) set_thresholds(q);
        ++h->greedy_windows;
        h->greedy_window_ms += ms_since(tw);
        const auto tr = Clock::now();
        double fb_ms = 0;
        bool wrapped = false;
        // the best current candidate of sorted position q (window-start score - old static +
        // new static) and whether it is certified: every node outside the list scored <= T at
        // window start (ties: higher index) and its score can only have dropped since
        auto certify = [&](uint32_t q, uint32_t* best_node) {
          const uint32_t nf = counts[q];
          const uint32_t len = std::min<uint32_t>(nf, KT);
          double bs = -1.0;
          uint32_t bi = 0xffffffffu;
          for (uint32_t k = 0; k < len; ++k) {
            const uint32_t node = ti[(size_t)k * wn + q];
            const uint32_t n = node - h->node_offset;
            double cur = ts[(size_t)k * wn + q];
            if (g.touched_w[n]) cur = cur - (double)g.stat_w[n] + (double)g.stat[n];
            if (cur > bs || (cur == bs && node < bi)) {
              bs = cur;
              bi = node;
            }
          }
          *best_node = bi;
          return nf <= KT || bs > Tw[q] || (bs == Tw[q] && bi <= Tidx[q]);
        };
        // Mid-window list refresh: a window whose lists went stale (similar pods took their
        // shared top nodes) would otherwise send each of its remaining similar pods to an
        // exact fallback.  Every kFbCheck (8) fallbacks the next kScan (256) window pods are
        // checked; if at least kScanMin (16) of them are uncertified already (they stay so:
        // scores only drop),
        // the window's top-k K2 runs again against the current state (the window's K1 masks
        // and maxima stay valid: only static scores change in this mode).  A refreshed entry
        // is stored as  score + old static - current static  of its node, so the certificate
        // above yields its current score from then on; the threshold is the refresh-time
        // score (unlisted nodes scored at most that then and only dropped since).
        // YODA_GREEDY_REFRESH=0: off (A/B knob).
        static const bool refresh_on = YODA_KNOB("YODA_GREEDY_REFRESH", 1) != 0;
        // (YODA_GREEDY_REFRESH_EVERY / _MIN: A/B knobs for the check period and the bar)
        static const uint32_t kFbCheck =
            std::max<uint32_t>(1, YODA_KNOB("YODA_GREEDY_REFRESH_EVERY", 8));
        static const uint32_t kScanMin = YODA_KNOB("YODA_GREEDY_REFRESH_MIN", 16);
        constexpr uint32_t kScan = 256;
        uint32_t fb_since = 0;
        auto maybe_refresh = [&](uint32_t i) -> int {
          if (!refresh_on || wrapped || N == 0 || ++fb_since < kFbCheck || wn - i < 2 * kScan)
            return YODA_OK;
          fb_since = 0;
          uint32_t unc = 0, bj;
          for (uint32_t j = i + 1; j < std::min(wn, i + 1 + kScan); ++j) {
            const uint32_t qj = pos[j];
            if (counts[qj] >= 2 && counts[(size_t)wn + qj] == 0 && !certify(qj, &bj)) ++unc;
          }
          if (unc < kScanMin) return YODA_OK;
          int r = g.push_dirty();
          if (r) return r;
          if ((r = topk_lists(h, wn, KT, h->counts.as<uint32_t>()))) return r;
          ts2.resize((size_t)KT * wn), ti2.resize((size_t)KT * wn);
          HIP_TRY(h, hipMemcpyAsync(ts2.data(), h->tk_s.p, (size_t)KT * wn * 8,
                                    hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(h, hipMemcpyAsync(ti2.data(), h->tk_i.p, (size_t)KT * wn * 4,
                                    hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(h, hipStreamSynchronize(h->stream));
          for (uint32_t j = i; j < wn; ++j) {
            const uint32_t qj = pos[j];
            const uint32_t len = std::min<uint32_t>(counts[qj], KT);
            for (uint32_t k = 0; k < len; ++k) {
              const size_t o = (size_t)k * wn + qj;
              const uint32_t n = ti2[o] - h->node_offset;
              ti[o] = ti2[o];
              ts[o] = g.touched_w[n] ? ts2[o] + (double)g.stat_w[n] - (double)g.stat[n] : ts2[o];
            }
            if (len) {
              Tw[qj] = ts2[(size_t)(len - 1) * wn + qj];
              Tidx[qj] = ti2[(size_t)(len - 1) * wn + qj];
            }
          }
          ++h->greedy_refreshes;
          return YODA_OK;
        };
        for (uint32_t i = 0; i < wn; ++i) {
          const uint32_t p = order[ws + i];
          const uint32_t q = pos[i];  // sorted position: the device outputs' index
          const uint32_t nf = counts[q], nz = counts[(size_t)wn + q];
          int32_t pk;
          if (nf == 0) {
            pk = YODA_PICK_NONE;
          } else if (nf >= 2 && nz > 0) {
            pk = YODA_PICK_ERROR;  // Score would divide by TotalMemorySum == 0
          } else if (nf == 1) {
            pk = (int32_t)ti[q];   // the only feasible node, returned without scoring
          } else if (wrapped) {
            const auto tf = Clock::now();
            if ((rc = greedy_eval_fast(g, q, &pk))) return rc;
            ++h->greedy_fallbacks;
            fb_ms += ms_since(tf);
          } else {
            uint32_t bi;
            bool certified = certify(q, &bi);
            if (!certified) {
              const auto tf = Clock::now();
              const uint32_t before = h->greedy_refreshes;
              if ((rc = maybe_refresh(i))) return rc;
              if (h->greedy_refreshes != before) certified = certify(q, &bi);
              if (!certified) {
                if ((rc = greedy_eval_fast(g, q, &pk))) return rc;
                ++h->greedy_fallbacks;
              }
              fb_ms += ms_since(tf);
            }
            if (certified) pk = (int32_t)bi;
          }
          pick[p] = pk;
          if (pk >= 0) {
            const uint32_t n = (uint32_t)pk - h->node_offset;
            const uint64_t before = g.alloc[n];
            apply_pick(p, pk);
            if (g.alloc[n] < before) wrapped = true;  // Allocate may grow: stop certifying
          }
        }
        h->greedy_fallback_ms += fb_ms;
        h->greedy_resolve_ms += ms_since(tr) - fb_ms;
      }
    }
    if (std::getenv("YODA_GREEDY_DEBUG"))
      std::fprintf(stderr, "greedy: windows %u (%.1f ms, of which host prep %.1f ms), fallbacks %u "
                   "(%.1f ms), resolve %.1f ms\n", h->greedy_windows, h->greedy_window_ms,
                   h->greedy_prep_ms, h->greedy_fallbacks, h->greedy_fallback_ms,
                   h->greedy_resolve_ms);
    if (std::getenv("YODA_GREEDY_DEBUG"))
      std::fprintf(stderr, "greedy: mid-window list refreshes %u\n", h->greedy_refreshes);
    // Leave the uploaded snapshot unchanged: restore static score and CardNumber.
    for (uint32_t n : all_touched) {
      g.stat[n] = stat0[n];
      g.card_number[n] = h->h_card_number[n];
    }
    if ((rc = g.push(all_touched, nullptr))) return rc;
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    h->ran = false;
    return YODA_OK;
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_greedy_restarts(const yoda_t* h, uint32_t* restarts) {
  if (!h || !restarts) return YODA_ERR_INVALID_ARG;
  *restarts = h->greedy_restarts;
  return YODA_OK;
}

int yoda_greedy_refreshes(const yoda_t* h, uint32_t* refreshes) {
  if (!h || !refreshes) return YODA_ERR_INVALID_ARG;
  *refreshes = h->greedy_refreshes;
  return YODA_OK;
}

int yoda_greedy_stats(const yoda_t* h, uint32_t* windows, uint32_t* fallbacks,
                      double* times_ms) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (windows) *windows = h->greedy_windows;
  if (fallbacks) *fallbacks = h->greedy_fallbacks;
  if (times_ms) {
    times_ms[0] = h->greedy_window_ms;
    times_ms[1] = h->greedy_resolve_ms;
    times_ms[2] = h->greedy_fallback_ms;
  }
  return YODA_OK;
}

// ---- sharded greedy (config 5 across GPUs) ---------------------------------------------
// Each rank's handle holds a node shard.  Per window: yoda_shard_phase1 (+ MAX/SUM
// all-reduce) -> yoda_shard_topk (local top-k with the global maxima) -> the caller merges
// the shards' lists -> the host session resolves the window in queue order; pods it cannot
// certify are scored exactly on every shard (yoda_shard_best_one) and merged by the caller.
// Between steps the caller pushes the nodes the session changed (yoda_gs_take_dirty ->
// yoda_set_node_state on every shard).

int yoda_topk_k(void) { return topk_k(); }
int yoda_topk_k_capacity(void) { return topk_k_capacity(); }

namespace {

// Overwrite the static score (and CardNumber) of a few local nodes on the device.
int push_node_state(yoda_t* h, const std::vector<uint32_t>& loc, const std::vector<uint64_t>& val,
                    const std::vector<uint64_t>& cn) {
  const uint32_t cnt = (uint32_t)loc.size();
  if (cnt == 0) return YODA_OK;
  const size_t o_val = ((size_t)cnt * 4 + 15) / 16 * 16, o_cn = o_val + (size_t)cnt * 8;
  const size_t bytes = o_cn + (size_t)cnt * 8;
  if (h->upd_pending) HIP_TRY(h, hipEventSynchronize(h->upd_event));
  HIP_TRY(h, h->upd_stage.ensure(bytes));
  HIP_TRY(h, h->upd_node.ensure(bytes));
  unsigned char* st = static_cast<unsigned char*>(h->upd_stage.p);
  std::memcpy(st, loc.data(), (size_t)cnt * 4);
  std::memcpy(st + o_val, val.data(), (size_t)cnt * 8);
  std::memcpy(st + o_cn, cn.data(), (size_t)cnt * 8);
  HIP_TRY(h, hipMemcpyAsync(h->upd_node.p, st, bytes, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(h, hipEventRecord(h->upd_event, h->stream));
  h->upd_pending = true;
  unsigned char* d = h->upd_node.as<unsigned char>();
  const uint32_t stride = h->path == Path::N32 ? n32_stride(h->K) : node_stride(h->K);
  h->blksum_loose = true;  // (the atomics keep the block bounds valid, not tight)
  for (uint32_t t = 0; t < cnt; ++t) {  // the K2 block bounds stay valid while scores only fall
    uint64_t sv = val[t];
    if (!h->generic) {
      double d;
      std::memcpy(&d, &val[t], 8);
      sv = (uint64_t)d;
    }
    h->note_static(loc[t], sv);
  }
  HIP_TRY(h, launch_set_static(h->nodes.as<unsigned char>(), stride,
                               reinterpret_cast<const uint32_t*>(d),
                               reinterpret_cast<const uint64_t*>(d + o_val),
                               reinterpret_cast<const uint64_t*>(d + o_cn), cnt,
                               h->has_k1sum ? h->k1sum.as<unsigned char>() : nullptr,
                               k1sum_stride(h->K),
                               h->has_k2sum ? h->k2sum.as<unsigned char>() : nullptr,
                               k2sum_stride(h->K), h->perm_copy(), h->stream));
  return YODA_OK;
}

}  // namespace

int yoda_set_node_state(yoda_t* h, uint32_t count, const uint32_t* nodes, const uint64_t* alloc,
                        const uint64_t* card_number) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!h->has_nodes) return fail(h, YODA_ERR_NO_NODES, "no node snapshot uploaded");
  if (count && (!nodes || !alloc || !card_number))
    return fail(h, YODA_ERR_INVALID_ARG, "NULL node state array");
  try {
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<uint32_t> loc;
    std::vector<uint64_t> stat, val, cn;
    for (uint32_t t = 0; t < count; ++t) {
      if (nodes[t] < h->node_offset || nodes[t] - h->node_offset >= h->n_nodes) continue;
      const uint32_t i = nodes[t] - h->node_offset;
      bool z = false;
      const uint64_t s = static_score(h->h_free_sum[i], h->h_total_sum[i], alloc[t], &z);
      if (!h->generic && s >= (1ull << 51))
        return fail(h, YODA_ERR_RANGE, "static score leaves the fast path; re-upload the nodes");
      loc.push_back(i);
      stat.push_back(s);
      cn.push_back(card_number[t]);
      uint64_t bits = s;
      if (!h->generic) {
        const double d = (double)s;
        std::memcpy(&bits, &d, 8);
      }
      val.push_back(bits);
    }
    // keep the host copies current (yoda_update_alloc / yoda_greedy start from them)
    const size_t stride = h->path == Path::N32 ? n32_stride(h->K) : node_stride(h->K);
    for (size_t t = 0, ti = 0; t < count; ++t) {
      if (nodes[t] < h->node_offset || nodes[t] - h->node_offset >= h->n_nodes) continue;
      const uint32_t i = loc[ti];
      h->h_alloc[i] = alloc[t];
      h->h_card_number[i] = cn[ti];
      unsigned char* r = h->host_records.data() + (size_t)i * stride;
      std::memcpy(r, &val[ti], 8);       // header word 0: static score
      std::memcpy(r + 8, &cn[ti], 8);    // header word 1: CardNumber
      if (h->has_k2sum) {
        h->host_k2sum[sum_index(i, kS2Static, k2sum_stride(h->K))] = (uint32_t)val[ti];
        h->host_k2sum[sum_index(i, kS2Static + 1, k2sum_stride(h->K))] = (uint32_t)(val[ti] >> 32);
      }
      ++ti;
    }
    return push_node_state(h, loc, val, cn);
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_topk_depth(const yoda_t* h) {
  if (!h) return YODA_ERR_INVALID_ARG;
  // the capacity windows' deeper lists after the witness phase 1 (yoda_greedy's depths)
  return h->phase1_wit ? topk_k_capacity() : topk_k();
}

namespace {
int shard_topk_impl(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_counts, uint32_t k,
                    uint32_t deep, uint32_t* counts, double* top_score, uint32_t* top_node);
}  // namespace

int yoda_shard_topk(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_counts, uint32_t k,
                    uint32_t* counts, double* top_score, uint32_t* top_node) {
  return shard_topk_impl(h, d_maxima, d_counts, k, 0, counts, top_score, top_node);
}

namespace {
// deep > 0 (libyoda's sharded capacity windows): lists `deep` long, exact down to their last
// entry and empty past it -- the 8-deep chunk lists merged deeper where the block kernels run
// (k_topk_merge_deep), else the k-deep lists padded -- whatever this shard's kernels.
int shard_topk_impl(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_counts, uint32_t k,
                    uint32_t deep, uint32_t* counts, double* top_score, uint32_t* top_node) {
  int rc = check_ready(h, YODA_MODE_SCV);
  if (rc) return rc;
  if (h->xo)  // (the window top-k reads the shared radix order's buffers)
    return fail(h, YODA_ERR_STATE, "yoda_shard_topk after a caller-order phase 1: turn "
                                   "yoda_shard_exchange_order off for greedy windows");
  if (!h->phase1_done) return fail(h, YODA_ERR_STATE, "yoda_shard_topk before yoda_shard_phase1");
  if (h->generic)
    return fail(h, YODA_ERR_STATE, "top-k lists need a fast record path (N32 or F64)");
  if (!d_maxima || !d_counts || !counts || !top_score || !top_node)
    return fail(h, YODA_ERR_INVALID_ARG, "NULL buffer");
  const uint32_t KT = (uint32_t)yoda_shard_topk_depth(h);
  if (k != KT)
    return fail(h, YODA_ERR_INVALID_ARG,
                "yoda_shard_topk: k = " + std::to_string(k) + " but this phase 1 lists " +
                    std::to_string(KT) + " candidates per pod (yoda_shard_topk_depth)");
  try {
    const uint32_t P = h->n_pods, N = h->n_nodes;
    h->h_pos.resize(P);
    for (uint32_t i = 0; i < P; ++i) h->h_pos[i] = i;
    h->topk_ready = false;
    if (P == 0) return YODA_OK;
    const uint32_t KO = std::max(KT, deep);  // the depth written to the caller
    std::vector<uint32_t> cnt(2 * (size_t)P), ti((size_t)KO * P, 0xffffffffu), perm(P);
    std::vector<double> ts((size_t)KO * P, -1.0);
    uint32_t KD = KT;  // the depth the device lists hold
    HIP_TRY(h, hipMemcpyAsync(h->maxima.p, d_maxima, 6ull * P * 8, hipMemcpyDeviceToDevice,
                              h->stream));
    HIP_TRY(h, hipMemcpyAsync(cnt.data(), d_counts, 2ull * P * 4, hipMemcpyDeviceToHost,
                              h->stream));
    if (N > 0) {
      HIP_TRY(h, launch_prep2(h->maxima.as<uint64_t>(), P, h->rcp.as<double>(),
                               h->stream));
      if (deep > KT && topk_block_ok(h)) {
        if ((rc = topk_lists(h, P, (uint32_t)topk_k(), d_counts, deep, &KD))) return rc;
      } else if ((rc = topk_lists(h, P, KT, d_counts))) {
        return rc;
      }
      HIP_TRY(h, hipMemcpyAsync(ts.data(), h->tk_s.p, (size_t)KD * P * 8, hipMemcpyDeviceToHost,
                                h->stream));
      HIP_TRY(h, hipMemcpyAsync(ti.data(), h->tk_i.p, (size_t)KD * P * 4, hipMemcpyDeviceToHost,
                                h->stream));
    }
    if (h->ordered)
      HIP_TRY(h, hipMemcpyAsync(perm.data(), h->perm.p, (size_t)P * 4, hipMemcpyDeviceToHost,
                                h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    if (h->ordered)
      for (uint32_t q = 0; q < P; ++q) h->h_pos[perm[q]] = q;  // perm[q]: pod at sorted q
    for (uint32_t i = 0; i < P; ++i) {
      const uint32_t q = h->h_pos[i];
      counts[i] = cnt[q];
      counts[(size_t)P + i] = cnt[(size_t)P + q];
      for (uint32_t k = 0; k < KO; ++k) {
        top_score[(size_t)k * P + i] = k < KD ? ts[(size_t)k * P + q] : -1.0;
        top_node[(size_t)k * P + i] = k < KD ? ti[(size_t)k * P + q] : 0xffffffffu;
      }
    }
    h->topk_ready = true;
    return YODA_OK;
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}
}  // namespace

int yoda_shard_phase1_witness(yoda_t* h, uint64_t* d_maxima, uint32_t* d_counts,
                              uint32_t* d_wit) {
  if (!h) return YODA_ERR_INVALID_ARG;
  h->xo = false;  // (greedy windows: the shared radix order)
  int rc = prepare_run(h, YODA_MODE_SCV);
  if (rc) return rc;
  if (h->generic)
    return fail(h, YODA_ERR_STATE, "witness phase 1 needs a fast record path (N32 or F64)");
  if (!d_maxima || !d_counts || !d_wit) return fail(h, YODA_ERR_INVALID_ARG, "NULL buffer");
  try {
    if ((rc = order_pods(h, YODA_MODE_SCV))) return rc;
    if ((rc = phase1_witness(h, d_maxima, d_counts, d_wit, h->node_offset))) return rc;
    h->phase1_done = true;
    h->phase1_wit = true;
    h->ran = false;
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_witness_prepare(yoda_t* h, const uint64_t* d_maxima_global,
                               const uint64_t* d_maxima_local, uint32_t* d_wit) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!d_maxima_global || !d_maxima_local || !d_wit)
    return fail(h, YODA_ERR_INVALID_ARG, "NULL buffer");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, launch_wit_prepare(d_maxima_global, d_maxima_local, h->n_pods, d_wit, h->stream));
  return YODA_OK;
}

int yoda_shard_witness_download(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_wit,
                                uint64_t* maxima, uint32_t* wit) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!d_maxima || !d_wit || !maxima || !wit) return fail(h, YODA_ERR_INVALID_ARG, "NULL buffer");
  if (!h->topk_ready)
    return fail(h, YODA_ERR_STATE, "yoda_shard_witness_download before yoda_shard_topk");
  try {
    const uint32_t P = h->n_pods;
    if (P == 0) return YODA_OK;
    HIP_TRY(h, hipSetDevice(h->device));
    std::vector<uint64_t> mx(6 * (size_t)P);
    std::vector<uint32_t> wt(12 * (size_t)P);
    HIP_TRY(h, hipMemcpyAsync(mx.data(), d_maxima, mx.size() * 8, hipMemcpyDeviceToHost,
                              h->stream));
    HIP_TRY(h, hipMemcpyAsync(wt.data(), d_wit, wt.size() * 4, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    for (uint32_t i = 0; i < P; ++i) {
      const uint32_t q = h->h_pos[i];
      for (int f = 0; f < 6; ++f) maxima[(size_t)f * P + i] = mx[(size_t)f * P + q];
      for (int f = 0; f < 12; ++f) wit[(size_t)f * P + i] = wt[(size_t)f * P + q];
    }
    return YODA_OK;
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_shard_best_one(yoda_t* h, uint32_t pod, double* score, int32_t* node) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!score || !node) return fail(h, YODA_ERR_INVALID_ARG, "NULL output");
  if (!h->topk_ready) return fail(h, YODA_ERR_STATE, "yoda_shard_best_one before yoda_shard_topk");
  if (pod >= h->n_pods) return fail(h, YODA_ERR_INVALID_ARG, "pod index out of range");
  *score = -1.0;
  *node = -1;
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->n_nodes == 0) return YODA_OK;
  const uint32_t s = h->h_pos[pod];
  const uint32_t nb = greedy_one_blocks();
  if (h->g1_done.bytes == 0) {
    HIP_TRY(h, h->g1_done.ensure(16));
    HIP_TRY(h, hipMemsetAsync(h->g1_done.p, 0, 16, h->stream));
  }
  HIP_TRY(h, h->g1_part.ensure((size_t)nb * 12 + 16));
  double* ps = h->g1_part.as<double>();
  uint32_t* pi = reinterpret_cast<uint32_t*>(ps + nb);
  uint32_t* done = h->g1_done.as<uint32_t>();
  HIP_TRY(h, launch_greedy_one(h->K, h->path, h->nodes.as<unsigned char>(),
                               h->has_k2sum ? h->k2sum.as<unsigned char>() : nullptr, h->n_nodes,
                               pod_params(h), h->rcp.as<double>(), 
                               h->n_pods, s, h->bitmask.as<uint64_t>(), bm_row(h->n_nodes),
                               h->bs_ptr(), bs_row(h->n_nodes), h->blk_ptr(),
                               blk_row(h->n_nodes), ps, pi, done, done + 1, h->stream));
  HIP_TRY(h, h->pick_stage.ensure(16));
  HIP_TRY(h, hipMemcpyAsync(h->pick_stage.p, done, 16, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  const unsigned char* st = static_cast<const unsigned char*>(h->pick_stage.p);
  uint32_t n;
  double b;
  std::memcpy(&n, st + 4, 4);
  std::memcpy(&b, st + 8, 8);
  if (n != 0xffffffffu) {
    *node = (int32_t)(n + h->node_offset);
    *score = b;
  }
  return YODA_OK;
}

}  // extern "C"

// ---- host-side greedy session ---------------------------------------------------------
// The sequential part of the greedy batch (yoda_greedy's resolve), over the GLOBAL node set,
// fed with merged candidate lists.  Pure host code: identical on every rank.
struct yoda_greedy_session {
  static constexpr uint32_t kCrossQ = 64;  // capacity mode: per-q removal counts up to here
  uint32_t N = 0, P = 0, flags = 0;
  std::vector<uint64_t> free_sum, total_sum, alloc, card_number, alloc0, cn0, stat, stat_w;
  std::vector<uint64_t> cn_w;  // CardNumber of a window-touched node at the window start
  std::vector<uint8_t> has_memory, has_number, has_clock, touched_w, dirty, ever;
  std::vector<uint64_t> memory, number, clock;
  // capacity mode: the nodes' cards (when the snapshot passed them), [N][K] in CardField
  // order, to tell which lost nodes were witnesses of a pod's maxima
  uint32_t K = 0;
  std::vector<uint64_t> cards;  // [N][6][K]
  std::vector<uint32_t> hmask, rmask;  // healthy / real card bits per node
  std::vector<uint32_t> order, touched_list, dirty_list, ever_list;
  std::vector<int32_t> pick;
  // current window (queue positions [ws, ws + wn)), inputs in window order
  uint32_t ws = 0, wn = 0, k = 0, next = 0, resolved = 0, assigned = 0, refreshes = 0;
  bool in_window = false, wrapped = false;
  // some node's static score rose within the window (never, short of a wrap: Allocate only
  // grows): a listed node's current score may then exceed its window-start one
  bool stat_rose = false;
  std::vector<uint32_t> counts, ti_own;
  std::vector<double> ts_own;
  // the window's lists [k][wn]: the session's copies, or (greedy_capacity, gs_begin_window_at)
  // the caller's staging, valid until the window ends
  double* ts = nullptr;
  uint32_t* ti = nullptr;
  // entry kk of window pod i: [k][wn] (the API's layout), or [wn][k] (row_major: a pod's list
  // contiguous, as k_window_out writes the capacity windows' staging)
  bool row_major = false;
  size_t at(uint32_t i, uint32_t kk) const {
    return row_major ? (size_t)i * k + kk : (size_t)kk * wn + i;
  }
  // each list's certificate threshold (flags 0): its last entry's window-start -- or, after a
  // mid-window refresh (yoda_gs_refresh), refresh-time -- score and node
  std::vector<double> Tw;
  // entries of each list before its first empty one (a deep merge stops where it is no longer
  // exact, k_topk_merge_deep): the list holds every feasible node only when that is nf
  std::vector<uint32_t> vlen;
  std::vector<uint32_t> Tix;
  // YODA_GREEDY_CARD_CAPACITY (greedy): cross[q] = window-touched nodes whose
  // CardNumber has dropped from >= q (window start) to < q, i.e. nodes a pod needing q cards
  // has lost since its candidate list was made; and the window's PreScore maxima with their
  // witnesses ([6][wn] each, window order), when the caller supplied them.
  uint32_t cross[kCrossQ + 1] = {};
  std::vector<uint32_t> cross_list[kCrossQ + 1];  // the nodes counted in cross[q]
  bool has_wit = false;
  std::vector<uint64_t> wmax;
  std::vector<uint32_t> wcnt, wnode;

  void apply(uint32_t p, int32_t node) {
    if (node < 0) return;
    const uint32_t n = (uint32_t)node;
    if (!touched_w[n]) {
      touched_w[n] = 1;
      stat_w[n] = stat[n];
      cn_w[n] = card_number[n];
      touched_list.push_back(n);
    }
    if (!dirty[n]) {
      dirty[n] = 1;
      dirty_list.push_back(n);
    }
    if (!ever[n]) {
      ever[n] = 1;
      ever_list.push_back(n);
    }
    const uint64_t before = alloc[n];
    if (has_memory[p]) alloc[n] += memory[p];  // uint64 wrap (algorithm.go:301)
    if (alloc[n] < before) wrapped = true;     // Allocate may grow: stop certifying
    if (flags & YODA_GREEDY_CARD_CAPACITY) {
      const uint64_t num = has_number[p] ? number[p] : 1;
      const uint64_t a = card_number[n], b = a >= num ? a - num : 0;
      card_number[n] = b;
      // pods needing q in (b, a] cards have just lost this node
      for (uint64_t q = b + 1; q <= std::min<uint64_t>(a, kCrossQ); ++q) {
        ++cross[q];
        cross_list[q].push_back(n);
      }
    }
    bool z;
    const int64_t before_stat = stat[n];
    stat[n] = static_score(free_sum[n], total_sum[n], alloc[n], &z);
    if (stat[n] > before_stat) stat_rose = true;
  }
  // PodFitsNumber operand of pod p (filter.go:11-16): the label, or 1 (CardNumber > 0)
  uint64_t need_cards(uint32_t p) const { return has_number[p] ? number[p] : 1; }
  // node n was feasible for a pod needing q cards at the window start and is not any more
  bool removed(uint32_t n, uint64_t q) const {
    return touched_w[n] && card_number[n] < q && cn_w[n] >= q;
  }
  // how many nodes a pod needing q cards has lost in this window (an upper bound on its
  // feasible nodes lost: a touched node may never have passed its other predicates)
  uint64_t lost(uint64_t q) const {
    if (q <= kCrossQ) return cross[q];
    uint64_t r = 0;
    for (uint32_t n : touched_list) r += removed(n, q) ? 1 : 0;
    return r;
  }
  // Node n passed pod p's Filter at the window start (it needs q cards; PodFitsNumber held
  // then, n being a lost node): PodFitsMemory / PodFitsClock (filter.go:18-50) on its cards.
  bool fit_ws(uint32_t n, uint32_t p, uint64_t q) const {
    const uint64_t* c = cards.data() + (size_t)n * 6 * K;
    uint64_t cm = 0, cc = 0;
    for (uint32_t j = 0; j < K; ++j) {
      if (!((hmask[n] >> j) & 1u)) continue;
      cm += c[0 * K + j] >= memory[p];  // kFree
      cc += c[1 * K + j] == clock[p];   // kClock
    }
    return (!has_memory[p] || cm >= q) && (!has_clock[p] || cc >= q);
  }
  // Node n's contribution to pod p's maxima (ProcessMaxValueWithCard over the cards with
  // FreeMemory >= m and Clock >= c, collection.go:46-76), MaxValue field order.
  // per node (MaxValue order) the largest value over its real cards: no pod's contrib() from
  // the node exceeds it (scan_lost skips nodes that cannot be a witness)
  std::vector<uint64_t> nodemax;
  bool contrib(uint32_t n, uint32_t p, uint64_t v[6]) const {
    const uint64_t* c = cards.data() + (size_t)n * 6 * K;
    const uint64_t m = has_memory[p] ? memory[p] : 0, ck = has_clock[p] ? clock[p] : 0;
    bool any = false;
    for (int f = 0; f < 6; ++f) v[f] = 0;
    for (uint32_t j = 0; j < K; ++j) {
      if (!((rmask[n] >> j) & 1u) || c[0 * K + j] < m || c[1 * K + j] < ck) continue;
      any = true;
      // CardField (free, clock, total, bw, core, power) -> MaxValue (bw, clock, core, free,
      // power, total)
      v[0] = std::max(v[0], c[3 * K + j]);
      v[1] = std::max(v[1], c[1 * K + j]);
      v[2] = std::max(v[2], c[4 * K + j]);
      v[3] = std::max(v[3], c[0 * K + j]);
      v[4] = std::max(v[4], c[5 * K + j]);
      v[5] = std::max(v[5], c[2 * K + j]);
    }
    return any;
  }
  // The nodes pod p (needing q cards, window pod i) has lost in this window, examined with
  // the cards at hand: how many had passed its Filter at the window start (lf), how many of
  // those had TotalMemorySum == 0 (lz), and how many were witnesses of each of its maxima
  // (lw).  False (nothing computed) without the cards or when too many nodes were lost.
  static constexpr uint64_t kExactLost = 512;
  // witness_only: the caller needs lw only (nf0 >= 2 + lq and no zero-total node at the window
  // start: lf and lz cannot change its outcome) -- and only for the fields whose witnesses lq
  // lost nodes could all be (wcnt <= lq); a node below every such maximum is skipped unvisited
  // (lf / lz then count only the visited nodes)
  bool scan_lost(uint32_t i, uint32_t p, uint64_t q, uint64_t lq, uint64_t* lf, uint64_t* lz,
                 uint64_t lw[6], bool witness_only = false) const {
    *lf = *lz = 0;
    for (int f = 0; f < 6; ++f) lw[f] = 0;
    if (lq == 0) return true;
    if (cards.empty() || lq > kExactLost) return false;
    ++n_scan;
    uint32_t fmask = 0x3fu;
    if (witness_only && has_wit) {
      fmask = 0;
      for (int f = 0; f < 6; ++f) {
        const size_t o = (size_t)f * wn + i;
        if (wmax[o] > 1 && wcnt[o] <= lq) fmask |= 1u << f;
      }
      if (fmask == 0) return true;
    }
    auto visit = [&](uint32_t x) {
      if (witness_only && has_wit) {
        const uint64_t* nm = nodemax.data() + (size_t)x * 6;
        bool maybe = false;
        for (int f = 0; f < 6 && !maybe; ++f)
          maybe = ((fmask >> f) & 1u) && nm[f] >= wmax[(size_t)f * wn + i];
        if (!maybe) return;
      }
      ++n_scan_nodes;
      if (!fit_ws(x, p, q)) return;
      ++*lf;
      *lz += total_sum[x] == 0 ? 1 : 0;
      uint64_t v[6];
      if (has_wit && contrib(x, p, v))
        for (int f = 0; f < 6; ++f) lw[f] += v[f] == wmax[(size_t)f * wn + i] ? 1 : 0;
    };
    if (q <= kCrossQ) {
      for (uint32_t x : cross_list[q]) visit(x);
    } else {
      for (uint32_t x : touched_list)
        if (removed(x, q)) visit(x);
    }
    return true;
  }
  // CollectMaxValues over the remaining feasible nodes still gives window pod i's maxima:
  // every field keeps a witness.  A maximum of 1 is the floor and cannot drop
  // (collection.go:31-38).  Exact: a field keeps its maximum iff fewer of its witnesses were
  // lost than it had (lw from scan_lost).  Bounds only: more witnesses than lost nodes, or a
  // single witness that is not lost.
  bool maxima_kept(uint32_t i, uint64_t q, uint64_t lq, bool exact, const uint64_t lw[6]) const {
    if (lq == 0) return true;
    if (!has_wit) return false;
    for (int f = 0; f < 6; ++f) {
      const size_t o = (size_t)f * wn + i;
      if (wmax[o] <= 1) continue;
      if (exact) {
        if (wcnt[o] > lw[f]) continue;
      } else {
        if (wcnt[o] > lq) continue;
        if (wcnt[o] == 1 && wnode[o] < N && !removed(wnode[o], q)) continue;
      }
      return false;
    }
    return true;
  }
  // Capacity-mode resolve of window pod i (input pod p): true with *pk when certified.
  bool resolve_capacity(uint32_t i, uint32_t p, int32_t* pk);
  // flags 0: window pod i's best current candidate (window-start score - old static + new
  // static) and whether the list certifies it: every unlisted node scored <= T at the window
  // start or last refresh (ties: higher index) and its score can only have dropped since
  bool certify0(uint32_t i, uint32_t* best) const {
    const uint32_t nf = counts[i], len = std::min<uint32_t>(nf, vlen[i]);
    double bs = -1.0;
    uint32_t bi = 0xffffffffu;
    for (uint32_t kk = 0; kk < len; ++kk) {  // (the listed entries: none empty, every id < N)
      const uint32_t n = ti[at(i, kk)];
      double cur = ts[at(i, kk)];
      if (touched_w[n]) cur = cur - (double)stat_w[n] + (double)stat[n];
      if (cur > bs || (cur == bs && n < bi)) {
        bs = cur;
        bi = n;
      }
    }
    *best = bi;
    if (bi == 0xffffffffu) return false;  // nothing listed
    return (nf <= k && vlen[i] >= nf) || bs > Tw[i] || (bs == Tw[i] && bi <= Tix[i]);
  }
  // why capacity certificates failed: wrap, few feasible left, zero-total, maxima, list
  // exhausted, below the threshold
  uint64_t why[6] = {};
  // (diagnostics, YODA_GREEDY_DEBUG) capacity resolves, lost-node scans and nodes they visited
  mutable uint64_t n_resolve = 0, n_scan = 0, n_scan_nodes = 0;
};

bool yoda_greedy_session::resolve_capacity(uint32_t i, uint32_t p, int32_t* pk) {
  const uint32_t KT = k;
  const uint32_t nf0 = counts[i], nz0 = counts[(size_t)wn + i];
  ++n_resolve;
  if (nf0 == 0) {  // feasibility only shrinks: still no node
    *pk = YODA_PICK_NONE;
    return true;
  }
  if (wrapped) return ++why[0], false;
  const uint64_t q = need_cards(p);
  const uint32_t len = std::min<uint32_t>(nf0, KT);
  // the list holds every feasible node of the window start
  const bool whole = nf0 <= KT && vlen[i] >= nf0;
  const uint64_t lq = lost(q);
  uint32_t alive = 0, first = 0xffffffffu, alive_zero = 0;
  double bs = -1.0;
  uint32_t bi = 0xffffffffu;
  // the list's best current candidate; alive / first / alive_zero too on a full scan.  A
  // partial scan stops at the first entry whose window-start score is below the best so far:
  // the list is in descending window-start order and a score only falls in a window (deep
  // lists, k_topk_merge_deep, make the full scan the resolve's main cost)
  auto scan = [&](bool full) {
    alive = 0, first = 0xffffffffu, alive_zero = 0;
    bs = -1.0, bi = 0xffffffffu;
    for (uint32_t kk = 0; kk < len; ++kk) {
      const size_t o = at(i, kk);
      if (!full && ts[o] < bs) break;
      const uint32_t n = ti[o];
      if (n >= N || removed(n, q)) continue;
      ++alive;
      if (first == 0xffffffffu) first = n;
      alive_zero += total_sum[n] == 0 ? 1u : 0u;
      double cur = ts[o];
      if (touched_w[n]) cur = cur - (double)stat_w[n] + (double)stat[n];
      if (cur > bs || (cur == bs && n < bi)) {
        bs = cur;
        bi = n;
      }
    }
  };
  const bool full_scan = whole || stat_rose;
  scan(full_scan);
  uint64_t lf = 0, lz = 0, lw[6] = {};
  // The bounds-only certificate first (no card scan): whatever it certifies, the exact one
  // certifies with the same outcome (nf0 >= 2 + lq leaves >= 2 feasible nodes; a field with
  // more witnesses than lost nodes, or an unlost single witness, keeps its maximum since
  // lw[f] <= lq).  The lost nodes' cards are examined only when it fails.
  bool exact = false;
  if (!whole && lq > 0 && nf0 >= 2 + lq && nz0 == 0 && bi != 0xffffffffu &&
      maxima_kept(i, q, lq, false, lw)) {
    // (falls through to the list certificate below with exact == false)
  } else {
    exact = scan_lost(i, p, q, lq, &lf, &lz, lw, nf0 >= 2 + lq && nz0 == 0);
  }
  if (whole) {
    if (alive == 0) {
      *pk = YODA_PICK_NONE;
      return true;
    }
    if (alive == 1) {  // k8s returns the only feasible node without scoring
      *pk = (int32_t)first;
      return true;
    }
    if (alive_zero > 0) {  // Score would divide by TotalMemorySum == 0
      *pk = YODA_PICK_ERROR;
      return true;
    }
  } else if (exact) {
    // the feasible set is the window start's minus the lost nodes that were in it
    const uint64_t nf = nf0 - std::min<uint64_t>(nf0, lf);
    if (nf == 0) {
      *pk = YODA_PICK_NONE;
      return true;
    }
    if (nf == 1) {  // the only feasible node: listed and alive, or somewhere unlisted
      if (!full_scan) scan(true);
      if (alive != 1) return ++why[1], false;
      *pk = (int32_t)first;
      return true;
    }
    if (nz0 > lz) {  // a feasible zero-total node remains
      *pk = YODA_PICK_ERROR;
      return true;
    }
  } else {
    if (nf0 < 2 + lq) return ++why[1], false;  // might be down to 0 or 1 feasible nodes
    if (nz0 > 0) {
      if (lq > 0) return ++why[2], false;      // a zero-total node may be among the lost ones
      *pk = YODA_PICK_ERROR;
      return true;
    }
  }
  if (!maxima_kept(i, q, lq, exact, lw)) return ++why[3], false;  // unlisted scores may move
  if (bi == 0xffffffffu) return ++why[4], false;       // every listed node lost
  if (!whole) {
    // every unlisted node scored <= T at the window start or the list's last refresh (ties:
    // higher index) and has only lost Allocate since, or feasibility
    if (!(bs > Tw[i] || (bs == Tw[i] && bi <= Tix[i]))) return ++why[5], false;
  }
  *pk = (int32_t)bi;
  return true;
}

extern "C" {

int yoda_gs_create(const yoda_node_soa* nodes, const yoda_pod_soa* pods, uint32_t flags,
                   yoda_gs_t** out) {
  if (!out || !nodes || !pods) return YODA_ERR_INVALID_ARG;
  *out = nullptr;
  const uint32_t N = nodes->n_nodes, P = pods->n_pods;
  if (N && (!nodes->free_memory_sum || !nodes->total_memory_sum || !nodes->card_number))
    return YODA_ERR_INVALID_ARG;
  if (P && (!pods->has_memory || !pods->memory || !pods->has_number || !pods->number))
    return YODA_ERR_INVALID_ARG;
  if (N >= 0x7fffffffu) return YODA_ERR_RANGE;
  try {
    yoda_gs_t* g = new yoda_gs_t();
    g->N = N, g->P = P, g->flags = flags;
    g->free_sum.assign(nodes->free_memory_sum, nodes->free_memory_sum + N);
    g->total_sum.assign(nodes->total_memory_sum, nodes->total_memory_sum + N);
    g->card_number.assign(nodes->card_number, nodes->card_number + N);
    if (nodes->alloc_memory)
      g->alloc.assign(nodes->alloc_memory, nodes->alloc_memory + N);
    else
      g->alloc.assign(N, 0);
    g->alloc0 = g->alloc;
    g->cn0 = g->card_number;
    g->stat.resize(N);
    g->stat_w.resize(N);
    g->cn_w.resize(N);
    for (uint32_t n = 0; n < N; ++n) {
      bool z;
      g->stat[n] = static_score(g->free_sum[n], g->total_sum[n], g->alloc[n], &z);
    }
    g->touched_w.assign(N, 0);
    g->dirty.assign(N, 0);
    g->ever.assign(N, 0);
    g->has_memory.assign(pods->has_memory, pods->has_memory + P);
    g->memory.assign(pods->memory, pods->memory + P);
    g->has_number.assign(pods->has_number, pods->has_number + P);
    g->number.assign(pods->number, pods->number + P);
    if (pods->has_clock && pods->clock) {
      g->has_clock.assign(pods->has_clock, pods->has_clock + P);
      g->clock.assign(pods->clock, pods->clock + P);
    } else {
      g->has_clock.assign(P, 0);
      g->clock.assign(P, 0);
    }
    // capacity mode: keep the cards for the exact witness accounting (optional)
    if ((flags & YODA_GREEDY_CARD_CAPACITY) && N && nodes->max_cards >= 1 &&
        nodes->max_cards <= YODA_MAX_CARDS && nodes->card_count && nodes->card_free_memory &&
        nodes->card_total_memory && nodes->card_clock && nodes->card_bandwidth &&
        nodes->card_core && nodes->card_power && nodes->card_healthy) {
      const uint32_t K = nodes->max_cards;
      g->K = K;
      g->cards.assign((size_t)N * 6 * K, 0);
      g->hmask.assign(N, 0);
      g->rmask.assign(N, 0);
      const uint64_t* src[6] = {nodes->card_free_memory, nodes->card_clock,
                                nodes->card_total_memory, nodes->card_bandwidth,
                                nodes->card_core, nodes->card_power};  // CardField order
      for (uint32_t n = 0; n < N; ++n) {
        const uint32_t cnt = std::min<uint32_t>(nodes->card_count[n], K);
        for (uint32_t j = 0; j < cnt; ++j) {
          const size_t k = (size_t)n * K + j;
          for (int f = 0; f < 6; ++f) g->cards[((size_t)n * 6 + f) * K + j] = src[f][k];
          g->rmask[n] |= 1u << j;
          if (nodes->card_healthy[k]) g->hmask[n] |= 1u << j;
        }
      }
      // each node's largest contribution to any pod's maxima (contrib() over every real card)
      g->nodemax.assign((size_t)N * 6, 0);
      for (uint32_t n = 0; n < N; ++n) {
        uint64_t* v = g->nodemax.data() + (size_t)n * 6;
        const uint64_t* c = g->cards.data() + (size_t)n * 6 * K;
        for (uint32_t j = 0; j < K; ++j) {
          if (!((g->rmask[n] >> j) & 1u)) continue;
          v[0] = std::max(v[0], c[3 * K + j]);
          v[1] = std::max(v[1], c[1 * K + j]);
          v[2] = std::max(v[2], c[4 * K + j]);
          v[3] = std::max(v[3], c[0 * K + j]);
          v[4] = std::max(v[4], c[5 * K + j]);
          v[5] = std::max(v[5], c[2 * K + j]);
        }
      }
    }
    g->pick.assign(P, YODA_PICK_NONE);
    // queue order: sort.Less (sort.go:8-10), scv/priority descending, then input index
    queue_order(pods->priority, P, g->order);
    *out = g;
    return YODA_OK;
  } catch (...) {
    return YODA_ERR_INVALID_ARG;
  }
}

int yoda_gs_destroy(yoda_gs_t* g) {
  if (!g) return YODA_ERR_INVALID_ARG;
  delete g;
  return YODA_OK;
}

int yoda_gs_queue_order(const yoda_gs_t* g, uint32_t* order) {
  if (!g || (!order && g->P)) return YODA_ERR_INVALID_ARG;
  std::copy(g->order.begin(), g->order.end(), order);
  return YODA_OK;
}

namespace {
// yoda_gs_begin_window without copying the lists: the session reads (and, on a refresh,
// writes) top_score / top_node in place until the window ends (greedy_capacity's staging)
int gs_begin_window_at(yoda_gs_t* g, uint32_t ws, uint32_t wn, uint32_t k,
                       const uint32_t* counts, double* top_score, uint32_t* top_node,
                       bool borrow, bool row_major = false);
}  // namespace

int yoda_gs_begin_window(yoda_gs_t* g, uint32_t ws, uint32_t wn, uint32_t k,
                         const uint32_t* counts, const double* top_score,
                         const uint32_t* top_node) {
  return gs_begin_window_at(g, ws, wn, k, counts, const_cast<double*>(top_score),
                            const_cast<uint32_t*>(top_node), false, false);
}

namespace {
int gs_begin_window_at(yoda_gs_t* g, uint32_t ws, uint32_t wn, uint32_t k,
                       const uint32_t* counts, double* top_score, uint32_t* top_node,
                       bool borrow, bool row_major) {
  if (row_major && !borrow) return YODA_ERR_INVALID_ARG;
  if (!g || ws > g->P || wn > g->P - ws || k == 0 || !counts || !top_score || !top_node)
    return YODA_ERR_INVALID_ARG;
  if (!borrow)  // (the borrowed lists are libyoda's own kernel output)
    for (uint32_t i = 0; i < (uint32_t)k * wn; ++i)
      if (top_node[i] != 0xffffffffu && top_node[i] >= g->N) return YODA_ERR_RANGE;
  try {
    for (uint32_t n : g->touched_list) g->touched_w[n] = 0;
    g->touched_list.clear();
    g->ws = ws, g->wn = wn, g->k = k, g->next = 0;
    g->row_major = row_major;
    g->in_window = true;
    g->wrapped = false;
    g->stat_rose = false;
    std::fill(std::begin(g->cross), std::end(g->cross), 0u);
    for (auto& l : g->cross_list) l.clear();
    g->has_wit = false;
    g->counts.assign(counts, counts + 2 * (size_t)wn);
    if (borrow) {
      g->ts = top_score;
      g->ti = top_node;
    } else {
      g->ts_own.assign(top_score, top_score + (size_t)k * wn);
      g->ti_own.assign(top_node, top_node + (size_t)k * wn);
      g->ts = g->ts_own.data();
      g->ti = g->ti_own.data();
    }
    g->Tw.resize(wn);
    g->Tix.resize(wn);
    g->vlen.resize(wn);
    for (uint32_t i = 0; i < wn; ++i) {
      const uint32_t cap = std::min<uint32_t>(counts[i], k);
      uint32_t v = 0;
      while (v < cap && top_node[g->at(i, v)] != 0xffffffffu) ++v;
      g->vlen[i] = v;
      const uint32_t len = std::max<uint32_t>(1, v);  // (threshold: the last entry listed)
      g->Tw[i] = top_score[g->at(i, len - 1)];
      g->Tix[i] = top_node[g->at(i, len - 1)];
    }
    return YODA_OK;
  } catch (...) {
    return YODA_ERR_INVALID_ARG;
  }
}
}  // namespace

int yoda_gs_set_witness(yoda_gs_t* g, const uint64_t* maxima, const uint32_t* wit_count,
                        const uint32_t* wit_node) {
  if (!g || !g->in_window || (g->wn && (!maxima || !wit_count || !wit_node)))
    return YODA_ERR_INVALID_ARG;
  try {
    const size_t n = 6 * (size_t)g->wn;
    g->wmax.assign(maxima, maxima + n);
    g->wcnt.assign(wit_count, wit_count + n);
    g->wnode.assign(wit_node, wit_node + n);
    g->has_wit = true;
    return YODA_OK;
  } catch (...) {
    return YODA_ERR_INVALID_ARG;
  }
}

// Resolve the window in queue order until a pod cannot be certified from its candidate list
// (greedy): *next = its window index, or wn when the window is done.
int yoda_gs_resolve(yoda_gs_t* g, uint32_t* next) {
  if (!g || !next || !g->in_window) return YODA_ERR_INVALID_ARG;
  const uint32_t wn = g->wn;
  const bool capacity = (g->flags & YODA_GREEDY_CARD_CAPACITY) != 0;
  while (g->next < wn) {
    const uint32_t i = g->next;
    const uint32_t p = g->order[g->ws + i];
    const uint32_t nf = g->counts[i], nz = g->counts[(size_t)wn + i];
    int32_t pk;
    if (capacity) {
      if (!g->resolve_capacity(i, p, &pk)) break;
    } else if (nf == 0) {
      pk = YODA_PICK_NONE;
    } else if (nf >= 2 && nz > 0) {
      pk = YODA_PICK_ERROR;  // Score would divide by TotalMemorySum == 0
    } else if (nf == 1) {
      if (g->vlen[i] == 0) break;  // (not listed: the caller evaluates it)
      pk = (int32_t)g->ti[g->at(i, 0)];  // the only feasible node, returned without scoring
    } else if (g->wrapped) {
      break;
    } else {
      uint32_t bi;
      if (!g->certify0(i, &bi)) break;
      pk = (int32_t)bi;
    }
    g->pick[p] = pk;
    g->apply(p, pk);
    ++g->next;
    ++g->resolved;
  }
  *next = g->next;
  return YODA_OK;
}

uint32_t yoda_greedy_next_window(uint32_t progress, uint32_t wmax) {
  // the next window holds 130 % of this one's progress, in whole waves: small windows cost
  // less (K1 / K2 time grows with the pods) and most restart near where the last one did;
  // profiles/r03/greedy_capacity/grow_ab.txt (1.81-1.91 s with the earlier power of two >=
  // twice the progress, 1.57-1.64 s at 130 %).  YODA_GREEDY_GROW_PCT: A/B knob (0: that
  // power of two)
  static const uint32_t grow = YODA_KNOB("YODA_GREEDY_GROW_PCT", 130);
  wmax = std::max<uint32_t>(wmax, 1);
  uint32_t w2 = 64;
  if (grow) {
    const uint64_t t = (uint64_t)progress * grow / 100;
    w2 = (uint32_t)std::min<uint64_t>(wmax, std::max<uint64_t>(64, (t + 63) / 64 * 64));
  } else {
    while (w2 < 2 * progress && w2 < wmax) w2 <<= 1;
  }
  return std::min(w2, wmax);
}

int yoda_gs_uncertified(const yoda_gs_t* g, uint32_t from, uint32_t scan, uint32_t* count) {
  if (!g || !count || !g->in_window) return YODA_ERR_INVALID_ARG;
  if (g->flags & YODA_GREEDY_CARD_CAPACITY) return YODA_ERR_STATE;
  uint32_t c = 0, bi;
  // once Allocate has wrapped (alloc < before) no list certifies any more: a refresh cannot
  // help, so report none (the one rule of yoda_greedy, yoda_comm_greedy and dist.sharded_greedy)
  if (g->wrapped) {
    *count = 0;
    return YODA_OK;
  }
  const uint32_t end = (uint32_t)std::min<uint64_t>(g->wn, (uint64_t)from + scan);
  for (uint32_t i = from; i < end; ++i)
    if (g->counts[i] >= 2 && g->counts[(size_t)g->wn + i] == 0 && !g->certify0(i, &bi)) ++c;
  *count = c;
  return YODA_OK;
}

int yoda_gs_refresh(yoda_gs_t* g, uint32_t from, const double* top_score,
                    const uint32_t* top_node) {
  if (!g || !g->in_window || !top_score || !top_node || from > g->wn) return YODA_ERR_INVALID_ARG;
  // capacity sessions judge feasibility and maxima against the window start and restart
  // instead of refreshing (as yoda_gs_uncertified)
  if (g->flags & YODA_GREEDY_CARD_CAPACITY) return YODA_ERR_STATE;
  const uint32_t wn = g->wn, k = g->k;
  // validate every listed node first: a bad id leaves the session unchanged
  for (uint32_t i = from; i < wn; ++i) {
    const uint32_t len = std::min<uint32_t>(g->counts[i], k);
    for (uint32_t kk = 0; kk < len; ++kk)
      if (top_node[(size_t)kk * wn + i] >= g->N) return YODA_ERR_RANGE;
  }
  for (uint32_t i = from; i < wn; ++i) {
    const uint32_t len = std::min<uint32_t>(g->counts[i], k);
    for (uint32_t kk = 0; kk < len; ++kk) {
      const size_t o = (size_t)kk * wn + i;
      const uint32_t n = top_node[o];
      // stored so that the certificate's  stored - old static + current static  is its
      // current score (the refresh scored it with the current static)
      g->ti[g->at(i, kk)] = n;
      g->ts[g->at(i, kk)] = g->touched_w[n] ? top_score[o] + (double)g->stat_w[n] - (double)g->stat[n]
                                 : top_score[o];
    }
    g->vlen[i] = len;  // (a refresh's lists are whole: every id validated above)
    if (len) {
      g->Tw[i] = top_score[(size_t)(len - 1) * wn + i];
      g->Tix[i] = top_node[(size_t)(len - 1) * wn + i];
    }
  }
  ++g->refreshes;
  return YODA_OK;
}

int yoda_gs_assign(yoda_gs_t* g, uint32_t queue_pos, int32_t pick) {
  if (!g || queue_pos >= g->P) return YODA_ERR_INVALID_ARG;
  if (pick >= 0 && (uint32_t)pick >= g->N) return YODA_ERR_RANGE;
  const uint32_t p = g->order[queue_pos];
  g->pick[p] = pick;
  g->apply(p, pick);
  ++g->assigned;
  if (g->in_window && queue_pos == g->ws + g->next) ++g->next;
  return YODA_OK;
}

int yoda_gs_take_dirty(yoda_gs_t* g, uint32_t cap, uint32_t* nodes, uint64_t* alloc,
                       uint64_t* card_number, uint32_t* count) {
  if (!g || !count || (cap && (!nodes || !alloc || !card_number))) return YODA_ERR_INVALID_ARG;
  const uint32_t n = std::min<uint32_t>(cap, (uint32_t)g->dirty_list.size());
  for (uint32_t t = 0; t < n; ++t) {
    const uint32_t v = g->dirty_list[t];
    nodes[t] = v;
    alloc[t] = g->alloc[v];
    card_number[t] = g->card_number[v];
    g->dirty[v] = 0;
  }
  g->dirty_list.erase(g->dirty_list.begin(), g->dirty_list.begin() + n);
  *count = n;
  return YODA_OK;
}

int yoda_gs_touched_original(const yoda_gs_t* g, uint32_t cap, uint32_t* nodes, uint64_t* alloc,
                             uint64_t* card_number, uint32_t* count) {
  if (!g || !count || (cap && (!nodes || !alloc || !card_number))) return YODA_ERR_INVALID_ARG;
  const uint32_t n = std::min<uint32_t>(cap, (uint32_t)g->ever_list.size());
  for (uint32_t t = 0; t < n; ++t) {
    const uint32_t v = g->ever_list[t];
    nodes[t] = v;
    alloc[t] = g->alloc0[v];
    card_number[t] = g->cn0[v];
  }
  *count = n;
  return YODA_OK;
}

int yoda_gs_picks(const yoda_gs_t* g, int32_t* pick, uint32_t* resolved, uint32_t* assigned) {
  if (!g) return YODA_ERR_INVALID_ARG;
  if (pick) std::copy(g->pick.begin(), g->pick.end(), pick);
  if (resolved) *resolved = g->resolved;
  if (assigned) *assigned = g->assigned;
  return YODA_OK;
}

}  // extern "C"

// Pod p of `pods` scheduled exactly against the CURRENT device node state (k_one_*: Filter,
// CollectMaxValues, Score, then k8s' outcome rules as k_finalize applies them).  Local pick.
static int greedy_eval_exact(yoda_t* h, const yoda_pod_soa* pods, uint32_t p, int32_t* pick) {
  const uint32_t N = h->n_nodes;
  *pick = YODA_PICK_NONE;
  if (N == 0) return YODA_OK;
  OnePod op{};
  const uint64_t number = pods->has_number[p] ? pods->number[p] : 1;  // filter.go:12-15
  const uint32_t need = number > 0xffffffffull ? 0xffffffffu : (uint32_t)number;
  const uint64_t m = pods->has_memory[p] ? pods->memory[p] : 0;
  const uint64_t c = pods->has_clock[p] ? pods->clock[p] : 0;
  op.number = number;
  op.need_mem = pods->has_memory[p] ? need : 0;
  op.need_clk = pods->has_clock[p] ? need : 0;
  op.m32 = (uint32_t)std::min<uint64_t>(m, 0xffffffffull);
  if (h->mem_ranks)  // the rank threshold (yoda_layout.h MemTab)
    op.m32 = 2u + (uint32_t)(std::lower_bound(h->h_frees.begin(), h->h_frees.end(), m) -
                             h->h_frees.begin());
  op.c32 = (uint32_t)std::min<uint64_t>(c, 0xffffffffull);
  op.mf = (double)std::min<uint64_t>(m, 1ull << 53);
  op.cf = (double)std::min<uint64_t>(c, 1ull << 53);
  HIP_TRY(h, h->one_feas.ensure(((size_t)N + 63) / 64 * 8 + 64));
  HIP_TRY(h, h->one_part.ensure((size_t)one_blocks() * 9 * 8));
  HIP_TRY(h, h->one_out.ensure(sizeof(OneOut)));
  if (h->one_done.bytes == 0) {
    HIP_TRY(h, h->one_done.ensure(16));
    HIP_TRY(h, hipMemsetAsync(h->one_done.p, 0, 16, h->stream));
  }
  HIP_TRY(h, launch_one(h->K, h->path, h->nodes.as<unsigned char>(), N, op,
                        h->one_feas.as<uint64_t>(), h->one_part.p, h->one_done.as<uint32_t>(),
                        h->one_out.as<OneOut>(), pod_params(h).mt, h->stream));
  HIP_TRY(h, h->pick_stage.ensure(sizeof(OneOut)));
  HIP_TRY(h, hipMemcpyAsync(h->pick_stage.p, h->one_out.p, sizeof(OneOut), hipMemcpyDeviceToHost,
                            h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  OneOut o;
  std::memcpy(&o, h->pick_stage.p, sizeof(o));
  if (o.nf == 0)
    *pick = YODA_PICK_NONE;
  else if (o.nf == 1)  // k8s: the only feasible node is returned without scoring
    *pick = (int32_t)o.first;
  else if (o.nz > 0)   // Score would divide by TotalMemorySum == 0
    *pick = YODA_PICK_ERROR;
  else
    *pick = (int32_t)o.idx;
  return YODA_OK;
}

// ---- capacity-decrement greedy on one handle -------------------------------------------
// YODA_GREEDY_CARD_CAPACITY on a fast record path (greedy): windows of pods
// are evaluated on the device against the state at the window start (k1_witness + top-k
// K2), then the host session resolves them in queue order with the capacity certificate
// (yoda_greedy_session::resolve_capacity).  A pod it cannot certify starts the next window,
// so it is evaluated against the current state; the window size adapts to how far the last
// window got.  Node ids inside are local; picks are returned global.
static FILE* greedy_trace_file() {
  static FILE* f = [] {
    const char* p = std::getenv("YODA_GREEDY_TRACE");
    return p && *p ? std::fopen(p, "w") : nullptr;
  }();
  return f;
}

static int greedy_capacity(yoda_t* h, const yoda_pod_soa* pods, int32_t* pick) {
  using Clock = std::chrono::steady_clock;
  auto ms_since = [](Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
  };
  // the chunks' list depth: 8 where the lists are merged deeper (k_topk_merge_deep: the same
  // 64-deep lists as from 16, and a cheaper K2 -- 1.00-1.02 vs 1.07-1.09 s,
  // profiles/r05/pqr/tk_ab.txt), else 16; YODA_GREEDY_CAP_TOPK=16 (A/B knob): 16 always
  static const uint32_t kt_knob = YODA_KNOB("YODA_GREEDY_CAP_TOPK", 0);
  const uint32_t kt_cap = kt_knob == (uint32_t)topk_k_capacity() || !topk_block_ok(h)
                              ? (uint32_t)topk_k_capacity()
                              : (uint32_t)topk_k();
  const uint32_t P = pods->n_pods, N = h->n_nodes, KT = kt_cap;
  yoda_node_soa nv{};
  nv.n_nodes = N;
  nv.max_cards = 1;
  nv.card_number = h->h_card_number.data();
  nv.free_memory_sum = h->h_free_sum.data();
  nv.total_memory_sum = h->h_total_sum.data();
  nv.alloc_memory = h->h_alloc.data();
  // the cards, decoded from the host copy of the records, for the session's exact witness
  // accounting (CardField order: free, clock, total, bandwidth, core, power)
  const uint32_t K = (uint32_t)h->K;
  const size_t stride = h->path == Path::N32 ? n32_stride(h->K) : node_stride(h->K);
  std::vector<uint32_t> ccount(N);
  std::vector<uint64_t> fld[6];
  std::vector<uint8_t> healthy((size_t)N * K);
  for (auto& v : fld) v.resize((size_t)N * K);
  for (uint32_t n = 0; n < N; ++n) {
    const unsigned char* r = h->host_records.data() + (size_t)n * stride;
    const NodeHdrG* hd = reinterpret_cast<const NodeHdrG*>(r);
    ccount[n] = (uint32_t)__builtin_popcount(hd->real_mask);
    for (uint32_t j = 0; j < K; ++j) {
      healthy[(size_t)n * K + j] = (hd->healthy_mask >> j) & 1u;
      for (int f = 0; f < 6; ++f)
        fld[f][(size_t)n * K + j] =
            h->path == Path::N32
                ? reinterpret_cast<const uint32_t*>(r + n32_u32_off(f, h->K))[j]
                : (uint64_t) reinterpret_cast<const double*>(r + 32 + 8 * (size_t)f * K)[j];
      if (h->path == Path::N32) {  // memory values from the f64 groups (the u32 ones may be ranks)
        fld[kFree][(size_t)n * K + j] =
            (uint64_t) reinterpret_cast<const double*>(r + n32_f64_off(kF64Free, h->K))[j];
        fld[kTotal][(size_t)n * K + j] =
            (uint64_t) reinterpret_cast<const double*>(r + n32_f64_off(kF64Total, h->K))[j];
      }
    }
  }
  nv.max_cards = K;
  nv.card_count = ccount.data();
  nv.card_free_memory = fld[kFree].data();
  nv.card_clock = fld[kClock].data();
  nv.card_total_memory = fld[kTotal].data();
  nv.card_bandwidth = fld[kBandwidth].data();
  nv.card_core = fld[kCore].data();
  nv.card_power = fld[kPower].data();
  nv.card_healthy = healthy.data();
  yoda_gs_t* g = nullptr;
  int rc = yoda_gs_create(&nv, pods, YODA_GREEDY_CARD_CAPACITY, &g);
  if (rc) return fail(h, rc, "greedy: session setup failed");
  struct Guard {
    yoda_gs_t* g;
    ~Guard() { yoda_gs_destroy(g); }
  } guard{g};
  const uint32_t Wmax = greedy_window();
  uint32_t W = Wmax;
  std::vector<uint32_t> ids, cnt_w, ti_w, wc_w;
  std::vector<uint64_t> al, cn, mx_w;
  std::vector<double> ts_w;
  auto push = [&]() -> int {  // nodes the session changed -> the device
    const uint32_t d = (uint32_t)g->dirty_list.size();
    if (d == 0) return YODA_OK;
    ids.resize(d), al.resize(d), cn.resize(d);
    uint32_t got = 0;
    int r = yoda_gs_take_dirty(g, d, ids.data(), al.data(), cn.data(), &got);
    if (r) return fail(h, r, "greedy: take_dirty");
    for (uint32_t t = 0; t < got; ++t) ids[t] += h->node_offset;
    return yoda_set_node_state(h, got, ids.data(), al.data(), cn.data());
  };
  PodGather win;
  uint32_t ws = 0;
  while (ws < P) {
    const auto tw = Clock::now();
    if ((rc = push())) return rc;
    const uint32_t wn = std::min(W, P - ws);
    win.build(pods, g->order.data() + ws, wn);
    if ((rc = yoda_upload_pods(h, &win.soa))) return rc;
    const double t_up = ms_since(tw);
    if ((rc = prepare_run(h, YODA_MODE_SCV))) return rc;
    if ((rc = order_pods(h, YODA_MODE_SCV))) return rc;
    HIP_TRY(h, h->wit.ensure(12 * (size_t)wn * 4));
    if ((rc = phase1_witness(h, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(),
                             h->wit.as<uint32_t>(), 0)))
      return rc;
    // the lists' depth: KT from the chunks, merged deeper where the block kernels run
    // (k_topk_merge_deep: exact as far as they reach; YODA_GREEDY_CAP_DEPTH, A/B knob: 32 /
    // 64 / 128, 0 = KT).  128 with the exact-fallback scan below (windows 1558 -> 822,
    // capacity 0.97 -> 0.89-0.90 s; 128 alone 0.98 s, the scan alone 0.92-0.93 s;
    // profiles/r06/greedy_scan/)
    static const uint32_t cap_depth = YODA_KNOB("YODA_GREEDY_CAP_DEPTH", 128);
    uint32_t KD = KT;
    // pinned staging of the window's outputs, in window order (k_window_out writes them there
    // from the sorted order in one launch): counts | maxima | wit | top scores | top nodes
    size_t o_cnt = 0, o_mx = 0, o_wit = 0, o_ts = 0, o_ti = 0, total = 0;
    auto layout = [&](uint32_t kd) {
      o_cnt = 0, o_mx = o_cnt + 8 * (size_t)wn, o_wit = o_mx + 48 * (size_t)wn,
      o_ts = o_wit + 48 * (size_t)wn, o_ti = o_ts + 8 * (size_t)kd * wn,
      total = o_ti + 4 * (size_t)kd * wn;
    };
    layout(std::max(KT, cap_depth));
    HIP_TRY(h, h->win_stage.ensure(total));
    unsigned char* st = static_cast<unsigned char*>(h->win_stage.p);
    const uint32_t *cnt_p, *wc_p, *ti_p;
    const uint64_t* mx_p;
    const double* ts_p;
    double t_issued, t_sync;
    if (N > 0) {
      HIP_TRY(h, launch_prep2(h->maxima.as<uint64_t>(), wn, h->rcp.as<double>(),
                               h->stream));
      // (node ids local here: the session works on this handle's nodes)
      const uint32_t off = h->node_offset;
      h->node_offset = 0;
      rc = topk_lists(h, wn, KT, h->counts.as<uint32_t>(), cap_depth, &KD);
      h->node_offset = off;
      if (rc) return rc;
      layout(KD);
      // (YODA_WIN_DMA=0, A/B knob: k_window_out writes the pinned pages directly)
      static const bool win_dma = YODA_KNOB("YODA_WIN_DMA", 1) != 0;
      if (win_dma) HIP_TRY(h, h->win_dev.ensure(total));
      HIP_TRY(h, h->win_inv.ensure((size_t)wn * 4));
      HIP_TRY(h, launch_window_out(h->counts.as<uint32_t>(), h->maxima.as<uint64_t>(),
                                   h->wit.as<uint32_t>(), h->tk_s.as<double>(),
                                   h->tk_i.as<uint32_t>(),
                                   h->ordered ? h->perm.as<uint32_t>() : nullptr, wn, KD, true,
                                   win_dma ? h->win_dev.as<unsigned char>()
                                           : static_cast<unsigned char*>(h->win_stage.dp),
                                   h->win_inv.as<uint32_t>(), h->stream));
      if (win_dma)
        HIP_TRY(h, hipMemcpyAsync(h->win_stage.p, h->win_dev.p, total, hipMemcpyDeviceToHost,
                                  h->stream));
      t_issued = ms_since(tw);
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      t_sync = ms_since(tw);
      cnt_p = reinterpret_cast<const uint32_t*>(st + o_cnt);
      mx_p = reinterpret_cast<const uint64_t*>(st + o_mx);
      wc_p = reinterpret_cast<const uint32_t*>(st + o_wit);
      ts_p = reinterpret_cast<const double*>(st + o_ts);
      ti_p = reinterpret_cast<const uint32_t*>(st + o_ti);
    } else {  // no nodes: every pod infeasible
      t_issued = ms_since(tw);
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      t_sync = ms_since(tw);
      cnt_w.assign(2 * (size_t)wn, 0u);
      mx_w.assign(6 * (size_t)wn, 1ull);
      wc_w.assign(12 * (size_t)wn, 0u);
      for (size_t t = 6 * (size_t)wn; t < 12 * (size_t)wn; ++t) wc_w[t] = 0xffffffffu;
      ts_w.assign((size_t)KD * wn, -1.0);
      ti_w.assign((size_t)KD * wn, 0xffffffffu);
      cnt_p = cnt_w.data(), mx_p = mx_w.data(), wc_p = wc_w.data();
      ts_p = ts_w.data(), ti_p = ti_w.data();
    }
    ++h->greedy_windows;
    const double t_win = ms_since(tw);
    h->greedy_window_ms += t_win;
    const auto tr = Clock::now();
    if ((rc = gs_begin_window_at(g, ws, wn, KD, cnt_p, const_cast<double*>(ts_p),
                                 const_cast<uint32_t*>(ti_p), true, N > 0)) ||
        (rc = yoda_gs_set_witness(g, mx_p, wc_p, wc_p + 6 * (size_t)wn)))
      return fail(h, rc, "greedy: session window");
    // resolve; an uncertified pod is scheduled exactly against the current state (k_one_*)
    // while such pods stay rare in the window, else it opens the next window
    uint32_t next = 0, fails = 0;
    double fb_ms = 0;
    uint64_t why0[6];
    std::copy(std::begin(g->why), std::end(g->why), why0);
    for (;;) {
      if ((rc = yoda_gs_resolve(g, &next))) return fail(h, rc, "greedy: resolve");
      // YODA_GREEDY_FAIL_DIV (A/B knob): one exact evaluation allowed per that many resolved pods
      static const uint32_t rate = YODA_KNOB("YODA_GREEDY_FAIL_DIV", 0);
      // fall back exactly (instead of restarting the window) when at most
      // YODA_GREEDY_CAP_SCAN_MAX of the next YODA_GREEDY_CAP_SCAN window pods are uncertified
      // already (A/B knobs; 64 / 1: a restart re-runs the window's kernels for one pod whose
      // witness was lost while its successors still hold theirs; 32 / 128 / 256: 0.97 / 0.92 /
      // 0.91 s, 0: 0.97 s)
      static const uint32_t scan_n = YODA_KNOB("YODA_GREEDY_CAP_SCAN", 64);
      static const uint32_t scan_max = YODA_KNOB("YODA_GREEDY_CAP_SCAN_MAX", 1);
      if (next >= wn) break;
      bool fallback = false;
      if (rate) {
        fallback = ++fails <= next / rate;
      } else if (scan_n && wn - next > scan_n) {
        uint64_t saved[6];
        std::copy(std::begin(g->why), std::end(g->why), saved);
        uint32_t unc = 0;
        int32_t dummy;
        for (uint32_t j = next + 1; j <= next + scan_n && unc <= scan_max; ++j)
          unc += g->resolve_capacity(j, g->order[ws + j], &dummy) ? 0u : 1u;
        std::copy(std::begin(saved), std::end(saved), std::begin(g->why));
        fallback = unc <= scan_max;
      }
      if (!fallback) break;
      const auto tf = Clock::now();
      if ((rc = push())) return rc;
      int32_t pk = YODA_PICK_NONE;
      if ((rc = greedy_eval_exact(h, pods, g->order[ws + next], &pk))) return rc;
      if ((rc = yoda_gs_assign(g, ws + next, pk))) return fail(h, rc, "greedy: assign");
      ++h->greedy_fallbacks;
      fb_ms += ms_since(tf);
    }
    h->greedy_fallback_ms += fb_ms;
    h->greedy_resolve_ms += ms_since(tr) - fb_ms;
    // YODA_GREEDY_TRACE=<file> (diagnostic): one line per window -- start, size, pods
    // resolved, the failed certificate (index into why[], -1 = none), pods assigned so far
    if (FILE* tf = greedy_trace_file()) {
      int reason = -1;
      for (int r = 0; r < 6; ++r)
        if (g->why[r] != why0[r]) reason = r;
      uint32_t placed = 0;
      for (uint32_t t = 0; t < next; ++t) placed += g->pick[g->order[ws + t]] >= 0 ? 1u : 0u;
      uint64_t q = 0, nf0 = 0, lq = 0;
      if (next < wn) {
        q = g->need_cards(g->order[ws + next]);
        nf0 = g->counts[next];
        lq = g->lost(q);
      }
      std::fprintf(tf, "%u %u %u %d %u %llu %llu %llu %.1f %.1f %.1f %.1f %.1f\n", ws, wn, next,
                   reason, placed, (unsigned long long)q, (unsigned long long)nf0,
                   (unsigned long long)lq, 1e3 * ms_since(tw), 1e3 * t_up, 1e3 * t_issued,
                   1e3 * t_sync, 1e3 * t_win);
      std::fflush(tf);
    }
    if (next < wn) {
      // pod ws + next could not be certified: it opens the next window (evaluated against the
      // current state, so it is always resolved there); size it after this one's progress
      ++h->greedy_restarts;
      // the next window holds 130 % of this one's progress, in whole waves: small windows cost
      // less (K1 / K2 time grows with the pods) and most restart near where the last one did;
      // profiles/r03/greedy_capacity/grow_ab.txt (1.81-1.91 s with the earlier power of two >=
      // twice the progress, 1.57-1.64 s at 130 %).  YODA_GREEDY_GROW_PCT: A/B knob (0: that
      // power of two)
      W = yoda_greedy_next_window(next, Wmax);
      ws += next;
    } else {
      ws += wn;
      W = std::min(2 * W, Wmax);
    }
  }
  if ((rc = yoda_gs_picks(g, pick, nullptr, nullptr))) return fail(h, rc, "greedy: picks");
  if (std::getenv("YODA_GREEDY_DEBUG"))
    std::fprintf(stderr,
                 "greedy capacity: windows %u restarts %u; failed certificates: wrap %llu, "
                 "few-left %llu, zero-total %llu, maxima %llu, list-lost %llu, threshold %llu; "
                 "resolves %llu, lost-node scans %llu visiting %llu nodes\n",
                 h->greedy_windows, h->greedy_restarts, (unsigned long long)g->why[0],
                 (unsigned long long)g->why[1], (unsigned long long)g->why[2],
                 (unsigned long long)g->why[3], (unsigned long long)g->why[4],
                 (unsigned long long)g->why[5], (unsigned long long)g->n_resolve,
                 (unsigned long long)g->n_scan, (unsigned long long)g->n_scan_nodes);
  for (uint32_t p = 0; p < P; ++p)
    if (pick[p] >= 0) pick[p] += (int32_t)h->node_offset;
  // leave the uploaded snapshot as it was
  const uint32_t ne = (uint32_t)g->ever_list.size();
  ids.resize(ne), al.resize(ne), cn.resize(ne);
  uint32_t got = 0;
  if ((rc = yoda_gs_touched_original(g, ne, ids.data(), al.data(), cn.data(), &got)))
    return fail(h, rc, "greedy: restore");
  for (uint32_t t = 0; t < got; ++t) ids[t] += h->node_offset;
  if ((rc = yoda_set_node_state(h, got, ids.data(), al.data(), cn.data()))) return rc;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  h->ran = false;
  return YODA_OK;
}

// ---- multi-GPU step inside libyoda (RCCL, no torch) ---------------------------------------
// One node shard per handle; a step is the sharded evaluation of yoda_shard_* with the
// exchanges done here:
//   1. one group of two all-reduces: MAX (u64) over [maxima 6P | score bits, node-id bits]
//      -- CollectMaxValues is a reduction over all nodes; the two trailing words make every
//      shard take the same phase-2 form -- and SUM (u32) over the feasible / zero-total
//      counts [2P];
//   2. fast record paths (and Mode B): the packed-key merge -- each shard's (best score,
//      lowest node reaching it) as one u64 key, all-reduce(MAX) [P], then the winners' tie
//      counts all-reduce(SUM) [P] (k_pack_key / k_unpack_key); the U64 path in Mode A, whose
//      normalize check needs the lowest score too, all-gathers each shard's ShardRec [P]
//      (best, lowest index reaching it, ties, lowest) and folds them (k_merge_rec).
// `hs` are the shards this process drives: one handle with an RCCL communicator
// (yoda_comm_run), or every shard of the batch on one device with device copies as the
// transport (yoda_comm_run_local, for tests and single-process use).
static uint32_t bit_length(uint64_t v) {
  uint32_t b = 0;
  while (b < 64 && (v >> b)) ++b;
  return b;
}

// The words every shard contributes to exchange 1 (MAX-reduced with the maxima):
//   [0] score bits and [1] node-id bits this shard needs (the phase-2 form: packed key or
//       records);
//   [2] the shard's largest small card field (bandwidth / clock / core / power) and [3] 1 when
//       the shard's block K2 computes its small-field quotients in f32 (N32 path, every small
//       field <= kF32SmallMax).  The exchanged maxima are the GLOBAL ones, so an
//       f32 shard is exact only while the global small-field max is <= kF32SmallMax too;
//       otherwise the shards must re-upload with YODA_UPLOAD_F64_QUOTIENTS (dist.agree_on_path
//       does) -- quotient_disagreement names that instead of returning inexact scores.
constexpr int kAgreeWords = 4;
constexpr size_t kAgreeBytes = 8 * kAgreeWords;

static void agreement_words(const yoda_t* h, int mode, uint64_t* w) {
  w[0] = h->generic && mode == YODA_MODE_SCV ? 64u : bit_length(h->score_bound);
  w[1] = bit_length((uint64_t)h->node_offset + h->n_nodes + 1);
  const bool f32q = mode == YODA_MODE_SCV && h->path == Path::N32 && h->q32;
  w[2] = mode == YODA_MODE_SCV ? h->small_max : 0;
  w[3] = f32q ? 1 : 0;
}

static const char* quotient_disagreement(uint64_t global_small_max, uint64_t any_f32) {
  if (any_f32 && global_small_max > kF32SmallMax)
    return "shards disagree on the quotient type: a shard computes f32 small-field quotients "
           "but another shard holds a small card field beyond 55738, so the reduced maxima "
           "break the f32 lemma; upload every shard with YODA_UPLOAD_F64_QUOTIENTS (see "
           "yoda_small_field_max)";
  return nullptr;
}

static int comm_step(yoda_t* const* hs, int n, int world, int mode, bool local) {
  yoda_t* h0 = hs[0];
  const uint32_t P = h0->n_pods;
  const size_t n1 = 6 * (size_t)P + kAgreeWords;  // maxima | agreement words
  for (int i = 0; i < n; ++i) {
    yoda_t* h = hs[i];
    if (h->n_pods != P) return fail(h0, YODA_ERR_INVALID_ARG, "shards hold different batches");
    // the fast record paths exchange in the caller's pod order, so each shard runs its private
    // order (padded counting sort, block-grouped nodes: xfer); the U64 path, whose exact-
    // normalize records go per sorted position, keeps the radix order all shards share
    h->xo = !h->generic;
    int rc = prepare_run(h, mode, h->xo);
    if (rc) return rc;
    if ((rc = order_pods(h, mode))) return rc;
    HIP_TRY(h, h->ex1.ensure(n1 * 8));
    HIP_TRY(h, h->rec.ensure((size_t)std::max<uint32_t>(P, 1) * sizeof(ShardRec)));
    HIP_TRY(h, h->rec_all.ensure((size_t)world * std::max<uint32_t>(P, 1) * sizeof(ShardRec)));
    if ((rc = xo_ensure(h))) return rc;
    if (P == 0) continue;
    uint64_t* ex = h->ex1.as<uint64_t>();
    if (h->xo) {
      if ((rc = phase1(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>()))) return rc;
      if ((rc = xfer(h, true, {{h->maxima.p, ex, 6, 8}, {h->counts.p, h->xcnt.p, 2, 4}})))
        return rc;
    } else if ((rc = phase1(h, mode, ex, h->counts.as<uint32_t>()))) {
      return rc;
    }
    // agreement words (pinned staging, one slot per shard; the previous step's copies
    // finished before its read-back below)
    uint64_t agree[kAgreeWords];
    agreement_words(h, mode, agree);
    HIP_TRY(h0, h0->win_stage.ensure(kAgreeBytes * ((size_t)n + 1)));
    unsigned char* slot =
        static_cast<unsigned char*>(h0->win_stage.p) + kAgreeBytes * ((size_t)i + 1);
    std::memcpy(slot, agree, kAgreeBytes);
    HIP_TRY(h, hipMemcpyAsync(ex + 6 * (size_t)P, slot, kAgreeBytes, hipMemcpyHostToDevice,
                              h->stream));
  }
  if (P == 0) {
    for (int i = 0; i < n; ++i) hs[i]->ran = true;
    return YODA_OK;
  }
  // the caller-order views of the exchanged buffers (the handle's own ones on the U64 path)
  auto cnt_x = [](yoda_t* h) { return h->xo ? h->xcnt.as<uint32_t>() : h->counts.as<uint32_t>(); };
  auto best_x = [](yoda_t* h) { return h->xo ? h->xbest.as<int64_t>() : h->best.as<int64_t>(); };
  auto idx_x = [](yoda_t* h) { return h->xo ? h->xidx.as<uint32_t>() : h->idx.as<uint32_t>(); };
  auto ties_x = [](yoda_t* h) { return h->xo ? h->xties.as<uint32_t>() : h->ties.as<uint32_t>(); };
  auto low_x = [](yoda_t* h) { return h->xo ? h->xlow.as<int64_t>() : h->lowest.as<int64_t>(); };
  if (local) {  // exchange 1: elementwise MAX / SUM over the shards, back to each
    PtrList l{}, c{};
    for (int i = 0; i < n; ++i) {
      l.p[i] = hs[i]->ex1.p;
      c.p[i] = cnt_x(hs[i]);
    }
    HIP_TRY(h0, h0->rec.ensure(std::max<size_t>(2 * (size_t)P * 4, (size_t)P * sizeof(ShardRec))));
    HIP_TRY(h0, launch_max_multi(l, (uint32_t)n, n1, h0->ex1.as<uint64_t>(), h0->stream));
    HIP_TRY(h0, launch_sum_multi_u32(c, (uint32_t)n, 2 * (uint64_t)P, h0->rec.as<uint32_t>(),
                                     h0->stream));
    for (int i = 0; i < n; ++i) {
      if (i > 0)
        HIP_TRY(h0, hipMemcpyAsync(hs[i]->ex1.p, h0->ex1.p, n1 * 8, hipMemcpyDeviceToDevice,
                                   h0->stream));
      HIP_TRY(h0, hipMemcpyAsync(cnt_x(hs[i]), h0->rec.p, 2 * (size_t)P * 4,
                                 hipMemcpyDeviceToDevice, h0->stream));
    }
  } else {
    rccl().group_start();
    ncclResult_t r = rccl().all_reduce(h0->ex1.p, h0->ex1.p, n1, ncclUint64, ncclMax, h0->comm,
                                       h0->stream);
    const ncclResult_t r2 = rccl().all_reduce(cnt_x(h0), cnt_x(h0), 2 * (size_t)P,
                                              ncclUint32, ncclSum, h0->comm, h0->stream);
    const ncclResult_t r3 = rccl().group_end();
    if (r == ncclSuccess) r = r2;
    if (r == ncclSuccess) r = r3;
    if (r != ncclSuccess)
      return fail(h0, YODA_ERR_HIP, std::string("ncclAllReduce: ") + rccl().error_string(r));
  }
  // the agreed phase-2 form (every shard reads the same reduced words; one host wait per step)
  uint64_t agreed[kAgreeWords] = {64, 64, 0, 0};
  HIP_TRY(h0, hipMemcpyAsync(h0->win_stage.p, h0->ex1.as<uint64_t>() + 6 * (size_t)P,
                             kAgreeBytes, hipMemcpyDeviceToHost, h0->stream));
  HIP_TRY(h0, hipStreamSynchronize(h0->stream));
  std::memcpy(agreed, h0->win_stage.p, kAgreeBytes);
  // every rank reads the same reduced words, so every rank fails here together
  if (const char* why = quotient_disagreement(agreed[2], agreed[3]))
    return fail(h0, YODA_ERR_STATE, why);
  const uint32_t ib = (uint32_t)std::max<uint64_t>(1, agreed[1]);
  const bool packed = agreed[0] + ib <= 63 && ib <= 40;
  for (int i = 0; i < n; ++i) {
    yoda_t* h = hs[i];
    uint64_t* ex = h->ex1.as<uint64_t>();
    int rc;
    if (h->xo) {
      if ((rc = xfer(h, false, {{h->maxima.p, ex, 6, 8}, {h->counts.p, h->xcnt.p, 2, 4}})))
        return rc;
    } else {
      HIP_TRY(h, hipMemcpyAsync(h->maxima.p, ex, 6 * (size_t)P * 8, hipMemcpyDeviceToDevice,
                                h->stream));
    }
    rc = phase2(h, mode, h->maxima.as<uint64_t>(), h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>());
    if (rc) return rc;
    if (h->xo && (rc = xfer(h, true, {{h->best.p, h->xbest.p, 1, 8}, {h->idx.p, h->xidx.p, 1, 4},
                                      {h->ties.p, h->xties.p, 1, 4},
                                      {h->lowest.p, h->xlow.p, 1, 8}})))
      return rc;
    if (packed)
      HIP_TRY(h, launch_pack_key(best_x(h), idx_x(h), P, ib, h->rec.as<uint64_t>(), h->stream));
    else
      HIP_TRY(h, launch_pack_rec(best_x(h), idx_x(h), ties_x(h), low_x(h), P,
                                 h->rec.as<ShardRec>(), h->stream));
  }
  if (packed) {  // exchange 2: MAX of the keys, then SUM of the winners' ties
    if (local) {
      PtrList l{};
      for (int i = 0; i < n; ++i) l.p[i] = hs[i]->rec.p;
      HIP_TRY(h0, launch_max_multi(l, (uint32_t)n, P, h0->rec_all.as<uint64_t>(), h0->stream));
      for (int i = 0; i < n; ++i)
        HIP_TRY(h0, hipMemcpyAsync(hs[i]->rec.p, h0->rec_all.p, (size_t)P * 8,
                                   hipMemcpyDeviceToDevice, h0->stream));
    } else {
      const ncclResult_t r = rccl().all_reduce(h0->rec.p, h0->rec.p, P, ncclUint64, ncclMax,
                                               h0->comm, h0->stream);
      if (r != ncclSuccess)
        return fail(h0, YODA_ERR_HIP, std::string("ncclAllReduce: ") + rccl().error_string(r));
    }
    for (int i = 0; i < n; ++i) {
      yoda_t* h = hs[i];
      HIP_TRY(h, launch_unpack_key(h->rec.as<uint64_t>(), P, ib, best_x(h), idx_x(h), ties_x(h),
                                   low_x(h), h->stream));
    }
    if (local) {
      PtrList t{};
      for (int i = 0; i < n; ++i) t.p[i] = ties_x(hs[i]);
      HIP_TRY(h0, launch_sum_multi_u32(t, (uint32_t)n, P, h0->rec_all.as<uint32_t>(), h0->stream));
      for (int i = 0; i < n; ++i)
        HIP_TRY(h0, hipMemcpyAsync(ties_x(hs[i]), h0->rec_all.p, (size_t)P * 4,
                                   hipMemcpyDeviceToDevice, h0->stream));
    } else {
      const ncclResult_t r = rccl().all_reduce(ties_x(h0), ties_x(h0), P, ncclUint32, ncclSum,
                                               h0->comm, h0->stream);
      if (r != ncclSuccess)
        return fail(h0, YODA_ERR_HIP, std::string("ncclAllReduce: ") + rccl().error_string(r));
    }
  } else {
    const size_t rb = (size_t)P * sizeof(ShardRec);
    if (local) {  // exchange 2: every shard's records to every shard
      for (int r = 0; r < n; ++r)
        for (int i = 0; i < n; ++i)
          HIP_TRY(h0, hipMemcpyAsync(hs[i]->rec_all.as<unsigned char>() + r * rb, hs[r]->rec.p,
                                     rb, hipMemcpyDeviceToDevice, h0->stream));
    } else {
      const ncclResult_t r = rccl().all_gather(h0->rec.p, h0->rec_all.p, rb / 8, ncclUint64,
                                               h0->comm, h0->stream);
      if (r != ncclSuccess)
        return fail(h0, YODA_ERR_HIP, std::string("ncclAllGather: ") + rccl().error_string(r));
    }
    for (int i = 0; i < n; ++i) {
      yoda_t* h = hs[i];
      HIP_TRY(h, launch_merge_rec(h->rec_all.as<ShardRec>(), P, (uint32_t)world, best_x(h),
                                  idx_x(h), ties_x(h), low_x(h), h->stream));
    }
  }
  for (int i = 0; i < n; ++i) {
    yoda_t* h = hs[i];
    int rc;
    if (h->xo && (rc = xfer(h, false, {{h->best.p, h->xbest.p, 1, 8}, {h->idx.p, h->xidx.p, 1, 4},
                                       {h->ties.p, h->xties.p, 1, 4},
                                       {h->lowest.p, h->xlow.p, 1, 8}})))
      return rc;
    rc = finalize(h, mode, h->counts.as<uint32_t>(), h->best.as<int64_t>(),
                  h->idx.as<uint32_t>(), h->ties.as<uint32_t>(), h->lowest.as<int64_t>(), true);
    if (rc) return rc;
    h->ran = true;
    h->ran_bitmask = false;
    h->last_mode = mode;
  }
  // exchange 3 (rare: U64 pods whose NormalizeScore can overflow int64, scheduler.go:176-179):
  // every shard's exact-normalize records to every shard, then the merge (all shards flag the
  // same pods, so all of them take this branch)
  if (h0->k3_pending) {
    const size_t rb = (size_t)h0->n_work * sizeof(ShardRec);
    for (int i = 0; i < n; ++i) HIP_TRY(hs[i], hs[i]->k3all.ensure(rb * (size_t)world));
    if (local) {
      for (int r = 0; r < n; ++r)
        for (int i = 0; i < n; ++i)
          HIP_TRY(h0, hipMemcpyAsync(hs[i]->k3all.as<unsigned char>() + r * rb, hs[r]->k3rec.p,
                                     rb, hipMemcpyDeviceToDevice, h0->stream));
    } else {
      const ncclResult_t r = rccl().all_gather(h0->k3rec.p, h0->k3all.p, rb / 8, ncclUint64,
                                               h0->comm, h0->stream);
      if (r != ncclSuccess)
        return fail(h0, YODA_ERR_HIP, std::string("ncclAllGather: ") + rccl().error_string(r));
    }
    for (int i = 0; i < n; ++i) {
      int rc = yoda_shard_exact_merge(hs[i], hs[i]->k3all.p, world);
      if (rc) return rc;
    }
  }
  return YODA_OK;
}

// Collectives of the libyoda-driven multi-GPU paths: over RCCL (one handle per process, the
// handle's communicator) or, for tests on one device, over the `n` handles of this process
// (host-staged: every handle's buffer read back, reduced or concatenated, written back).
struct Coll {
  yoda_t* const* hs;
  int n, world;
  bool local;
  uint32_t* calls = nullptr;  // collective launches made (yoda_comm_greedy_stats): a group of
                              // collectives (begin() .. end()) counts once
  bool in_group = false;
  int nccl(ncclResult_t r, const char* what) const {
    if (r == ncclSuccess) return YODA_OK;
    return fail(hs[0], YODA_ERR_HIP, std::string(what) + ": " + rccl().error_string(r));
  }
  void count() const {
    if (calls && !in_group) ++*calls;
  }
  // ncclGroupStart / End: the collectives issued in between run as ONE launch (RCCL fuses
  // them); the local transport runs each at once
  void begin() {
    if (!local) rccl().group_start();
    in_group = true;
  }
  int end() {
    in_group = false;
    count();
    return local ? YODA_OK : nccl(rccl().group_end(), "ncclGroupEnd");
  }
  // in-place elementwise all-reduce of `count` u64 or u32 device words (MAX / SUM / MIN)
  int allreduce(const std::vector<void*>& bufs, size_t count, bool u64, ncclRedOp_t op) const {
    if (count == 0) return YODA_OK;
    this->count();
    if (!local)
      return nccl(rccl().all_reduce(bufs[0], bufs[0], count, u64 ? ncclUint64 : ncclUint32, op,
                                    hs[0]->comm, hs[0]->stream),
                  "ncclAllReduce");
    const size_t w = u64 ? 8 : 4;
    std::vector<unsigned char> acc(count * w), one(count * w);
    for (int i = 0; i < n; ++i) {
      HIP_TRY(hs[i], hipMemcpyAsync(i ? one.data() : acc.data(), bufs[i], count * w,
                                    hipMemcpyDeviceToHost, hs[i]->stream));
      HIP_TRY(hs[i], hipStreamSynchronize(hs[i]->stream));
      if (i == 0) continue;
      for (size_t e = 0; e < count; ++e) {
        if (u64) {
          uint64_t& a = reinterpret_cast<uint64_t*>(acc.data())[e];
          const uint64_t b = reinterpret_cast<const uint64_t*>(one.data())[e];
          a = op == ncclMax ? std::max(a, b) : op == ncclMin ? std::min(a, b) : a + b;
        } else {
          uint32_t& a = reinterpret_cast<uint32_t*>(acc.data())[e];
          const uint32_t b = reinterpret_cast<const uint32_t*>(one.data())[e];
          a = op == ncclMax ? std::max(a, b) : op == ncclMin ? std::min(a, b) : a + b;
        }
      }
    }
    for (int i = 0; i < n; ++i) {
      HIP_TRY(hs[i], hipMemcpyAsync(bufs[i], acc.data(), count * w, hipMemcpyHostToDevice,
                                    hs[i]->stream));
      HIP_TRY(hs[i], hipStreamSynchronize(hs[i]->stream));
    }
    return YODA_OK;
  }
  // all-gather of host blocks: out = the world's `bytes`-byte blocks in rank order (RCCL:
  // staged through the first handle's device scratch).  In a group: allgather_issue before
  // end(), allgather_finish after it (the copies back must follow the collective's launch).
  int allgather(const std::vector<const void*>& in, size_t bytes,
                std::vector<unsigned char>& out) const {
    int rc = allgather_issue(in, bytes, out);
    return rc ? rc : allgather_finish(bytes, out);
  }
  int allgather_issue(const std::vector<const void*>& in, size_t bytes,
                      std::vector<unsigned char>& out) const {
    out.resize((size_t)world * bytes);
    count();
    if (local) {
      for (int i = 0; i < n; ++i) std::memcpy(out.data() + (size_t)i * bytes, in[i], bytes);
      return YODA_OK;
    }
    yoda_t* h = hs[0];
    const size_t b8 = (bytes + 7) / 8 * 8;
    HIP_TRY(h, h->cg_gather.ensure(b8 * ((size_t)world + 1)));
    unsigned char* d = h->cg_gather.as<unsigned char>();
    HIP_TRY(h, hipMemcpyAsync(d, in[0], bytes, hipMemcpyHostToDevice, h->stream));
    return nccl(rccl().all_gather(d, d + b8, b8 / 8, ncclUint64, h->comm, h->stream),
                "ncclAllGather");
  }
  int allgather_finish(size_t bytes, std::vector<unsigned char>& out) const {
    if (local) return YODA_OK;
    yoda_t* h = hs[0];
    const size_t b8 = (bytes + 7) / 8 * 8;
    unsigned char* d = h->cg_gather.as<unsigned char>();
    for (int r = 0; r < world; ++r)
      HIP_TRY(h, hipMemcpyAsync(out.data() + (size_t)r * bytes, d + b8 * ((size_t)r + 1), bytes,
                                hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    return YODA_OK;
  }
};

static int comm_step(yoda_t* const* hs, int n, int world, int mode, bool local);

// The sharded greedy's list merge (window exchange 2), shared by comm_greedy and the caller-
// driven protocol (yoda_merge_shard_lists, dist.sharded_greedy): shard rk's list of window pod
// p is (sc[rk][l*wn + p], nd[rk][l*wn + p]), l < kl, sorted score desc / node asc and ended by
// a 0xFFFFFFFF node.  ts/ti [kl][wn] receive the first kl of the union in that order (pods
// [from, wn) only).  Deep lists (exact down to their last entry only): every node a shard left
// out scores at most the shard's last entry, so the union is certain only above the latest of
// those -- and for its first topk_k(), which lie within their shards' exact prefixes.
static void merge_shard_lists(int world, uint32_t wn, uint32_t kl, bool deep, uint32_t from,
                              const double* const* sc, const uint32_t* const* nd, double* ts,
                              uint32_t* ti) {
  auto before = [](const std::pair<double, uint32_t>& a, const std::pair<double, uint32_t>& b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  };
  std::vector<uint32_t> head(world), len(world);
  for (uint32_t p = from; p < wn; ++p) {
    bool any_last = false;
    std::pair<double, uint32_t> last_max{-1.0, 0xffffffffu};
    for (int rk = 0; rk < world; ++rk) {
      uint32_t l = 0;
      while (l < kl && nd[rk][(size_t)l * wn + p] != 0xffffffffu) ++l;
      len[rk] = l;
      head[rk] = 0;
      if (deep && l > 0) {
        const std::pair<double, uint32_t> last{sc[rk][(size_t)(l - 1) * wn + p],
                                               nd[rk][(size_t)(l - 1) * wn + p]};
        if (!any_last || before(last_max, last)) last_max = last;
        any_last = true;
      }
    }
    for (uint32_t k = 0; k < kl; ++k) {
      int best = -1;
      std::pair<double, uint32_t> bv{-1.0, 0xffffffffu};
      for (int rk = 0; rk < world; ++rk) {
        if (head[rk] >= len[rk]) continue;
        const size_t o = (size_t)head[rk] * wn + p;
        const std::pair<double, uint32_t> v{sc[rk][o], nd[rk][o]};
        if (best < 0 || before(v, bv)) best = rk, bv = v;
      }
      if (best < 0) break;
      if (any_last && k >= (uint32_t)topk_k() && !before(bv, last_max)) break;
      ++head[best];
      ts[(size_t)k * wn + p] = bv.first;
      ti[(size_t)k * wn + p] = bv.second;
    }
  }
}

// the capacity windows' list depth across shards (YODA_GREEDY_CAP_DEPTH, as yoda_greedy's)
static uint32_t greedy_cap_depth() {
  static const uint32_t d = YODA_KNOB("YODA_GREEDY_CAP_DEPTH", 64);
  return std::max<uint32_t>(d, (uint32_t)topk_k_capacity());
}

// Greedy batch over node shards, inside libyoda ("Across GPUs"): the protocol of
// dist.sharded_greedy with RCCL (or the in-process transport): per window, K1 on every shard,
// maxima MAX / counts SUM (capacity mode: + the witnesses), the shards' candidate lists
// all-gathered and merged, the host session (identical on every rank, over `all`, the FULL
// snapshot) resolves the window; an uncertified pod is scored exactly on every shard and the
// (score, node) candidates all-gathered (capacity mode: it opens the next window).  The U64
// record path has no candidate lists: every pod is a sharded exact step (comm_step) against
// the current state.  The shards' node state is restored at the end.
static int comm_greedy(yoda_t* const* hs, int n, int world, bool local, const yoda_node_soa* all,
                       const yoda_pod_soa* pods, int mode, uint32_t flags, int32_t* pick) {
  yoda_t* h0 = hs[0];
  Coll co{hs, n, world, local};
  uint32_t* st = h0->comm_greedy_stats;  // windows, exact pods, restarts, refreshes, collectives
  std::fill(st, st + 5, 0u);
  co.calls = st + 4;
  const uint32_t P = pods->n_pods;
  for (int i = 0; i < n; ++i)
    if (!hs[i]->has_nodes) return fail(h0, YODA_ERR_NO_NODES, "no node snapshot uploaded");
  if (P == 0) return YODA_OK;
  int rc;
  PodGather win;
  if (mode == YODA_MODE_DISKIO) {  // Mode B reads no assumed-pod state: independent cycles
    std::vector<uint32_t> idx(P);
    for (uint32_t i = 0; i < P; ++i) idx[i] = i;
    win.build(pods, idx.data(), P);
    for (int i = 0; i < n; ++i)
      if ((rc = yoda_upload_pods(hs[i], &win.soa))) return rc;
    if ((rc = comm_step(hs, n, world, mode, local))) return rc;
    HIP_TRY(h0, hipMemcpyAsync(pick, h0->pick.p, (size_t)P * 4, hipMemcpyDeviceToHost,
                               h0->stream));
    HIP_TRY(h0, hipStreamSynchronize(h0->stream));
    return YODA_OK;
  }
  yoda_gs_t* g = nullptr;
  if ((rc = yoda_gs_create(all, pods, flags, &g))) return fail(h0, rc, "greedy: session setup");
  struct Guard {
    yoda_gs_t* g;
    ~Guard() { yoda_gs_destroy(g); }
  } guard{g};
  const bool capacity = (flags & YODA_GREEDY_CARD_CAPACITY) != 0;
  const bool generic = h0->generic;
  for (int i = 0; i < n; ++i)
    if (hs[i]->generic != generic)
      return fail(h0, YODA_ERR_STATE, "shards on different record paths");
  if (!generic) {  // the quotient type too (comm_step's agreement words [2], [3]), once per batch
    std::vector<void*> bq;
    std::vector<uint64_t> w((size_t)kAgreeWords * n);  // alive until the stream syncs below
    for (int i = 0; i < n; ++i) {
      uint64_t* wi = w.data() + (size_t)kAgreeWords * i;
      agreement_words(hs[i], YODA_MODE_SCV, wi);
      HIP_TRY(hs[i], hs[i]->cg_max.ensure(2 * 8));
      HIP_TRY(hs[i], hipMemcpyAsync(hs[i]->cg_max.p, wi + 2, 16, hipMemcpyHostToDevice,
                                    hs[i]->stream));
      bq.push_back(hs[i]->cg_max.p);
    }
    if ((rc = co.allreduce(bq, 2, true, ncclMax))) return rc;
    uint64_t q[2] = {0, 0};
    HIP_TRY(h0, hipMemcpyAsync(q, h0->cg_max.p, 16, hipMemcpyDeviceToHost, h0->stream));
    HIP_TRY(h0, hipStreamSynchronize(h0->stream));
    if (const char* why = quotient_disagreement(q[0], q[1])) return fail(h0, YODA_ERR_STATE, why);
  }
  std::vector<uint32_t> ids;
  std::vector<uint64_t> al, cn;
  auto push = [&](bool original) -> int {  // the session's node changes -> every shard
    const uint32_t cap = std::max<uint32_t>(g->N, 1);
    ids.resize(cap), al.resize(cap), cn.resize(cap);
    uint32_t got = 0;
    int r = original ? yoda_gs_touched_original(g, cap, ids.data(), al.data(), cn.data(), &got)
                     : yoda_gs_take_dirty(g, cap, ids.data(), al.data(), cn.data(), &got);
    if (r) return fail(h0, r, "greedy: node state");
    if (got == 0) return YODA_OK;
    for (int i = 0; i < n; ++i)
      if ((r = yoda_set_node_state(hs[i], got, ids.data(), al.data(), cn.data()))) return r;
    return YODA_OK;
  };
  auto run = [&]() -> int {
    if (generic) {  // every pod exactly, in queue order, against the current state
      for (uint32_t q = 0; q < P; ++q) {
        if ((rc = push(false))) return rc;
        win.build(pods, g->order.data() + q, 1);
        for (int i = 0; i < n; ++i)
          if ((rc = yoda_upload_pods(hs[i], &win.soa))) return rc;
        if ((rc = comm_step(hs, n, world, YODA_MODE_SCV, local))) return rc;
        int32_t pk = 0;
        HIP_TRY(h0, hipMemcpyAsync(&pk, h0->pick.p, 4, hipMemcpyDeviceToHost, h0->stream));
        HIP_TRY(h0, hipStreamSynchronize(h0->stream));
        if ((rc = yoda_gs_assign(g, q, pk))) return fail(h0, rc, "greedy: assign");
        ++h0->greedy_fallbacks;
        ++st[1];
      }
      return push(false);
    }
    const uint32_t K = (uint32_t)(capacity ? topk_k_capacity() : topk_k()),
                   W0 = std::min<uint32_t>(P, greedy_window());
    // capacity windows: each shard's lists merged deeper (shard_topk_impl, exact down to their
    // last entry), the union cut where a shard's unlisted nodes could enter (merge_shard_lists);
    // the same depth on every rank
    const uint32_t KL = capacity ? greedy_cap_depth() : K;
    std::vector<uint32_t> counts, ti, wit_h;
    std::vector<double> ts;
    std::vector<uint64_t> mx_h;
    std::vector<unsigned char> gathered, mine, one;
    uint32_t ws = 0, W = W0;
    while (ws < P) {
      const uint32_t wn = std::min(W, P - ws);
      if ((rc = push(false))) return rc;
      win.build(pods, g->order.data() + ws, wn);
      std::vector<void*> bmax, bcnt, bwc, bwn;
      for (int i = 0; i < n; ++i) {
        yoda_t* h = hs[i];
        if ((rc = yoda_upload_pods(h, &win.soa))) return rc;
        HIP_TRY(h, h->cg_max.ensure(12ull * wn * 8));  // the maxima, and a local copy
        HIP_TRY(h, h->cg_cnt.ensure(2ull * wn * 4));
        HIP_TRY(h, h->cg_wit.ensure(12ull * wn * 4));
        uint64_t* dmax = h->cg_max.as<uint64_t>();
        if (capacity) {
          if ((rc = yoda_shard_phase1_witness(h, dmax, h->cg_cnt.as<uint32_t>(),
                                              h->cg_wit.as<uint32_t>())))
            return rc;
          HIP_TRY(h, hipMemcpyAsync(dmax + 6ull * wn, dmax, 6ull * wn * 8,
                                    hipMemcpyDeviceToDevice, h->stream));
        } else if ((rc = yoda_shard_phase1(h, YODA_MODE_SCV, dmax, h->cg_cnt.as<uint32_t>()))) {
          return rc;
        }
        bmax.push_back(dmax);
        bcnt.push_back(h->cg_cnt.p);
        bwc.push_back(h->cg_wit.p);
        bwn.push_back(h->cg_wit.as<uint32_t>() + 6ull * wn);
      }
      // window exchange 1 (one group): maxima MAX, counts SUM
      co.begin();
      rc = co.allreduce(bmax, 6ull * wn, true, ncclMax);
      const int rc2 = co.allreduce(bcnt, 2ull * wn, false, ncclSum);
      const int rc3 = co.end();
      if (rc || (rc = rc2) || (rc = rc3)) return rc;
      if (capacity) {
        for (int i = 0; i < n; ++i) {
          uint64_t* dmax = hs[i]->cg_max.as<uint64_t>();
          if ((rc = yoda_shard_witness_prepare(hs[i], dmax, dmax + 6ull * wn,
                                               hs[i]->cg_wit.as<uint32_t>())))
            return rc;
        }
      }
      // the shards' candidate lists, all-gathered and merged: the first K of the union in
      // (score desc, node asc) order contain the global top K (window pods [from, wn) only).
      // Window exchange 2 (one group): the lists' all-gather and, in capacity mode, the
      // witness counts SUM and lowest witnesses MIN (they need only exchange 1's maxima)
      counts.resize(2ull * wn);
      auto merged_lists = [&](uint32_t from, bool with_witness) -> int {
        const size_t lb = (size_t)KL * wn * 12;  // per shard: KL x wn scores (f64) + nodes (u32)
        mine.resize((size_t)n * lb);
        for (int i = 0; i < n; ++i) {
          unsigned char* m = mine.data() + (size_t)i * lb;
          int r = shard_topk_impl(hs[i], hs[i]->cg_max.as<uint64_t>(),
                                  hs[i]->cg_cnt.as<uint32_t>(), K, KL > K ? KL : 0u,
                                  counts.data(), reinterpret_cast<double*>(m),
                                  reinterpret_cast<uint32_t*>(m + (size_t)KL * wn * 8));
          if (r) return r;
        }
        std::vector<const void*> ins;
        for (int i = 0; i < n; ++i) ins.push_back(mine.data() + (size_t)i * lb);
        co.begin();
        int r = with_witness ? co.allreduce(bwc, 6ull * wn, false, ncclSum) : YODA_OK;
        if (!r && with_witness) r = co.allreduce(bwn, 6ull * wn, false, ncclMin);
        if (!r) r = co.allgather_issue(ins, lb, gathered);
        const int re = co.end();
        if (r || (r = re) || (r = co.allgather_finish(lb, gathered))) return r;
        ts.assign((size_t)KL * wn, -1.0);
        ti.assign((size_t)KL * wn, 0xffffffffu);
        std::vector<const double*> sc(world);
        std::vector<const uint32_t*> nd(world);
        for (int rk = 0; rk < world; ++rk) {
          const unsigned char* b = gathered.data() + (size_t)rk * lb;
          sc[rk] = reinterpret_cast<const double*>(b);
          nd[rk] = reinterpret_cast<const uint32_t*>(b + (size_t)KL * wn * 8);
        }
        merge_shard_lists(world, wn, KL, KL > K, from, sc.data(), nd.data(), ts.data(),
                          ti.data());
        return YODA_OK;
      };
      if ((rc = merged_lists(0, capacity))) return rc;
      if ((rc = yoda_gs_begin_window(g, ws, wn, KL, counts.data(), ts.data(), ti.data())))
        return fail(h0, rc, "greedy: begin window");
      ++h0->greedy_windows;
      ++st[0];
      if (capacity) {
        mx_h.resize(6ull * wn);
        wit_h.resize(12ull * wn);
        if ((rc = yoda_shard_witness_download(h0, h0->cg_max.as<uint64_t>(),
                                              h0->cg_wit.as<uint32_t>(), mx_h.data(),
                                              wit_h.data())))
          return rc;
        if ((rc = yoda_gs_set_witness(g, mx_h.data(), wit_h.data(), wit_h.data() + 6ull * wn)))
          return fail(h0, rc, "greedy: witnesses");
        uint32_t nxt = 0;
        if ((rc = yoda_gs_resolve(g, &nxt))) return fail(h0, rc, "greedy: resolve");
        if (nxt < wn) {  // the uncertified pod opens the next window (yoda_greedy's rule)
          ++h0->greedy_restarts;
          ++st[2];
          ws += nxt;
          W = yoda_greedy_next_window(nxt, W0);
        } else {
          ws += wn;
          W = std::min<uint32_t>(W0, 2 * W);
        }
        continue;
      }
      // mid-window list refresh (yoda_greedy's): every kFbCheck exact pods,
      // when >= kScanMin of the next kScan window pods are uncertified already, every shard's
      // top-k runs again against the current state and the merged lists replace the old ones
      constexpr uint32_t kFbCheck = 8, kScan = 256, kScanMin = 16;
      uint32_t fb_since = 0;
      for (;;) {
        uint32_t nxt = 0;
        if ((rc = yoda_gs_resolve(g, &nxt))) return fail(h0, rc, "greedy: resolve");
        if (nxt >= wn) break;
        if (++fb_since >= kFbCheck && wn - nxt >= 2 * kScan && !g->wrapped) {
          fb_since = 0;
          uint32_t unc = 0;
          if ((rc = yoda_gs_uncertified(g, nxt + 1, kScan, &unc))) return fail(h0, rc, "greedy");
          if (unc >= kScanMin) {
            if ((rc = push(false))) return rc;
            if ((rc = merged_lists(nxt, false))) return rc;
            if ((rc = yoda_gs_refresh(g, nxt, ts.data(), ti.data())))
              return fail(h0, rc, "greedy: refresh");
            ++h0->greedy_refreshes;
            ++st[3];
            uint32_t again = 0;
            if ((rc = yoda_gs_resolve(g, &again))) return fail(h0, rc, "greedy: resolve");
            if (again >= wn) break;
            nxt = again;
          }
        }
        if ((rc = push(false))) return rc;
        one.resize((size_t)n * 16);
        for (int i = 0; i < n; ++i) {
          double sc = -1.0;
          int32_t nd = -1;
          if ((rc = yoda_shard_best_one(hs[i], nxt, &sc, &nd))) return rc;
          const int64_t nd64 = nd;
          std::memcpy(one.data() + 16 * (size_t)i, &sc, 8);
          std::memcpy(one.data() + 16 * (size_t)i + 8, &nd64, 8);
        }
        std::vector<const void*> in1;
        for (int i = 0; i < n; ++i) in1.push_back(one.data() + 16 * (size_t)i);
        if ((rc = co.allgather(in1, 16, gathered))) return rc;
        double bs = -1.0;
        int64_t bn = -1;
        for (int r = 0; r < world; ++r) {
          double sc;
          int64_t nd;
          std::memcpy(&sc, gathered.data() + 16 * (size_t)r, 8);
          std::memcpy(&nd, gathered.data() + 16 * (size_t)r + 8, 8);
          if (nd >= 0 && (sc > bs || (sc == bs && nd < bn))) {
            bs = sc;
            bn = nd;
          }
        }
        if (bn < 0) return fail(h0, YODA_ERR_STATE, "greedy: no feasible node for a window pod");
        if ((rc = yoda_gs_assign(g, ws + nxt, (int32_t)bn))) return fail(h0, rc, "greedy: assign");
        ++h0->greedy_fallbacks;
        ++st[1];
      }
      ws += wn;
    }
    return push(false);
  };
  h0->greedy_windows = h0->greedy_fallbacks = h0->greedy_restarts = h0->greedy_refreshes = 0;
  {  // a greedy batch on every shard: its pushes keep the block bounds valid (no rebuilds)
    std::vector<std::unique_ptr<GreedyScope>> scopes;
    for (int i = 0; i < n; ++i) scopes.emplace_back(new GreedyScope(hs[i]));
    rc = run();
  }
  const int rr = push(true);  // restore the shards' original node state
  if (rc) return rc;
  if (rr) return rr;
  uint32_t resolved = 0, assigned = 0;
  return yoda_gs_picks(g, pick, &resolved, &assigned);
}

extern "C" {
int yoda_greedy_cap_depth(void) { return (int)greedy_cap_depth(); }

int yoda_shard_topk_deep(yoda_t* h, const uint64_t* d_maxima, const uint32_t* d_counts,
                         uint32_t k, uint32_t deep, uint32_t* counts, double* top_score,
                         uint32_t* top_node) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (deep > 1024) return fail(h, YODA_ERR_INVALID_ARG, "yoda_shard_topk_deep: deep > 1024");
  return shard_topk_impl(h, d_maxima, d_counts, k, deep, counts, top_score, top_node);
}

int yoda_merge_shard_lists(uint32_t world, uint32_t wn, uint32_t kl, uint32_t from,
                           const double* scores, const uint32_t* nodes, double* out_score,
                           uint32_t* out_node) {
  if (world < 1 || kl < 1 || from > wn || !scores || !nodes || !out_score || !out_node)
    return YODA_ERR_INVALID_ARG;
  try {
    std::vector<const double*> sc(world);
    std::vector<const uint32_t*> nd(world);
    for (uint32_t rk = 0; rk < world; ++rk) {
      sc[rk] = scores + (size_t)rk * kl * wn;
      nd[rk] = nodes + (size_t)rk * kl * wn;
    }
    for (uint32_t k = 0; k < kl; ++k)
      for (uint32_t p = from; p < wn; ++p) {
        out_score[(size_t)k * wn + p] = -1.0;
        out_node[(size_t)k * wn + p] = 0xffffffffu;
      }
    merge_shard_lists((int)world, wn, kl, kl > (uint32_t)topk_k_capacity(), from, sc.data(),
                      nd.data(), out_score, out_node);
    return YODA_OK;
  } catch (...) {
    return YODA_ERR_INVALID_ARG;
  }
}

int yoda_comm_greedy_stats(const yoda_t* h, uint32_t* out) {
  if (!h || !out) return YODA_ERR_INVALID_ARG;
  std::copy(h->comm_greedy_stats, h->comm_greedy_stats + 5, out);
  return YODA_OK;
}

int yoda_comm_unique_id(uint8_t* id) {
  if (!id) return YODA_ERR_INVALID_ARG;
  if (!rccl().load()) return YODA_ERR_HIP;
  ncclUniqueId u;
  if (rccl().get_unique_id(&u) != ncclSuccess) return YODA_ERR_HIP;
  std::memcpy(id, &u, sizeof(u));
  return YODA_OK;
}

int yoda_device_bus_id(const yoda_t* h, char* out, int len) {
  if (!h || !out || len < 2) return YODA_ERR_INVALID_ARG;
  std::memset(out, 0, (size_t)len);
  if (hipDeviceGetPCIBusId(out, len - 1, h->device) != hipSuccess) return YODA_ERR_HIP;
  return YODA_OK;
}

// The host's identity for the device check: FNV-1a 64 of the hostname and the kernel's boot id
// (what NCCL's hostHash takes), so identical servers -- equal PCI bus ids -- still differ.
static uint64_t host_hash() {
  uint64_t x = 1469598103934665603ull;
  const auto mix = [&](const char* s, size_t n) {
    for (size_t i = 0; i < n; ++i) x = (x ^ (unsigned char)s[i]) * 1099511628211ull;
  };
  char name[256] = {0};
  gethostname(name, sizeof(name) - 1);
  mix(name, strnlen(name, sizeof(name)));
  if (FILE* f = std::fopen("/proc/sys/kernel/random/boot_id", "r")) {
    char b[64] = {0};
    const size_t n = std::fread(b, 1, sizeof(b) - 1, f);
    std::fclose(f);
    mix(b, n);
  }
  return x;
}

int yoda_device_key(const yoda_t* h, char* out, int len) {
  if (!h || !out || len < 32) return YODA_ERR_INVALID_ARG;
  char bus[YODA_BUS_ID_BYTES];
  int rc = yoda_device_bus_id(h, bus, sizeof(bus));
  if (rc) return rc;
  const int n = std::snprintf(out, (size_t)len, "%016llx/%s", (unsigned long long)host_hash(), bus);
  return n > 0 && n < len ? YODA_OK : YODA_ERR_INVALID_ARG;
}

int yoda_comm_check_devices(const char* bus_ids, int world, int stride, int* rank_a,
                            int* rank_b) {
  if (!bus_ids || world < 1 || stride < 1) return YODA_ERR_INVALID_ARG;
  const auto id = [&](int r) {
    const char* p = bus_ids + (size_t)r * stride;
    return std::string(p, strnlen(p, (size_t)stride));
  };
  for (int a = 0; a < world; ++a) {
    const std::string ia = id(a);
    if (ia.empty()) return YODA_ERR_INVALID_ARG;
    for (int b = a + 1; b < world; ++b)
      if (ia == id(b)) {
        if (rank_a) *rank_a = a;
        if (rank_b) *rank_b = b;
        return YODA_ERR_SAME_DEVICE;
      }
  }
  return YODA_OK;
}

int yoda_comm_init(yoda_t* h, const uint8_t* id, int rank, int world) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!id || world < 1 || rank < 0 || rank >= world)
    return fail(h, YODA_ERR_INVALID_ARG, "bad communicator id / rank / world");
  if (!rccl().load()) return fail(h, YODA_ERR_HIP, rccl().err);
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->comm) {
    (void)rccl().comm_destroy(h->comm);
    h->comm = nullptr;
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t r = rccl().comm_init_rank(&h->comm, world, u, rank);
  if (r != ncclSuccess) {
    h->comm = nullptr;
    std::string msg = std::string("ncclCommInitRank: ") + rccl().error_string(r);
    if (r == ncclInvalidUsage)  // the usual cause: two ranks on one GPU
      msg += " (RCCL refuses two ranks of one communicator on the same GPU: check the "
             "ranks' devices with yoda_device_bus_id / yoda_comm_check_devices)";
    return fail(h, YODA_ERR_HIP, msg);
  }
  h->comm_rank = rank;
  h->comm_world = world;
  return YODA_OK;
}

int yoda_comm_run(yoda_t* h, int mode) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!h->comm) return fail(h, YODA_ERR_STATE, "yoda_comm_run before yoda_comm_init");
  try {
    yoda_t* hs[1] = {h};
    return comm_step(hs, 1, h->comm_world, mode, false);
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_comm_greedy(yoda_t* h, const yoda_node_soa* all_nodes, const yoda_pod_soa* pods,
                     int mode, uint32_t flags, int32_t* pick) {
  if (!h) return YODA_ERR_INVALID_ARG;
  if (!all_nodes || !pods || !pick) return fail(h, YODA_ERR_INVALID_ARG, "NULL argument");
  if (!h->comm) return fail(h, YODA_ERR_STATE, "yoda_comm_greedy before yoda_comm_init");
  try {
    HIP_TRY(h, hipSetDevice(h->device));
    yoda_t* hs[1] = {h};
    return comm_greedy(hs, 1, h->comm_world, false, all_nodes, pods, mode, flags, pick);
  } catch (const std::bad_alloc&) {
    return fail(h, YODA_ERR_INVALID_ARG, "host allocation failed");
  } catch (...) {
    return fail(h, YODA_ERR_INVALID_ARG, "unexpected exception");
  }
}

int yoda_comm_greedy_local(yoda_t* const* hs, int world, const yoda_node_soa* all_nodes,
                           const yoda_pod_soa* pods, int mode, uint32_t flags, int32_t* pick) {
  if (!hs || world < 1 || world > kMaxLocalShards || !all_nodes || !pods || !pick)
    return YODA_ERR_INVALID_ARG;
  for (int i = 0; i < world; ++i)
    if (!hs[i]) return YODA_ERR_INVALID_ARG;
  for (int i = 1; i < world; ++i)
    if (hs[i]->device != hs[0]->device)
      return fail(hs[0], YODA_ERR_INVALID_ARG, "local exchange: shards on different devices");
  // one stream for every shard (the device copies order after the kernels); a shard's own
  // queued work is ordered before it (switch_stream), and the shared stream's after it on exit
  std::vector<hipStream_t> saved(world);
  for (int i = 0; i < world; ++i) {
    saved[i] = hs[i]->stream;
    if (switch_stream(hs[i], hs[0]->stream) != YODA_OK) {
      for (int j = 0; j < i; ++j) (void)switch_stream(hs[j], saved[j]);
      return YODA_ERR_HIP;
    }
  }
  int rc;
  try {
    rc = hipSetDevice(hs[0]->device) == hipSuccess
             ? comm_greedy(hs, world, world, true, all_nodes, pods, mode, flags, pick)
             : YODA_ERR_HIP;
  } catch (...) {
    rc = fail(hs[0], YODA_ERR_INVALID_ARG, "unexpected exception");
  }
  for (int i = 0; i < world; ++i)
    if (switch_stream(hs[i], saved[i]) != YODA_OK && rc == YODA_OK) rc = YODA_ERR_HIP;
  return rc;
}

int yoda_comm_run_local(yoda_t* const* hs, int world, int mode) {
  if (!hs || world < 1 || world > kMaxLocalShards) return YODA_ERR_INVALID_ARG;
  for (int i = 0; i < world; ++i)
    if (!hs[i]) return YODA_ERR_INVALID_ARG;
  for (int i = 1; i < world; ++i)
    if (hs[i]->device != hs[0]->device)
      return fail(hs[0], YODA_ERR_INVALID_ARG, "local exchange: shards on different devices");
  // one stream for every shard (the device copies order after the kernels); a shard's own
  // queued work is ordered before it (switch_stream), and the shared stream's after it on exit
  std::vector<hipStream_t> saved(world);
  for (int i = 0; i < world; ++i) {
    saved[i] = hs[i]->stream;
    if (switch_stream(hs[i], hs[0]->stream) != YODA_OK) {
      for (int j = 0; j < i; ++j) (void)switch_stream(hs[j], saved[j]);
      return YODA_ERR_HIP;
    }
  }
  int rc;
  try {
    rc = comm_step(hs, world, world, mode, true);
  } catch (...) {
    rc = fail(hs[0], YODA_ERR_INVALID_ARG, "unexpected exception");
  }
  if (rc == YODA_OK && hipStreamSynchronize(hs[0]->stream) != hipSuccess) rc = YODA_ERR_HIP;
  for (int i = 0; i < world; ++i)
    if (switch_stream(hs[i], saved[i]) != YODA_OK && rc == YODA_OK) rc = YODA_ERR_HIP;
  return rc;
}

}  // extern "C"
