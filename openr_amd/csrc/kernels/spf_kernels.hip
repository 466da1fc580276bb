// Batched SPF and route-selection kernels for gfx950 (MI355X).
//
// Semantics: LinkState::runSpf (openr/decision/LinkState.cpp:808-882) in its
// closed form, valid for link metrics >= 1:
//   d(u)   shortest metric over up, non-ignored links, no transit through an
//          overloaded node other than the source (:831-838)
//   NH(u)  = OR over predecessors (l, v) with d(v) + w_v(l) == d(u) and v a
//          transit node of   (v == src ? {u} : NH(v))          (:857-873)
//
// Algorithm: one workgroup per source, level-synchronous Dijkstra that
// settles every node of the current minimum distance D at once (exact for
// positive integer metrics). Per level, ONE pass over the pending list
//   - nodes at distance D are settled: their first-hop mask is pulled from
//     already-settled predecessors (d < D), then their out-links are relaxed
//     with LDS atomicMin (push); newly touched nodes are appended;
//   - nodes above D are carried over;
// and ONE __syncthreads(). The next D is the minimum over values that were
// carried or that lowered a distance, reduced during the same pass.
//
// State lives in LDS. Packed variants hold a node's (dist, mask) in one word
// so the relaxation is a single ds_min:
//   K16: u32 = dist16 << 16 | mask16   (paths < 0xFFFF, <= 16 neighbours)
//   K32: u64 = dist32 << 32 | mask32   (paths < 2^32-1, <= 32 neighbours)
// KW: separate u32 dist and W mask words (any neighbour count).
// A node's mask half is garbage (all ones) until the node settles; pushes
// never touch settled nodes (they only write D + w > D), so the settle store
// and concurrent ds_min on the same word commute.
//
// HBM traffic per source: the CSR (16 B per directed edge + row offsets) is
// shared by every workgroup and stays L2/MALL-resident; each source writes
// its dist row and mask row once, coalesced, at the end.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spf_kernels.h"

namespace orh {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// ---------------------------------------------------------------------------
// state policies
// ---------------------------------------------------------------------------
struct K16 {
  using Word = uint32_t;
  static constexpr Word kInf = 0xFFFFFFFFu;
  static constexpr uint32_t kDistInf = 0xFFFFu;
  static constexpr int kMaxNbr = 16;
  __device__ static uint32_t dist(Word w) { return w >> 16; }
  __device__ static uint32_t mask(Word w) { return w & 0xFFFFu; }
  __device__ static Word tentative(uint32_t d) { return (d << 16) | 0xFFFFu; }
  __device__ static Word settled(uint32_t d, uint32_t m) { return (d << 16) | m; }
};

struct K32 {
  using Word = unsigned long long;
  static constexpr Word kInf = ~0ull;
  static constexpr uint32_t kDistInf = 0xFFFFFFFFu;
  static constexpr int kMaxNbr = 32;
  __device__ static uint32_t dist(Word w) { return static_cast<uint32_t>(w >> 32); }
  __device__ static uint32_t mask(Word w) { return static_cast<uint32_t>(w); }
  __device__ static Word tentative(uint32_t d) { return (static_cast<Word>(d) << 32) | 0xFFFFFFFFull; }
  __device__ static Word settled(uint32_t d, uint32_t m) {
    return (static_cast<Word>(d) << 32) | m;
  }
};

__device__ inline uint32_t lane_id() { return __lane_id(); }

// wave-aggregated append of `val` (where pred) to list[*cnt++]
template <typename IdT>
__device__ inline void wave_append(IdT* list, uint32_t* cnt, bool pred, uint32_t val) {
  const unsigned long long m = __ballot(pred);
  if (m == 0) return;
  const int lane = lane_id();
  const int leader = __ffsll(static_cast<long long>(m)) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(cnt, static_cast<uint32_t>(__popcll(m)));
  base = __shfl(base, leader);
  if (pred) {
    const unsigned long long below = (lane == 0) ? 0ull : (m & ((1ull << lane) - 1ull));
    list[base + __popcll(below)] = static_cast<IdT>(val);
  }
}

__device__ inline uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, static_cast<uint32_t>(__shfl_xor(v, off)));
  return v;
}

__device__ inline bool ignored(const uint32_t* ign, uint32_t n, uint32_t link) {
  // sorted ascending; n is tiny (KSP2 / what-if sets)
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t x = ign[mid];
    if (x == link) return true;
    if (x < link) lo = mid + 1; else hi = mid;
  }
  return false;
}

// ---------------------------------------------------------------------------
// packed-state kernel (K16 / K32)
// ---------------------------------------------------------------------------
template <class P, typename IdT>
__global__ __launch_bounds__(kBlock) void spf_packed_kernel(SpfArgs a) {
  using Word = typename P::Word;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t N = a.n_nodes;
  Word* word = reinterpret_cast<Word*>(smem);
  IdT* lists = reinterpret_cast<IdT*>(smem + a.lds_list_off);
  __shared__ uint32_t s_cnt[3];
  __shared__ uint32_t s_min[3];

  const uint32_t tid = threadIdx.x;
  const uint32_t sidx = blockIdx.x;
  const uint32_t src = a.srcs[sidx];
  const uint32_t ign_b = a.ignore_ptr ? a.ignore_ptr[sidx] : 0u;
  const uint32_t n_ign = a.ignore_ptr ? a.ignore_ptr[sidx + 1] - ign_b : 0u;
  const uint32_t* ign = a.ignore_links + ign_b;

  for (uint32_t i = tid; i < N; i += kBlock) word[i] = P::kInf;
  if (tid < 3) {
    s_cnt[tid] = 0;
    s_min[tid] = 0xFFFFFFFFu;
  }
  __syncthreads();
  if (tid == 0) {
    word[src] = P::settled(0, 0);
    lists[0] = static_cast<IdT>(src);
  }
  __syncthreads();

  uint32_t cur_n = 1;
  uint32_t D = 0;
  const bool use_metric = a.use_link_metric != 0;
  for (uint32_t level = 0;; ++level) {
    IdT* in = lists + ((level & 1) ? N : 0);
    IdT* out = lists + ((level & 1) ? 0 : N);
    uint32_t* cnt_w = &s_cnt[level % 3];
    uint32_t* min_w = &s_min[level % 3];
    if (tid == 0) {  // slot of the next level; last read one level ago
      s_cnt[(level + 1) % 3] = 0;
      s_min[(level + 1) % 3] = 0xFFFFFFFFu;
    }
    uint32_t local_min = 0xFFFFFFFFu;
    for (uint32_t base = 0; base < cur_n; base += kBlock) {
      const uint32_t i = base + tid;
      const bool active = i < cur_n;
      const uint32_t v = active ? static_cast<uint32_t>(in[i]) : 0u;
      const uint32_t dv = active ? P::dist(word[v]) : 0u;
      const bool settle = active && dv == D;
      // carry unsettled pending nodes to the next level
      wave_append(out, cnt_w, active && !settle, v);
      if (active && !settle) local_min = min(local_min, dv);
      if (settle) {
        const bool transit = (v == src) || !a.node_overloaded[v];
        const uint32_t e0 = a.row_ptr[v], e1 = a.row_ptr[v + 1];
        uint32_t acc = 0;
        for (uint32_t e = e0; e < e1; ++e) {
          const uint4 rec = a.edges[e];  // {col, w_out, w_in, meta}
          if (rec.w & ORH_META_DOWN_) continue;
          if (n_ign && ignored(ign, n_ign, rec.w & ORH_META_LINK_MASK_)) continue;
          const uint32_t u = rec.x;
          const uint32_t w_out = use_metric ? rec.y : 1u;
          const uint32_t w_in = use_metric ? rec.z : 1u;
          if (v != src) {  // pull the first-hop mask from settled predecessors
            const Word wu = word[u];
            const uint32_t du = P::dist(wu);
            const bool pred_transit = (u == src) || !(rec.w & ORH_META_COL_OVERLOADED_);
            if (du < D && du + w_in == D && pred_transit) {
              acc |= (u == src) ? (1u << a.rank_in_col[e]) : P::mask(wu);
            }
          }
          if (transit) {  // relax (push)
            const uint32_t nd = D + w_out;
            const Word old = atomicMin(&word[u], P::tentative(nd));
            const uint32_t od = P::dist(old);
            if (nd < od) local_min = min(local_min, nd);
            wave_append(out, cnt_w, od == P::kDistInf, u);
          }
        }
        if (v != src) word[v] = P::settled(D, acc);
      }
    }
    const uint32_t wm = wave_min(local_min);
    if (lane_id() == 0 && wm != 0xFFFFFFFFu) atomicMin(min_w, wm);
    __syncthreads();
    cur_n = *cnt_w;
    // every level settles at least one node: > N levels would be a bug, and
    // the bound guarantees every wave reaches the exit
    if (cur_n == 0 || level >= N) break;
    D = *min_w;
  }

  // coalesced write-out of the dist row and the first-hop mask row
  uint32_t* od = a.out_dist + static_cast<size_t>(sidx) * N;
  uint32_t* on = a.out_nh + static_cast<size_t>(sidx) * N * a.words;
  for (uint32_t i = tid; i < N; i += kBlock) {
    const Word w = word[i];
    const uint32_t d = P::dist(w);
    const bool reach = d != P::kDistInf;
    od[i] = reach ? d : 0xFFFFFFFFu;
    if (a.words == 1) {
      on[i] = reach ? P::mask(w) : 0u;
    } else {
      on[static_cast<size_t>(i) * a.words] = reach ? P::mask(w) : 0u;
      for (uint32_t k = 1; k < a.words; ++k) on[static_cast<size_t>(i) * a.words + k] = 0u;
    }
  }
}

// ---------------------------------------------------------------------------
// wide-mask kernel (KW): separate u32 dist and W mask words per node
// ---------------------------------------------------------------------------
template <typename IdT>
__global__ __launch_bounds__(kBlock) void spf_wide_kernel(SpfArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t N = a.n_nodes;
  const uint32_t W = a.words;
  uint32_t* dist = reinterpret_cast<uint32_t*>(smem);
  uint32_t* mask = reinterpret_cast<uint32_t*>(smem + a.lds_mask_off);
  IdT* lists = reinterpret_cast<IdT*>(smem + a.lds_list_off);
  __shared__ uint32_t s_cnt[3];
  __shared__ uint32_t s_min[3];

  const uint32_t tid = threadIdx.x;
  const uint32_t sidx = blockIdx.x;
  const uint32_t src = a.srcs[sidx];
  const uint32_t ign_b = a.ignore_ptr ? a.ignore_ptr[sidx] : 0u;
  const uint32_t n_ign = a.ignore_ptr ? a.ignore_ptr[sidx + 1] - ign_b : 0u;
  const uint32_t* ign = a.ignore_links + ign_b;

  for (uint32_t i = tid; i < N; i += kBlock) dist[i] = 0xFFFFFFFFu;
  for (uint32_t i = tid; i < N * W; i += kBlock) mask[i] = 0u;
  if (tid < 3) {
    s_cnt[tid] = 0;
    s_min[tid] = 0xFFFFFFFFu;
  }
  __syncthreads();
  if (tid == 0) {
    dist[src] = 0;
    lists[0] = static_cast<IdT>(src);
  }
  __syncthreads();

  uint32_t cur_n = 1;
  uint32_t D = 0;
  const bool use_metric = a.use_link_metric != 0;
  for (uint32_t level = 0;; ++level) {
    IdT* in = lists + ((level & 1) ? N : 0);
    IdT* out = lists + ((level & 1) ? 0 : N);
    uint32_t* cnt_w = &s_cnt[level % 3];
    uint32_t* min_w = &s_min[level % 3];
    if (tid == 0) {
      s_cnt[(level + 1) % 3] = 0;
      s_min[(level + 1) % 3] = 0xFFFFFFFFu;
    }
    uint32_t local_min = 0xFFFFFFFFu;
    for (uint32_t base = 0; base < cur_n; base += kBlock) {
      const uint32_t i = base + tid;
      const bool active = i < cur_n;
      const uint32_t v = active ? static_cast<uint32_t>(in[i]) : 0u;
      const uint32_t dv = active ? dist[v] : 0u;
      const bool settle = active && dv == D;
      wave_append(out, cnt_w, active && !settle, v);
      if (active && !settle) local_min = min(local_min, dv);
      if (settle) {
        const bool transit = (v == src) || !a.node_overloaded[v];
        const uint32_t e0 = a.row_ptr[v], e1 = a.row_ptr[v + 1];
        for (uint32_t e = e0; e < e1; ++e) {
          const uint4 rec = a.edges[e];
          if (rec.w & ORH_META_DOWN_) continue;
          if (n_ign && ignored(ign, n_ign, rec.w & ORH_META_LINK_MASK_)) continue;
          const uint32_t u = rec.x;
          const uint32_t w_out = use_metric ? rec.y : 1u;
          const uint32_t w_in = use_metric ? rec.z : 1u;
          if (v != src) {
            const uint32_t du = dist[u];
            const bool pred_transit = (u == src) || !(rec.w & ORH_META_COL_OVERLOADED_);
            if (du < D && du + w_in == D && pred_transit) {
              if (u == src) {
                const uint32_t r = a.rank_in_col[e];
                mask[static_cast<size_t>(v) * W + (r >> 5)] |= 1u << (r & 31u);
              } else {
                for (uint32_t k = 0; k < W; ++k)
                  mask[static_cast<size_t>(v) * W + k] |= mask[static_cast<size_t>(u) * W + k];
              }
            }
          }
          if (transit) {
            const uint32_t nd = D + w_out;
            const uint32_t old = atomicMin(&dist[u], nd);
            if (nd < old) local_min = min(local_min, nd);
            wave_append(out, cnt_w, old == 0xFFFFFFFFu, u);
          }
        }
      }
    }
    const uint32_t wm = wave_min(local_min);
    if (lane_id() == 0 && wm != 0xFFFFFFFFu) atomicMin(min_w, wm);
    __syncthreads();
    cur_n = *cnt_w;
    // every level settles at least one node: > N levels would be a bug, and
    // the bound guarantees every wave reaches the exit
    if (cur_n == 0 || level >= N) break;
    D = *min_w;
  }

  uint32_t* od = a.out_dist + static_cast<size_t>(sidx) * N;
  uint32_t* on = a.out_nh + static_cast<size_t>(sidx) * N * W;
  for (uint32_t i = tid; i < N; i += kBlock) od[i] = dist[i];
  for (uint32_t i = tid; i < N * W; i += kBlock) on[i] = mask[i];
}

// ---------------------------------------------------------------------------
// route selection: getMinCostNodes + nexthop OR (Decision.cpp:1152-1228)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void route_select_kernel(RouteSelectArgs a) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= a.n_prefix) return;
  const uint32_t b = a.adv_ptr[p], e = a.adv_ptr[p + 1];
  uint32_t best = 0xFFFFFFFFu;
  for (uint32_t i = b; i < e; ++i) best = min(best, a.dist[a.adv[i]]);
  a.min_out[p] = best;
  for (uint32_t k = 0; k < a.words; ++k) {
    uint32_t m = 0;
    if (best != 0xFFFFFFFFu) {
      for (uint32_t i = b; i < e; ++i) {
        const uint32_t v = a.adv[i];
        if (a.dist[v] == best) m |= a.nh[static_cast<size_t>(v) * a.words + k];
      }
    }
    a.nh_out[static_cast<size_t>(p) * a.words + k] = m;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <typename K>
static hipError_t launch(K kernel, const SpfArgs& a, uint32_t grid, size_t lds, hipStream_t s) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     static_cast<int>(lds));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), lds, s, a);
  return hipGetLastError();
}

static size_t align16(size_t x) { return (x + 15) & ~static_cast<size_t>(15); }

SpfPlan plan_spf(uint32_t n_nodes, uint32_t words, uint32_t max_nbr, uint64_t path_bound,
                 size_t lds_limit) {
  SpfPlan p{};
  const size_t id_bytes = n_nodes <= 0xFFFFu ? 2 : 4;
  p.id16 = id_bytes == 2;
  const size_t lists = 2 * static_cast<size_t>(n_nodes) * id_bytes;
  if (max_nbr <= 16 && path_bound < 0xFFFFu) {
    p.variant = SpfVariant::kK16;
    p.list_off = align16(static_cast<size_t>(n_nodes) * 4);
    p.mask_off = 0;
  } else if (max_nbr <= 32 && path_bound < 0xFFFFFFFFull) {
    p.variant = SpfVariant::kK32;
    p.list_off = align16(static_cast<size_t>(n_nodes) * 8);
    p.mask_off = 0;
  } else if (path_bound < 0xFFFFFFFFull) {
    p.variant = SpfVariant::kWide;
    p.mask_off = align16(static_cast<size_t>(n_nodes) * 4);
    p.list_off = p.mask_off + align16(static_cast<size_t>(n_nodes) * 4 * words);
  } else {
    p.variant = SpfVariant::kUnsupported;
    return p;
  }
  p.lds_bytes = p.list_off + align16(lists);
  if (p.lds_bytes > lds_limit) p.variant = SpfVariant::kUnsupported;
  return p;
}

hipError_t launch_spf(const SpfPlan& plan, SpfArgs a, uint32_t n_src, hipStream_t s) {
  a.lds_list_off = static_cast<uint32_t>(plan.list_off);
  a.lds_mask_off = static_cast<uint32_t>(plan.mask_off);
  switch (plan.variant) {
    case SpfVariant::kK16:
      return plan.id16 ? launch(spf_packed_kernel<K16, uint16_t>, a, n_src, plan.lds_bytes, s)
                       : launch(spf_packed_kernel<K16, uint32_t>, a, n_src, plan.lds_bytes, s);
    case SpfVariant::kK32:
      return plan.id16 ? launch(spf_packed_kernel<K32, uint16_t>, a, n_src, plan.lds_bytes, s)
                       : launch(spf_packed_kernel<K32, uint32_t>, a, n_src, plan.lds_bytes, s);
    case SpfVariant::kWide:
      return plan.id16 ? launch(spf_wide_kernel<uint16_t>, a, n_src, plan.lds_bytes, s)
                       : launch(spf_wide_kernel<uint32_t>, a, n_src, plan.lds_bytes, s);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_route_select(const RouteSelectArgs& a, hipStream_t s) {
  if (a.n_prefix == 0) return hipSuccess;
  const uint32_t grid = (a.n_prefix + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(route_select_kernel, dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace orh
