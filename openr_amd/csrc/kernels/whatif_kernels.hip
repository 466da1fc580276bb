// What-if repair: batched runSpf(src, useLinkMetric, linksToIgnore) derived
// from the plain SPF rows of the batch's sources (gfx950).
//
// A what-if batch (link-failure SPFs, "1,024 runSpf(src,
// true, {link})" = few sources x many links) repeats its sources. Removing
// links only lengthens paths, and only below a link that is tight on the
// source's shortest-path DAG (LinkState.cpp:857-873 closed form, SURVEY.md
// Appendix A.1):
//
//   A = the heads of the ignored links that are tight (d(x) + w_x = d(y), x
//       a transit node), closed under tight out-edges of transit nodes.
//
// Every node outside A keeps its distance AND its first-hop set: none of its
// tight predecessors is in A and none of its tight in-links is ignored, so by
// induction on d its predecessor set is unchanged. Nodes in A are re-derived
// from the closed form restricted to A: a boundary label per node (the lattice
// meet over its predecessors outside A: smaller distance replaces, equal
// distance ORs the masks) and then chaotic relaxation over the predecessor
// edges inside A until no label changes. Positive metrics make the predecessor
// graph of the final labels acyclic, so the fixpoint is unique and equals what
// a fresh search computes: results are bit-identical to runSpf on the reduced
// graph. A link-failure batch touches few nodes per request (C4: 55 % of the
// requests have an empty A, the mean is 4 nodes, the largest 932), so the
// batch costs its sources' searches plus one streaming copy of the rows.
//
// Kernels:
//   whatif_copy_kernel    base rows -> request rows (dist + one mask word),
//                         16-byte loads/stores, HBM-bound (the output floor)
//   whatif_repair_kernel  one workgroup per request: A in LDS (bitmap over
//                         the nodes, node list, labels, predecessor edges);
//                         a request whose A or edge list outgrows LDS is
//                         flagged, repaired again with its state in a global
//                         slot sized for the whole graph, and only when the
//                         slots run out re-searched by spf_global_nh_kernel
//                         with the flags as its row mask

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "spf_kernels.h"  // edge record flags
#include "whatif_kernels.h"

namespace orh {
namespace {

constexpr uint32_t kSlotBlock = 1024;  // slot pass: few large affected sets, one per CU
constexpr uint32_t kInfD = 0xFFFFFFFFu;
constexpr unsigned long long kInfLab = 0xFFFFFFFF00000000ull;  // {dist = inf, mask = 0}

__device__ inline bool is_ignored(const uint32_t* ign, uint32_t n, uint32_t link) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t x = ign[mid];
    if (x == link) return true;
    if (x < link) lo = mid + 1; else hi = mid;
  }
  return false;
}

// lattice meet of a label and the candidate {d, nh}: a smaller distance
// replaces, an equal one ORs the mask
__device__ inline unsigned long long meet(unsigned long long l, uint64_t d, uint32_t nh) {
  if (d >= kInfD) return l;
  const uint32_t ld = static_cast<uint32_t>(l >> 32);
  if (d < ld) return (d << 32) | nh;
  if (d == ld) return l | nh;
  return l;
}

// workgroup barrier that first drains this wave's global stores: the repair
// state (and the mask row used as index map) lives in global memory in the
// slot pass, and other waves read it with plain loads after the barrier
__device__ inline void bar() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// visit the live records of node v: ELL slots then the overflow list
template <int K, class F>
__device__ inline void for_records(const uint2* recs, uint32_t v, F&& f) {
  const uint2* slots = recs + static_cast<size_t>(v) * K;
  uint2 r[K];
#pragma unroll
  for (int j = 0; j < K; ++j) r[j] = slots[j];
#pragma unroll
  for (int j = 0; j < K; ++j)
    if (!(r[j].x & (ORH_REC_SKIP | ORH_REC_CONT))) f(r[j], static_cast<uint32_t>(v * K + j));
  if (r[K - 1].x & ORH_REC_CONT) {
    const uint32_t start = r[K - 1].x & ORH_REC_COL_MASK;
    for (uint32_t q = 0; q < r[K - 1].y; ++q) {
      const uint2 o = recs[start + q];
      if (!(o.x & ORH_REC_SKIP)) f(o, start + q);
    }
  }
}

constexpr uint32_t kCopyTile = 256 * 16;  // u32 elements of a row per copy workgroup

// base rows -> request rows; vec: every row is 16-byte aligned (N % 4 == 0
// and aligned buffers), so a thread moves uint4s
__global__ __launch_bounds__(256) void whatif_copy_kernel(RepairArgs a, uint32_t tiles, uint32_t vec) {
  uint32_t r = blockIdx.x / tiles;
  const uint32_t t = blockIdx.x % tiles;
  if (a.share_base) {  // block i copies the i-th queued request's row
    if (r >= a.counters[0]) return;
    r = a.queues[r];
  }
  const size_t N = a.n_nodes;
  const size_t b = a.base_row[r];
  const uint32_t* sd = a.base_dist + b * N;
  const uint32_t* sn = a.base_nh + b * N;
  uint32_t* dd = a.out_dist + r * N;
  uint32_t* dn = a.out_nh + r * N;
  const size_t lo = static_cast<size_t>(t) * kCopyTile, hi = min(lo + kCopyTile, N);
  if (vec) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    for (size_t i = lo / 4 + threadIdx.x; i < hi / 4; i += 256) {
      __builtin_nontemporal_store(reinterpret_cast<const v4*>(sd)[i], reinterpret_cast<v4*>(dd) + i);
      __builtin_nontemporal_store(reinterpret_cast<const v4*>(sn)[i], reinterpret_cast<v4*>(dn) + i);
    }
  } else {
    for (size_t i = lo + threadIdx.x; i < hi; i += 256) {
      dd[i] = sd[i];
      dn[i] = sn[i];
    }
  }
}

// One request: A (the nodes below a tight ignored link, closed under tight
// out-records of transit nodes), boundary labels from predecessors outside
// A, chaotic relaxation inside A, rows written. State at `base` with the
// caps cap_a / cap_e (LDS, or a global slot with whole-graph caps). Returns
// |A|, or ~0u when A or its edge list outgrows the caps. The membership
// bitmap must be all zero on entry; the caller clears it afterwards.
template <int K>
__device__ uint32_t repair_one(const RepairArgs& a, uint32_t r, uint32_t* base, uint32_t cap_a, uint32_t cap_e,
                               uint32_t* s_cnt, uint32_t* s_ecnt, uint32_t* s_ovf, uint32_t* s_flag) {
  const uint32_t N = a.n_nodes;
  const uint32_t tid = threadIdx.x, B = blockDim.x;
  // state: labels u64[cap_a] | boundary labels u64[cap_a] | edges uint2[cap_e] |
  //        edge ranges uint2[cap_a] | node list u32[cap_a] | membership bitmap u32[NB]
  unsigned long long* lab = reinterpret_cast<unsigned long long*>(base);
  unsigned long long* blab = lab + cap_a;
  uint2* edges = reinterpret_cast<uint2*>(blab + cap_a);
  uint2* erange = edges + cap_e;
  uint32_t* alist = reinterpret_cast<uint32_t*>(erange + cap_a);
  uint32_t* bits = alist + cap_a;

  const uint32_t s = a.srcs[r];
  const size_t b = a.base_row[r];
  const uint32_t* bd = a.base_dist + b * N;
  const uint32_t* bn = a.base_nh + b * N;
  uint32_t* od = a.out_dist + static_cast<size_t>(r) * N;
  uint32_t* on = a.out_nh + static_cast<size_t>(r) * N;
  const uint32_t* ign = a.ign + a.ign_ptr[r];
  const uint32_t n_ign = a.ign_ptr[r + 1] - a.ign_ptr[r];
  const bool metric = a.use_link_metric != 0;

  if (tid == 0) {
    *s_cnt = 0u;
    *s_ecnt = 0u;
    *s_ovf = 0u;
  }
  if (tid < 3) s_flag[tid] = 0u;
  bar();

  auto add = [&](uint32_t u) {
    const uint32_t bit = 1u << (u & 31u);
    if (atomicOr(&bits[u >> 5], bit) & bit) return;
    const uint32_t k = atomicAdd(s_cnt, 1u);
    if (k < cap_a) alist[k] = u;
    else *s_ovf = 1u;
  };
  // seeds: heads of tight ignored records whose tail is a transit node
  for (uint32_t c = a.cut_ptr[r] + tid; c < a.cut_ptr[r + 1]; c += B) {
    const uint4 cut = a.cuts[c];  // (tail, head, record of tail -> head, 0)
    const uint2 rec = a.recs[cut.z];
    if (rec.x & ORH_REC_SKIP) continue;  // link down: never on a path
    const uint32_t dx = bd[cut.x];
    if (dx == kInfD || (cut.x != s && a.ovl[cut.x])) continue;
    if (static_cast<uint64_t>(dx) + (metric ? rec.y : 1u) == bd[cut.y]) add(cut.y);
  }
  bar();
  if (*s_cnt == 0u) return 0u;  // nothing below a tight ignored link: the base row stands

  // A: closure under tight out-records of transit nodes, level by level
  uint32_t lo = 0;
  for (;;) {
    const uint32_t hi = min(*s_cnt, cap_a);
    const bool ovf = *s_ovf != 0u;
    bar();  // everyone has read the range before it grows
    if (ovf || lo == hi) break;
    for (uint32_t k = lo + tid; k < hi; k += B) {
      const uint32_t v = alist[k];
      if (a.ovl[v]) continue;  // reached, but no transit (v != s: s is never in A)
      const uint64_t dv = bd[v];
      for_records<K>(a.recs, v, [&](const uint2& rec, uint32_t) {
        const uint32_t u = rec.x & ORH_REC_COL_MASK;
        if (bits[u >> 5] & (1u << (u & 31u))) return;
        if (dv + (metric ? rec.y : 1u) == bd[u]) add(u);
      });
    }
    lo = hi;
    bar();
  }
  const uint32_t n = min(*s_cnt, cap_a);
  if (*s_ovf) return ~0u;
  // the request's mask row doubles as the node -> A index map (rewritten below)
  for (uint32_t k = tid; k < n; k += B) on[alist[k]] = k;
  bar();

  // boundary labels from predecessors outside A; edges from those inside
  auto pred = [&](const uint2& rec, uint32_t q, auto&& inside, auto&& outside) {
    if (n_ign && is_ignored(ign, n_ign, a.link[q])) return;
    const uint32_t p = rec.x & ORH_REC_COL_MASK;
    const uint32_t q2 = a.rev[q];
    const uint2 back = a.recs[q2];  // p -> v: p's metric and p's overload bit
    if (p != s && (back.x & ORH_REC_ROW_OVL)) return;
    const uint32_t w = metric ? back.y : 1u;
    if (bits[p >> 5] & (1u << (p & 31u))) inside(p, w);
    else outside(p, q2, w);
  };
  for (uint32_t k = tid; k < n; k += B) {
    const uint32_t v = alist[k];
    uint32_t cnt = 0;
    unsigned long long bl = kInfLab;
    for_records<K>(a.recs, v, [&](const uint2& rec, uint32_t q) {
      pred(rec, q, [&](uint32_t, uint32_t) { ++cnt; },
           [&](uint32_t p, uint32_t q2, uint32_t w) {
             const uint32_t dp = bd[p];
             if (dp == kInfD) return;
             bl = meet(bl, static_cast<uint64_t>(dp) + w, p == s ? (1u << a.rank_out[q2]) : bn[p]);
           });
    });
    const uint32_t e0 = cnt ? atomicAdd(s_ecnt, cnt) : 0u;
    if (e0 + cnt > cap_e) {
      *s_ovf = 1u;
      cnt = 0;
    }
    uint32_t e = e0;
    if (cnt)
      for_records<K>(a.recs, v, [&](const uint2& rec, uint32_t q) {
        pred(rec, q, [&](uint32_t p, uint32_t w) { edges[e++] = make_uint2(on[p], w); },
             [](uint32_t, uint32_t, uint32_t) {});
      });
    erange[k] = make_uint2(e0, e0 + cnt);
    blab[k] = bl;
    lab[k] = kInfLab;
  }
  bar();
  if (*s_ovf) return ~0u;

  // chaotic relaxation inside A until no label changes (labels only descend
  // in the lattice; a sweep that writes nothing proves the fixpoint)
  for (uint32_t it = 0;; ++it) {
    bool changed = false;
    for (uint32_t k = tid; k < n; k += B) {
      unsigned long long nl = blab[k];
      const uint2 er = erange[k];
      uint32_t e = er.x;
      for (; e + 4 <= er.y; e += 4) {  // four predecessor labels in flight
        uint2 ed[4];
        unsigned long long lj[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) ed[q] = edges[e + q];
#pragma unroll
        for (int q = 0; q < 4; ++q) lj[q] = lab[ed[q].x];
#pragma unroll
        for (int q = 0; q < 4; ++q) nl = meet(nl, (lj[q] >> 32) + ed[q].y, static_cast<uint32_t>(lj[q]));
      }
      for (; e < er.y; ++e) {
        const uint2 ed = edges[e];
        const unsigned long long lj = lab[ed.x];
        nl = meet(nl, (lj >> 32) + ed.y, static_cast<uint32_t>(lj));
      }
      if (nl != lab[k]) {
        lab[k] = nl;
        changed = true;
      }
    }
    const uint32_t par = it % 3u;
    if (changed) s_flag[par] = 1u;
    bar();
    const bool more = s_flag[par] != 0u;
    if (tid == 0) s_flag[(par + 2u) % 3u] = 0u;  // the previous sweep's flag, read before this barrier
    if (!more) break;
  }
  for (uint32_t k = tid; k < n; k += B) {
    const uint32_t v = alist[k];
    const unsigned long long l = lab[k];
    od[v] = static_cast<uint32_t>(l >> 32);
    on[v] = static_cast<uint32_t>(l);
  }
  return n;
}

// seed pass, one thread per request: a request with no tight ignored link
// keeps the copied base row (tier 0); the others join queue 0 (wave-aggregated
// appends: one atomic per wave)
__global__ __launch_bounds__(256) void whatif_seed_kernel(RepairArgs a) {
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  bool hit = false;
  if (r < a.n_req) {
    const uint32_t N = a.n_nodes;
    const uint32_t s = a.srcs[r];
    const uint32_t* bd = a.base_dist + static_cast<size_t>(a.base_row[r]) * N;
    const bool metric = a.use_link_metric != 0;
    for (uint32_t c = a.cut_ptr[r]; c < a.cut_ptr[r + 1] && !hit; ++c) {
      const uint4 cut = a.cuts[c];
      const uint2 rec = a.recs[cut.z];
      if (rec.x & ORH_REC_SKIP) continue;
      const uint32_t dx = bd[cut.x];
      if (dx == kInfD || (cut.x != s && a.ovl[cut.x])) continue;
      hit = static_cast<uint64_t>(dx) + (metric ? rec.y : 1u) == bd[cut.y];
    }
    if (a.info) a.info[r] = kWhatifTierBase;
  }
  const unsigned long long m = __ballot(hit);
  if (!m) return;
  const uint32_t lane = __lane_id();
  const uint32_t leader = static_cast<uint32_t>(__builtin_ctzll(m));
  uint32_t at = 0;
  if (lane == leader) at = atomicAdd(&a.counters[0], static_cast<uint32_t>(__popcll(m)));
  at = __shfl(at, static_cast<int>(leader));
  if (hit) a.queues[at + static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull)))] = r;
}

// tier kTier drains queue q into queue q + 1: LDS state (tiers 1, 2) or one global
// slot per workgroup (tier 3); a request that outgrows the caps moves on to
// the next queue. Every workgroup leaves once its claim passes the queue's
// length (fixed before this launch by the previous kernel).
template <int K, uint32_t kTier>
__global__ __launch_bounds__(kTier == kWhatifTierSmall ? 128 : kTier == kWhatifTierLarge ? 256 : kSlotBlock)
void whatif_repair_kernel(RepairArgs a, uint32_t cap_a, uint32_t cap_e, uint32_t q) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ uint32_t s_cnt, s_ecnt, s_ovf, s_req;
  __shared__ uint32_t s_flag[3];
  constexpr bool kSlot = kTier == kWhatifTierSlot;
  const uint32_t N = a.n_nodes, NB = (N + 31) / 32;
  const uint32_t tid = threadIdx.x, B = blockDim.x;
  uint32_t* base = kSlot ? reinterpret_cast<uint32_t*>(a.slot_mem + blockIdx.x * a.slot_bytes) : lds;
  uint32_t* alist = base + 2 * 2 * cap_a + 2 * cap_e + 2 * cap_a;  // see repair_one's layout
  uint32_t* bits = alist + cap_a;
  for (uint32_t i = tid; i < NB; i += B) bits[i] = 0u;
  const uint32_t len = a.counters[2 * q];
  const uint32_t skip = kSlot ? min(len, a.full_cap) : 0u;  // the full search's share
  if (kSlot && a.info)
    for (uint32_t i = blockIdx.x * B + tid; i < skip; i += gridDim.x * B)
      a.info[a.queues[static_cast<size_t>(q) * a.n_req + i]] = kWhatifTierSearch;
  for (;;) {
    if (tid == 0) {
      const uint32_t i = atomicAdd(&a.counters[2 * q + 1], 1u) + skip;
      s_req = i < len ? a.queues[static_cast<size_t>(q) * a.n_req + i] : ~0u;
    }
    bar();
    const uint32_t r = s_req;
    if (r == ~0u) break;
    const uint32_t n = repair_one<K>(a, r, base, cap_a, cap_e, &s_cnt, &s_ecnt, &s_ovf, s_flag);
    if (tid == 0) {
      if (n != ~0u) {
        if (a.info) a.info[r] = kTier | (n << 3);
        if (kSlot) a.fallback[r] = 0u;
      } else if (!kSlot) {
        const uint32_t j = atomicAdd(&a.counters[2 * (q + 1)], 1u);
        a.queues[static_cast<size_t>(q + 1) * a.n_req + j] = r;
        if (kTier == kWhatifTierLarge) a.fallback[r] = 1u;  // the full search takes it without slots
      }
    }
    // clear the membership bitmap: through the node list when it holds all
    // of A, else whole
    const uint32_t cnt = s_cnt;
    bar();
    if (cnt > cap_a) {
      for (uint32_t i = tid; i < NB; i += B) bits[i] = 0u;
    } else {
      for (uint32_t k = tid; k < cnt; k += B) bits[alist[k] >> 5] = 0u;
    }
    bar();
  }
}

}  // namespace

size_t repair_lds_bytes(uint32_t n_nodes, uint32_t cap_a, uint32_t cap_e) {
  return static_cast<size_t>(cap_a) * (8 + 8 + 8 + 4) + static_cast<size_t>(cap_e) * 8 +
         static_cast<size_t>((n_nodes + 31) / 32) * 4;
}

size_t repair_slot_bytes(uint32_t n_nodes, uint32_t n_recs) {
  return (repair_lds_bytes(n_nodes, n_nodes, n_recs) + 255) & ~static_cast<size_t>(255);
}

namespace {

size_t tier1_lds(const RepairArgs& a, uint32_t* sa, uint32_t* se) {
  *sa = std::min(kSmallA, a.cap_a);
  *se = std::min(kSmallE, a.cap_e);
  return repair_lds_bytes(a.n_nodes, *sa, *se);
}

// queue-draining grids: as many workgroups as the LDS lets share a CU (one
// request each at a time), never more than there are requests
uint32_t tier_grid(const RepairArgs& a, size_t lds_limit, size_t lds, uint32_t per_cu_cap) {
  const uint32_t per_cu = static_cast<uint32_t>(std::min<size_t>(per_cu_cap, std::max<size_t>(1, lds_limit / lds)));
  return std::max<uint32_t>(1u, std::min<uint32_t>(a.n_req, a.n_cu * per_cu));
}

}  // namespace

hipError_t launch_repair_front(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s) {
  if (a.n_req == 0) return hipSuccess;
  if (ell_k != 4 && ell_k != 8) return hipErrorInvalidValue;
  const uint32_t tiles = (a.n_nodes + kCopyTile - 1) / kCopyTile;
  const uint64_t grid = static_cast<uint64_t>(tiles) * a.n_req;
  if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(whatif_seed_kernel, dim3((a.n_req + 255) / 256), dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  const uint32_t vec = (a.n_nodes & 3u) == 0 && al(a.base_dist) && al(a.base_nh) && al(a.out_dist) &&
                       al(a.out_nh);
  hipLaunchKernelGGL(whatif_copy_kernel, dim3(static_cast<uint32_t>(grid)), dim3(256), 0, s, a, tiles, vec);
  return hipGetLastError();
}

hipError_t launch_repair_back(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s) {
  return launch_repair_back_split(a, ell_k, lds_limit, s, s, nullptr);
}

hipError_t launch_repair_back_split(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s,
                                    hipStream_t s3, hipEvent_t mid) {
  if (a.n_req == 0) return hipSuccess;
  if (ell_k != 4 && ell_k != 8) return hipErrorInvalidValue;
  uint32_t sa = 0, se = 0;
  const size_t lds1 = tier1_lds(a, &sa, &se);
  const size_t lds2 = repair_lds_bytes(a.n_nodes, a.cap_a, a.cap_e);
  if (lds1 < lds2) {
    if (ell_k == 8)
      hipLaunchKernelGGL((whatif_repair_kernel<8, kWhatifTierSmall>), dim3(tier_grid(a, lds_limit, lds1, 16)),
                         dim3(128), lds1, s, a, sa, se, 0u);
    else
      hipLaunchKernelGGL((whatif_repair_kernel<4, kWhatifTierSmall>), dim3(tier_grid(a, lds_limit, lds1, 16)),
                         dim3(128), lds1, s, a, sa, se, 0u);
    const hipError_t e1 = hipGetLastError();
    if (e1 != hipSuccess) return e1;
  }
  // without the small tier, tier 2 drains queue 0 itself
  const uint32_t q2 = lds1 < lds2 ? 1u : 0u;
  // skip_large: the slot tier (and the full searches) take tier 1's overflow
  const bool no_t2 = a.skip_large && lds1 < lds2;
  hipError_t e = hipSuccess;
  if (!no_t2) {
    if (ell_k == 8)
      hipLaunchKernelGGL((whatif_repair_kernel<8, kWhatifTierLarge>), dim3(tier_grid(a, lds_limit, lds2, 8)),
                         dim3(256), lds2, s, a, a.cap_a, a.cap_e, q2);
    else
      hipLaunchKernelGGL((whatif_repair_kernel<4, kWhatifTierLarge>), dim3(tier_grid(a, lds_limit, lds2, 8)),
                         dim3(256), lds2, s, a, a.cap_a, a.cap_e, q2);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (a.n_slots == 0) return e;
  const uint32_t qs = no_t2 ? q2 : q2 + 1u;
  if (s3 != s) {
    if ((e = hipEventRecord(mid, s)) != hipSuccess || (e = hipStreamWaitEvent(s3, mid, 0)) != hipSuccess) return e;
  }
  if (ell_k == 8)
    hipLaunchKernelGGL((whatif_repair_kernel<8, kWhatifTierSlot>), dim3(a.n_slots), dim3(kSlotBlock), 0, s3, a,
                       a.n_nodes, a.n_recs, qs);
  else
    hipLaunchKernelGGL((whatif_repair_kernel<4, kWhatifTierSlot>), dim3(a.n_slots), dim3(kSlotBlock), 0, s3, a,
                       a.n_nodes, a.n_recs, qs);
  return hipGetLastError();
}

uint32_t repair_slot_queue(const RepairArgs& a) {
  uint32_t sa = 0, se = 0;
  const bool t1 = tier1_lds(a, &sa, &se) < repair_lds_bytes(a.n_nodes, a.cap_a, a.cap_e);
  return t1 ? (a.skip_large ? 1u : 2u) : 1u;
}

hipError_t launch_repair(const RepairArgs& a, uint32_t ell_k, size_t lds_limit, hipStream_t s) {
  hipError_t e = launch_repair_front(a, ell_k, lds_limit, s);
  return e != hipSuccess ? e : launch_repair_back(a, ell_k, lds_limit, s);
}

namespace {

// ---- row digests (verification of whole batches) ---------------------------
// digest(row) = sum over v of mix(v, dist[v], nh[v][0..words)) mod 2^64: an
// order-free sum of a strong per-node hash, so equal rows give equal digests
// however they were produced, and one digest per row checks a batch whose rows
// do not fit the host (C4: 262,144 rows of 50,000 nodes). tests/helpers.py
// row_digest restates it in numpy.
__device__ inline uint64_t fmix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) row_digest_kernel(const uint32_t* __restrict__ dist,
                                                         const uint32_t* __restrict__ nh, uint32_t words,
                                                         uint32_t n, unsigned long long* __restrict__ out) {
  const size_t row = blockIdx.x;
  const uint32_t* d = dist + row * n;
  const uint32_t* m = nh + row * static_cast<size_t>(n) * words;
  uint64_t acc = 0;
  for (uint32_t v = threadIdx.x; v < n; v += blockDim.x) {
    uint64_t h = fmix64(static_cast<uint64_t>(v) * 0x9E3779B97F4A7C15ull + d[v]);
    for (uint32_t k = 0; k < words; ++k)
      h = fmix64(h ^ (static_cast<uint64_t>(m[static_cast<size_t>(v) * words + k]) +
                      static_cast<uint64_t>(k) * 0xC2B2AE3D27D4EB4Full));
    acc += h;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = static_cast<uint32_t>(__shfl_xor(static_cast<int>(acc), o));
    const uint32_t hi = static_cast<uint32_t>(__shfl_xor(static_cast<int>(acc >> 32), o));
    acc += (static_cast<uint64_t>(hi) << 32) | lo;
  }
  __shared__ uint64_t part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[row] = part[0] + part[1] + part[2] + part[3];
}

}  // namespace

hipError_t launch_row_digest(const uint32_t* dist, const uint32_t* nh, uint32_t words, uint32_t n,
                             uint32_t rows, uint64_t* out, hipStream_t s) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(row_digest_kernel, dim3(rows), dim3(256), 0, s, dist, nh, words, n,
                     reinterpret_cast<unsigned long long*>(out));
  return hipGetLastError();
}

}  // namespace orh
