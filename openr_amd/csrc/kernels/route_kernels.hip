// Per-prefix route selection for gfx950 (MI355X): the per-prefix half of
// SpfSolver::SpfSolverImpl::createRouteForPrefix (openr/decision/Decision.cpp
// :445-613) up to the first-hop set of the route, over the device prefix
// mirror (orh_prefix_set) and `me`'s SPF rows of every area.
//
// One thread per prefix; a prefix's advertisements are a contiguous run of
// 20-byte records, so consecutive threads read consecutive runs. The work per
// prefix is a handful of gathers into `me`'s distance / first-hop rows
// (L2-resident: 40 KB + 40 KB per 10k-node area), so the kernel streams the
// advertisement pool once and is HBM-bound (B_sel = 20 A + 8 A + 16 + 4 W
// bytes per prefix: records, dist + mask gathers, header + outputs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "route_kernels.h"

namespace orh {

namespace {

constexpr uint32_t kSelBlock = 256;
constexpr uint32_t kInfD = 0xFFFFFFFFu;
constexpr uint32_t kMaxAdvDevice = 64;  // longer advertisement lists take the host path

__device__ inline uint64_t bit64(uint32_t i) { return 1ull << i; }

// node id of a name in area b, or ORH_NO_NODE
__device__ inline uint32_t node_of(const SelArea& A, uint32_t name, uint32_t n_names) {
  return name < n_names ? A.name_node[name] : ORH_NO_NODE;
}

// -distance as the reference's int32 tuple element (Util.h:491-526)
__device__ inline int32_t neg(int32_t d) { return static_cast<int32_t>(0u - static_cast<uint32_t>(d)); }

__device__ inline bool key_less(int32_t pa, int32_t sa, int32_t da, int32_t pb, int32_t sb,
                                int32_t db) {
  if (pa != pb) return pa < pb;
  if (sa != sb) return sa < sb;
  return da < db;
}

}  // namespace

__global__ __launch_bounds__(kSelBlock) void route_select_kernel(RouteSelectArgs a) {
  const uint32_t p = a.pid_lo + blockIdx.x * kSelBlock + threadIdx.x;
  if (p >= a.n_prefix) return;
  const uint2 h = a.hdr[p];
  const uint32_t off = h.x, cnt = h.y & 0xFFFFu, pflags = h.y >> 16;
  uint32_t status = ORH_SEL_NONE, metric = kInfD, best = 0;
  const uint32_t TW = a.total_words;
  uint32_t* mask = a.mask + static_cast<size_t>(p) * TW;

  auto finish = [&]() {
    a.status[p] = static_cast<uint8_t>(status);
    a.metric[p] = metric;
    a.best[p] = best;
    if (status != ORH_SEL_ROUTE)
      for (uint32_t w = 0; w < TW; ++w) mask[w] = 0u;
  };
  if (cnt == 0) {  // withdrawn: no entry in PrefixState
    finish();
    return;
  }
  if (cnt > kMaxAdvDevice) {
    status = ORH_SEL_HOST;
    finish();
    return;
  }
  const orh_adv* adv = a.adv + off;

  // (1) advertisers reachable in their own area (Decision.cpp:468-480); an
  // advertiser of an area the solver does not have is kept (and later makes
  // the reference throw), one named `me` is always in me's SpfResult
  uint64_t R = 0;
  bool host = false, bgp = false;
  for (uint32_t i = 0; i < cnt; ++i) {
    const orh_adv r = adv[i];
    const uint32_t ar = r.meta & ORH_ADV_AREA_MASK;
    bool reach;
    if (ar >= a.n_areas || !a.areas[ar].present) {
      reach = true;
      host = true;
    } else if (r.name == a.me_name) {
      reach = true;
      host = true;  // self-advertised: prepend-label rules stay on the host
    } else {
      const SelArea A = a.areas[ar];
      const uint32_t v = A.dist ? node_of(A, r.name, a.n_names) : ORH_NO_NODE;
      reach = v != ORH_NO_NODE && A.dist[v] != kInfD;
    }
    if (!reach) continue;
    R |= bit64(i);
    bgp |= (r.meta & ORH_ADV_BGP) != 0;
  }
  if (!R || ((pflags & ORH_PFX_V4) && !(a.flags & ORH_SELECT_V4))) {  // :483-499
    finish();
    return;
  }
  if (host || bgp) {  // BGP metric vectors (:501-546, :864-902) stay on the host
    status = ORH_SEL_HOST;
    finish();
    return;
  }

  // (2) best-route selection (selectBestPrefixMetrics) or every advertiser
  uint64_t sel = R;
  if (a.flags & ORH_SELECT_BEST_ROUTE) {
    int32_t bp = 0, bs = 0, bd = 0;
    bool any = false;
    for (uint64_t q = R; q; q &= q - 1) {
      const orh_adv r = adv[__builtin_ctzll(q)];
      const int32_t nd = neg(r.distance);
      if (!any || key_less(bp, bs, bd, r.path_pref, r.source_pref, nd)) {
        bp = r.path_pref;
        bs = r.source_pref;
        bd = nd;
        any = true;
      }
    }
    sel = 0;
    for (uint64_t q = R; q; q &= q - 1) {
      const uint32_t i = __builtin_ctzll(q);
      const orh_adv r = adv[i];
      if (r.path_pref == bp && r.source_pref == bs && neg(r.distance) == bd) sel |= bit64(i);
    }
  }
  // bestNodeArea = smallest (node, area) of the selected set (std::set
  // order; `me` is never in it on this path)
  {
    uint32_t bn = 0xFFFFFFFFu, ba = 0xFFFFFFFFu;
    for (uint64_t q = sel; q; q &= q - 1) {
      const uint32_t i = __builtin_ctzll(q);
      const orh_adv r = adv[i];
      const uint32_t rn = r.name < a.n_names ? a.name_rank[r.name] : 0xFFFFFFFFu;
      const uint32_t ra = a.area_rank[r.meta & ORH_ADV_AREA_MASK];
      if (rn < bn || (rn == bn && ra < ba)) {
        bn = rn;
        ba = ra;
        best = i;
      }
    }
  }
  // (3) drained advertisers leave the set unless that empties it; the best
  // node area is kept as it was (maybeFilterDrainedNodes, :840-862)
  uint64_t S = sel;
  {
    uint64_t undrained = 0;
    for (uint64_t q = sel; q; q &= q - 1) {
      const uint32_t i = __builtin_ctzll(q);
      const orh_adv r = adv[i];
      const SelArea A = a.areas[r.meta & ORH_ADV_AREA_MASK];
      const uint32_t v = node_of(A, r.name, a.n_names);
      if (!A.ovl[v]) undrained |= bit64(i);
    }
    if (undrained) S = undrained;
  }
  // (4) forwarding type / algorithm = min over the selected entries
  // (Util.cpp:452-480); only (IP, SP_ECMP) without minNexthop is device work
  {
    bool ip = false, sp = false, minnh = false;
    for (uint64_t q = S; q; q &= q - 1) {
      const uint32_t m = adv[__builtin_ctzll(q)].meta;
      ip |= !(m & ORH_ADV_SR_MPLS);
      sp |= !(m & ORH_ADV_KSP2);
      minnh |= (m & ORH_ADV_MIN_NEXTHOP) != 0;
    }
    if (!ip || !sp || minnh) {
      status = ORH_SEL_HOST;
      finish();
      return;
    }
  }
  // (5) getNextHopsWithMetric (:1182-1228): per area the min over every
  // selected name (the area of the advertisement is ignored, :1159), the
  // smallest area minimum wins and equal areas union their first hops
  uint32_t shortest = kInfD;
  for (uint32_t b = 0; b < a.n_areas; ++b) {
    const SelArea A = a.areas[b];
    if (!A.dist) continue;
    for (uint64_t q = S; q; q &= q - 1) {
      const uint32_t v = node_of(A, adv[__builtin_ctzll(q)].name, a.n_names);
      if (v != ORH_NO_NODE) shortest = min(shortest, A.dist[v]);
    }
  }
  bool any = false;
  for (uint32_t b = 0; b < a.n_areas; ++b) {
    const SelArea A = a.areas[b];
    uint32_t* mb = mask + A.word_off;
    for (uint32_t w = 0; w < A.words; ++w) {
      uint32_t m = 0;
      if (A.dist && shortest != kInfD) {
        for (uint64_t q = S; q; q &= q - 1) {
          const uint32_t v = node_of(A, adv[__builtin_ctzll(q)].name, a.n_names);
          if (v != ORH_NO_NODE && A.dist[v] == shortest)
            m |= A.nh[static_cast<size_t>(v) * A.words + w];
        }
      }
      mb[w] = m;
      any |= m != 0;
    }
  }
  if (any) {
    status = ORH_SEL_ROUTE;
    metric = shortest;
  }
  a.status[p] = static_cast<uint8_t>(status);
  a.metric[p] = metric;
  a.best[p] = best;
  if (!any)
    for (uint32_t w = 0; w < TW; ++w) mask[w] = 0u;
}

__global__ __launch_bounds__(kSelBlock) void scatter_hdr_kernel(uint2* hdr, const uint32_t* ids,
                                                               const uint2* vals, uint32_t n) {
  const uint32_t i = blockIdx.x * kSelBlock + threadIdx.x;
  if (i < n) hdr[ids[i]] = vals[i];
}

// The device half of DecisionRouteDb::calculateUpdate (Decision.cpp:108-143)
// for a rebuild after topology changes: a route is a function of its
// selection record (status, shortest metric, best advertisement, first-hop
// mask) once the nexthop templates, the prefix entries and the policy are
// unchanged, so only prefixes whose record differs from the previous build's
// need a route built and compared on the host. One thread per prefix; the
// changed records are appended packed (one atomic per wave).
__global__ __launch_bounds__(kSelBlock) void route_diff_kernel(RouteDiffArgs a) {
  const uint32_t p = blockIdx.x * kSelBlock + threadIdx.x;
  bool diff = false;
  if (p < a.n_prefix) {
    if (p >= a.prev_n) {
      diff = true;
    } else {
      diff = a.status[p] != a.p_status[p];
      if (!diff && a.status[p] == ORH_SEL_ROUTE) {
        diff = a.metric[p] != a.p_metric[p] || a.best[p] != a.p_best[p];
        for (uint32_t k = 0; k < a.words && !diff; ++k)
          diff = a.mask[static_cast<size_t>(p) * a.words + k] != a.p_mask[static_cast<size_t>(p) * a.words + k];
      }
    }
  }
  const unsigned long long m = __ballot(diff);
  if (!m) return;
  const uint32_t lane = __lane_id();
  const uint32_t leader = static_cast<uint32_t>(__builtin_ctzll(m));
  uint32_t at = 0;
  if (lane == leader) at = atomicAdd(a.count, static_cast<uint32_t>(__popcll(m)));
  at = __shfl(at, static_cast<int>(leader));
  if (!diff) return;
  const size_t rec = 4 + a.words;
  uint32_t* o = a.out + (at + static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull)))) * rec;
  o[0] = p;
  o[1] = a.status[p];
  o[2] = a.metric[p];
  o[3] = a.best[p];
  for (uint32_t k = 0; k < a.words; ++k) o[4 + k] = a.mask[static_cast<size_t>(p) * a.words + k];
}

// RibPolicy::applyPolicy (RibPolicy.cpp:229-247) over a selection, one thread
// per prefix: the statement that applies to the route, if any (see
// orh_route_policy for the reduction of set_weight to keep[s] masks). The
// match reads one advertisement record (the best one's tag set id), a tag-set
// table entry and, when a statement has a prefix matcher, a binary search over
// the named prefix ids; the tables are a few KB and stay in L2, so the kernel
// streams the selection records (status, best, mask: 5 + 4 W bytes per prefix)
// plus one advertisement gather and writes one byte.
__global__ __launch_bounds__(kSelBlock) void route_policy_kernel(RoutePolicyArgs a) {
  const uint32_t p = a.pid_lo + blockIdx.x * kSelBlock + threadIdx.x;
  if (p >= a.n_prefix) return;
  uint32_t res = ORH_POL_NONE, inv = 0;
  if (a.status[p] == ORH_SEL_ROUTE) {
    const uint32_t meta = a.adv[a.hdr[p].x + a.best[p]].meta;
    const uint32_t ts = meta >> ORH_ADV_TAGSET_SHIFT;
    const uint32_t tm = ts < a.n_tagsets ? a.tagset_stmts[ts] : 0u;
    uint32_t pm = 0;
    if (a.n_pfx) {  // lower bound of p in the named prefix ids
      uint32_t lo = 0, hi = a.n_pfx;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.pfx_id[mid] < p) lo = mid + 1; else hi = mid;
      }
      if (lo < a.n_pfx && a.pfx_id[lo] == p) pm = a.pfx_stmts[lo];
    }
    const uint32_t all = a.n_stmts >= 32 ? ~0u : ((1u << a.n_stmts) - 1u);
    // RibPolicyStatement::match (:73-105): every non-empty matcher matches and
    // at least one is non-empty
    uint32_t match = all & (a.stmt_tags | a.stmt_pfx) & (~a.stmt_tags | tm) & (~a.stmt_pfx | pm);
    if (ts == ORH_ADV_TAGSET_OVF && (all & a.stmt_tags)) {
      res = ORH_POL_HOST;  // the tag set has no id: the host matches it
      match = 0;
    }
    const uint32_t* m = a.mask + static_cast<size_t>(p) * a.words;
    for (; match; match &= match - 1) {
      const uint32_t s = static_cast<uint32_t>(__builtin_ctz(match));
      const uint32_t* k = a.keep + static_cast<size_t>(s) * a.words;
      uint32_t any = 0;
      for (uint32_t w = 0; w < a.words; ++w) any |= m[w] & k[w];
      if (any) {  // applyAction (:108-158): the weights apply
        res = s;
        break;
      }
      ++inv;  // every nexthop weighted 0: kept unchanged, counted
    }
  }
  a.out[p] = static_cast<uint8_t>(res);
  if (inv) atomicAdd(a.invalidated, inv);
}

hipError_t launch_route_policy(const RoutePolicyArgs& a, hipStream_t s) {
  if (a.n_prefix <= a.pid_lo) return hipSuccess;
  hipLaunchKernelGGL(route_policy_kernel, dim3((a.n_prefix - a.pid_lo + kSelBlock - 1) / kSelBlock),
                     dim3(kSelBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_route_diff(const RouteDiffArgs& a, hipStream_t s) {
  if (a.n_prefix == 0) return hipSuccess;
  hipLaunchKernelGGL(route_diff_kernel, dim3((a.n_prefix + kSelBlock - 1) / kSelBlock), dim3(kSelBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_route_select(const RouteSelectArgs& a, hipStream_t s) {
  if (a.n_prefix <= a.pid_lo) return hipSuccess;
  const uint32_t grid = (a.n_prefix - a.pid_lo + kSelBlock - 1) / kSelBlock;
  hipLaunchKernelGGL(route_select_kernel, dim3(grid), dim3(kSelBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_scatter_hdr(uint2* hdr, const uint32_t* ids, const uint2* vals, uint32_t n,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_hdr_kernel, dim3((n + kSelBlock - 1) / kSelBlock), dim3(kSelBlock), 0,
                     s, hdr, ids, vals, n);
  return hipGetLastError();
}

}  // namespace orh
