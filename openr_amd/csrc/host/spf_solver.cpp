// Drop-in SpfSolver / PrefixState over device SPF rows (see spf_solver.h).
#include "spf_solver.h"

#include "parallel.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <ctime>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <list>
#include <stdexcept>
#include <tuple>
#include <unordered_set>

namespace openr_amd {

namespace {

// prefixes / adjacency databases below which the route build stays on the
// calling thread (the pool's hand-off costs more than it saves)
constexpr size_t kParallelMin = 2048;

// the phase sink of this thread's RoutePhaseCapture (null: none)
thread_local std::vector<std::pair<const char*, double>>* tlPhases = nullptr;

// phase times of buildRouteDb: on stderr with ORH_ROUTE_PROF=1, and into the
// calling thread's RoutePhaseCapture when one is open
struct RouteProf {
  bool on = std::getenv("ORH_ROUTE_PROF") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on && !tlPhases) return;
    const auto now = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(now - t).count();
    if (tlPhases) tlPhases->emplace_back(what, ms);
    if (on) std::fprintf(stderr, "route-prof %-16s %8.3f ms\n", what, ms);
    t = now;
  }
};

}  // namespace

RoutePhaseCapture::RoutePhaseCapture() : prev_(tlPhases) { tlPhases = &phases; }
RoutePhaseCapture::~RoutePhaseCapture() { tlPhases = prev_; }

namespace {

MplsAction mpls(int32_t code, std::optional<int32_t> swap = std::nullopt,
                std::optional<std::vector<int32_t>> push = std::nullopt) {
  // createMplsAction + checkMplsAction (Util.cpp:482-512, :793-803)
  if (code == kPush && (!push || push->empty())) throw std::logic_error("PUSH without labels");
  if (code == kSwap && (!swap || !isMplsLabelValid(*swap))) throw std::logic_error("bad SWAP");
  if (push)
    for (int32_t l : *push)
      if (!isMplsLabelValid(l)) throw std::logic_error("bad PUSH label");
  return MplsAction{code, swap, std::move(push)};
}

NextHopThrift nextHop(const BinaryAddress& addr, std::optional<std::string> ifName,
                      int32_t metric, std::optional<MplsAction> action,
                      std::optional<std::string> area, std::optional<std::string> nbr) {
  NextHopThrift nh;  // createNextHop (Util.cpp:775-789): metric is int32
  nh.address.addr = addr.addr;
  nh.address.ifName = std::move(ifName);
  nh.metric = metric;
  nh.mplsAction = std::move(action);
  nh.area = std::move(area);
  nh.neighborNodeName = std::move(nbr);
  return nh;
}

// SpfResult::count(name) on a device row
bool rowHas(const LinkState& ls, const SpfRow& row, const std::string& name) {
  if (name == row.srcName) return true;
  auto id = ls.nodeId(name);
  return id && row.reachable(*id);
}

std::optional<Metric> rowMetric(const LinkState& ls, const SpfRow& row, const std::string& name) {
  if (name == row.srcName) return 0;
  auto id = ls.nodeId(name);
  if (!id || !row.reachable(*id)) return std::nullopt;
  return row.metric(*id);
}

bool maskHas(const SpfRow& row, const std::vector<uint32_t>& mask, uint32_t nbr) {
  auto it = std::lower_bound(row.nbrs.begin(), row.nbrs.end(), nbr);
  if (it == row.nbrs.end() || *it != nbr) return false;
  const size_t k = static_cast<size_t>(it - row.nbrs.begin());
  return (mask[k >> 5] >> (k & 31)) & 1u;
}

enum class Cmp { kWinner, kTieWinner, kTie, kTieLooser, kLooser, kError };

Cmp invert(Cmp c) {
  switch (c) {
    case Cmp::kWinner: return Cmp::kLooser;
    case Cmp::kTieWinner: return Cmp::kTieLooser;
    case Cmp::kTie: return Cmp::kTie;
    case Cmp::kTieLooser: return Cmp::kTieWinner;
    case Cmp::kLooser: return Cmp::kWinner;
    default: return Cmp::kError;
  }
}
bool decisive(Cmp c) { return c == Cmp::kWinner || c == Cmp::kLooser || c == Cmp::kError; }
Cmp loner(const MetricEntity& e) {
  if (e.op == 1) return e.isBestPathTieBreaker ? Cmp::kTieWinner : Cmp::kWinner;
  if (e.op == 2) return e.isBestPathTieBreaker ? Cmp::kTieLooser : Cmp::kLooser;
  return Cmp::kTie;
}

// MetricVectorUtils::compareMetricVectors (Util.cpp:1044-1094)
Cmp compareMv(MetricVector l, MetricVector r) {
  if (l.version != r.version) return Cmp::kError;
  auto prio = [](const MetricEntity& a, const MetricEntity& b) { return a.priority > b.priority; };
  if (!std::is_sorted(l.metrics.begin(), l.metrics.end(), prio))
    std::sort(l.metrics.begin(), l.metrics.end(), prio);
  if (!std::is_sorted(r.metrics.begin(), r.metrics.end(), prio))
    std::sort(r.metrics.begin(), r.metrics.end(), prio);
  Cmp res = Cmp::kTie;
  auto upd = [&](Cmp u) {
    if (decisive(u) || res == Cmp::kTie) res = u;
  };
  size_t i = 0, j = 0;
  while (!decisive(res) && i < l.metrics.size() && j < r.metrics.size()) {
    const auto& a = l.metrics[i];
    const auto& b = r.metrics[j];
    if (a.type == b.type) {
      if (a.isBestPathTieBreaker != b.isBestPathTieBreaker) {
        upd(Cmp::kError);
      } else if (a.metric.size() != b.metric.size()) {
        upd(Cmp::kError);
      } else {
        Cmp c = Cmp::kTie;
        for (size_t k = 0; k < a.metric.size(); ++k) {
          if (a.metric[k] != b.metric[k]) {
            const bool win = a.metric[k] > b.metric[k];
            c = a.isBestPathTieBreaker ? (win ? Cmp::kTieWinner : Cmp::kTieLooser)
                                       : (win ? Cmp::kWinner : Cmp::kLooser);
            break;
          }
        }
        upd(c);
      }
      ++i;
      ++j;
    } else if (a.priority > b.priority) {
      upd(loner(a));
      ++i;
    } else if (a.priority < b.priority) {
      upd(invert(loner(b)));
      ++j;
    } else {
      upd(Cmp::kError);
    }
  }
  while (!decisive(res) && i < l.metrics.size()) upd(loner(l.metrics[i++]));
  while (!decisive(res) && j < r.metrics.size()) upd(invert(loner(r.metrics[j++])));
  return res;
}

// a selection output in one device block: status [n, padded to 4] | metric
// [n] | best [n] | mask [n][words]
orh_select_out selOut(uint8_t* base, uint32_t np, uint32_t words) {
  const size_t n4 = (static_cast<size_t>(np) + 3) & ~static_cast<size_t>(3);
  orh_select_out o{};
  o.d_status = base;
  o.d_metric = reinterpret_cast<uint32_t*>(base + n4);
  o.d_best = o.d_metric + np;
  o.d_mask = o.d_best + np;
  o.total_words = words;
  return o;
}

// no MPLS action on a template nexthop (unicast SP_ECMP routes)
const auto noAction = [](const NextHopThrift&) -> std::optional<MplsAction> { return std::nullopt; };

}  // namespace

// ---- SpfSolver ----------------------------------------------------------------
SpfSolver::SpfSolver(const std::string& me, bool enableV4, bool enableOrderedFib, bool bgpDryRun,
                     bool enableBestRouteSelection)
    : myNodeName_(me),
      enableV4_(enableV4),
      enableOrderedFib_(enableOrderedFib),
      bgpDryRun_(bgpDryRun),
      enableBestRouteSelection_(enableBestRouteSelection) {}

void SpfSolver::setPrefixShard(uint32_t rank, uint32_t world) {
  if (world == 0 || rank >= world) throw std::invalid_argument("setPrefixShard: bad rank / world");
  shardRank_ = rank;
  shardWorld_ = world;
}

SpfSolver::~SpfSolver() {
  for (auto& w : areaWork_) {
    if (w.dNameNode) orh_device_free(selCtx_, w.dNameNode);
    if (w.dRow) orh_device_free(selCtx_, w.dRow);
  }
  if (dSel_) orh_device_free(selCtx_, dSel_);
  if (dSelPrev_) orh_device_free(selCtx_, dSelPrev_);
  if (dDiff_) orh_device_free(selCtx_, dDiff_);
  if (dPolOut_) orh_device_free(selCtx_, dPolOut_);
}

void SpfSolver::updateStaticUnicastRoutes(
    const std::vector<std::pair<Cidr, std::vector<NextHopThrift>>>& upd,
    const std::vector<Cidr>& del) {
  for (const auto& [p, nhs] : upd) staticUnicastRoutes_[p] = nhs;
  for (const auto& p : del) staticUnicastRoutes_.erase(p);
  ++staticEpoch_;
}

void SpfSolver::updateStaticMplsRoutes(
    const std::vector<std::pair<int32_t, std::vector<NextHopThrift>>>& upd,
    const std::vector<int32_t>& del) {
  ++staticEpoch_;
  for (const auto& [l, nhs] : upd) staticMplsRoutes_[l] = nhs;
  for (int32_t l : del) staticMplsRoutes_.erase(l);
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefixOrGetStaticRoute(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps, const Cidr& prefix) {
  if (auto r = createRouteForPrefix(me, als, ps, prefix)) return r;
  auto it = staticUnicastRoutes_.find(prefix);
  if (it == staticUnicastRoutes_.end()) return std::nullopt;
  RibUnicastEntry e;
  e.prefix = prefix;
  e.nexthops.insert(it->second.begin(), it->second.end());
  return e;
}

std::vector<std::optional<RibUnicastEntry>> SpfSolver::createRoutesForPrefixes(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
    const std::vector<Cidr>& prefixes) {
  std::vector<std::optional<RibUnicastEntry>> out(prefixes.size());
  // KSP2 prefixes may trace paths lazily (memo writes): one prefix at a time
  const bool hasKsp = ps.ksp2Entries() > 0;
  bool dev = false;
  auto& pool = WorkerPool::instance();
  const bool parallel = !hasKsp && prefixes.size() >= 64 && pool.size() > 1;
  // the memoized rows of `me` are filled here, on this thread: the pool's
  // workers below only read them (a cold getSpfRow flushes the mirror and
  // inserts into the memo, which is not synchronised)
  if (parallel || (!hasKsp && shardWorld_ == 1 && prefixes.size() >= 64))
    for (const auto& [_, ls] : als) ls.getSpfRow(me);
  if (!hasKsp && shardWorld_ == 1 && prefixes.size() >= 64) dev = selectOnDevice(me, als, ps);
  // routes built without a selection pass no longer match the snapshot a
  // later buildRouteDelta would compare with
  if (!dev) havePrev_ = false;
  auto staticRoute = [&](const Cidr& p) -> std::optional<RibUnicastEntry> {
    auto it = staticUnicastRoutes_.find(p);
    if (it == staticUnicastRoutes_.end()) return std::nullopt;
    RibUnicastEntry e;
    e.prefix = p;
    e.nexthops.insert(it->second.begin(), it->second.end());
    return e;
  };
  auto one = [&](size_t i) {
    const Cidr& p = prefixes[i];
    if (!dev) {
      out[i] = createRouteForPrefixOrGetStaticRoute(me, als, ps, p);
      return;
    }
    if (auto pid = ps.pidOf(p); pid && ps.prefixLive(*pid)) {
      if (selStatus_[*pid] == ORH_SEL_ROUTE) {
        out[i] = materialize(*pid, ps);
        return;
      }
      if (selStatus_[*pid] == ORH_SEL_HOST) {
        if (auto r = createRouteForPrefix(me, als, ps, p)) {
          out[i] = std::move(r);
          return;
        }
      }
    }
    out[i] = staticRoute(p);
  };
  if (parallel) {
    pool.parallelFor(prefixes.size(), [&](size_t, size_t b, size_t e) {
      for (size_t i = b; i < e; ++i) one(i);
    });
  } else {
    for (size_t i = 0; i < prefixes.size(); ++i) one(i);
  }
  return out;
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefix(const std::string& me,
                                                               const AreaLinkStates& als,
                                                               const PrefixState& ps,
                                                               const Cidr& prefix) {
  // Decision.cpp:445-613
  auto search = ps.prefixes().find(prefix);
  if (search == ps.prefixes().end()) return std::nullopt;
  // advertisers unreachable in their own area are dropped (:468-480); the
  // entries are copied only when one is
  const PrefixEntries* ep = &search->second;
  PrefixEntries kept;
  for (const auto& [area, ls] : als) {
    const SpfRow& row = ls.getSpfRow(me);
    for (auto it = ep->begin(); it != ep->end();) {
      if (area != it->first.second || rowHas(ls, row, it->first.first)) {
        ++it;
      } else if (ep != &kept) {
        kept = *ep;
        ep = &kept;
        it = kept.begin();  // restart on the copy
      } else {
        it = kept.erase(it);
      }
    }
  }
  const PrefixEntries& entries = *ep;
  if (entries.empty()) return std::nullopt;
  if (prefix.first.size() == 4 && !enableV4_) return std::nullopt;

  bool hasBgp = false, hasNonBgp = false, missingMv = false, selfPrepend = true;
  for (const auto& [na, e] : entries) {
    const bool bgp = e->type == kPrefixTypeBgp;
    hasBgp |= bgp;
    hasNonBgp |= !bgp;
    if (na.first == me) selfPrepend &= e->prependLabel.has_value();
    if (bgp && !e->mv) missingMv = true;
  }
  if (hasBgp && ((hasNonBgp && !enableBestRouteSelection_) || missingMv)) return std::nullopt;

  const auto best = selectBestRoutes(me, entries, hasBgp, als);
  if (!best.success || best.allNodeAreas.empty()) return std::nullopt;
  if (best.hasNode(me) && !selfPrepend) return std::nullopt;

  // getPrefixForwardingTypeAndAlgorithm (Util.cpp:452-480)
  int32_t ft = kFwdSrMpls, fa = kAlgoKsp2EdEcmp;
  for (const auto& [na, e] : entries) {
    if (!best.allNodeAreas.count(na)) continue;
    ft = std::min(ft, e->forwardingType);
    fa = std::min(fa, e->forwardingAlgorithm);
    if (ft == kFwdIp && fa == kAlgoSpEcmp) break;
  }
  if (kspPlan_) {
    // planning pass of buildRouteDb: record the (me, node) pairs whose
    // k = 2 paths selectBestPathsKsp2 will ask for, build nothing
    if (fa == kAlgoKsp2EdEcmp && ft == kFwdSrMpls)
      for (const auto& [area, ls] : als)
        for (const auto& [node, bestArea] : best.allNodeAreas)
          if (area == bestArea) (*kspPlan_)[&ls].emplace_back(me, node);
    return std::nullopt;
  }
  if (fa == kAlgoSpEcmp) return selectBestPathsSpf(me, prefix, best, entries, hasBgp, ft, als);
  if (fa == kAlgoKsp2EdEcmp) return selectBestPathsKsp2(me, prefix, best, entries, hasBgp, ft, als);
  return std::nullopt;
}

BestRouteSelectionResult SpfSolver::filterDrained(BestRouteSelectionResult&& r,
                                                  const AreaLinkStates& als) const {
  // maybeFilterDrainedNodes, Decision.cpp:840-862
  bool anyDrained = false;
  for (const auto& na : r.allNodeAreas) anyDrained |= als.at(na.second).isNodeOverloaded(na.first);
  if (!anyDrained) return std::move(r);
  BestRouteSelectionResult f = r;
  for (auto it = f.allNodeAreas.begin(); it != f.allNodeAreas.end();) {
    if (als.at(it->second).isNodeOverloaded(it->first)) {
      it = f.allNodeAreas.erase(it);
    } else {
      ++it;
    }
  }
  if (!f.allNodeAreas.empty() && f.bestNodeArea != r.bestNodeArea)
    f.bestNodeArea = *f.allNodeAreas.begin();
  return f.allNodeAreas.empty() ? std::move(r) : std::move(f);
}

BestRouteSelectionResult SpfSolver::selectBestRoutes(const std::string& me,
                                                     const PrefixEntries& entries, bool isBgp,
                                                     const AreaLinkStates& als) const {
  BestRouteSelectionResult r;  // Decision.cpp:794-822
  if (enableBestRouteSelection_) {
    // selectBestPrefixMetrics (Util.h:491-526): max (path_pref, source_pref, -distance)
    std::tuple<int32_t, int32_t, int32_t> best{std::numeric_limits<int32_t>::min(),
                                               std::numeric_limits<int32_t>::min(),
                                               std::numeric_limits<int32_t>::min()};
    for (const auto& [na, e] : entries) {
      std::tuple<int32_t, int32_t, int32_t> t{
          e->pathPreference, e->sourcePreference,
          static_cast<int32_t>(0u - static_cast<uint32_t>(e->distance))};
      if (t < best) continue;
      if (t > best) {
        best = t;
        r.allNodeAreas.clear();
      }
      r.allNodeAreas.insert(na);
    }
    r.bestNodeArea = *r.allNodeAreas.begin();  // selectBestNodeArea (Util.cpp:902-913)
    for (const auto& na : r.allNodeAreas) {
      if (na.first == me) {
        r.bestNodeArea = na;
        break;
      }
    }
    r.success = true;
  } else if (isBgp) {
    r = runBestPathSelectionBgp(entries, als);
  } else {
    for (const auto& [na, _] : entries) r.allNodeAreas.insert(na);
    r.bestNodeArea = *r.allNodeAreas.begin();
    r.success = true;
  }
  return filterDrained(std::move(r), als);
}

BestRouteSelectionResult SpfSolver::runBestPathSelectionBgp(const PrefixEntries& entries,
                                                            const AreaLinkStates& als) const {
  BestRouteSelectionResult r;  // Decision.cpp:864-902
  std::optional<MetricVector> bestVector;
  for (const auto& [na, e] : entries) {
    const Cmp c = bestVector ? compareMv(*e->mv, *bestVector) : Cmp::kWinner;
    if (c == Cmp::kTie || c == Cmp::kError) return r;
    if (c == Cmp::kWinner) r.allNodeAreas.clear();
    if (c == Cmp::kWinner || c == Cmp::kTieWinner) {
      bestVector = e->mv;
      r.bestNodeArea = na;
    }
    if (c != Cmp::kLooser) r.allNodeAreas.insert(na);
  }
  r.success = true;
  return filterDrained(std::move(r), als);
}

bool SpfSolver::fastSpEcmp(const std::string& me, const LinkState& ls, const std::string& area,
                           const std::set<NodeAndArea>& dsts, bool isV4,
                           std::optional<int32_t> swapLabel, NextHopSet& out) const {
  // getMinCostNodes + getNextHopsWithMetric + getNextHopsThrift for one area
  // and non-per-destination forwarding (Decision.cpp:1152-1334) on the row:
  // min over advertisers, OR of first-hop masks, then my links whose metric
  // equals the distance to their neighbour.
  const SpfRow& row = ls.getSpfRow(me);
  Metric shortest = std::numeric_limits<Metric>::max();
  std::vector<uint32_t> mask(row.words, 0u);
  bool any = false;
  for (const auto& [dst, _] : dsts) {
    auto id = ls.nodeId(dst);
    if (!row.known || !id || !row.reachable(*id)) continue;
    const Metric d = row.metric(*id);
    if (d > shortest) continue;
    if (d < shortest) {
      shortest = d;
      std::fill(mask.begin(), mask.end(), 0u);
    }
    any = true;
    for (uint32_t k = 0; k < row.words; ++k) mask[k] |= row.nh[static_cast<size_t>(*id) * row.words + k];
  }
  bool nonEmpty = false;
  for (uint32_t m : mask) nonEmpty |= m != 0;
  if (!any || !nonEmpty) return false;
  const uint32_t myId = *ls.nodeId(me);
  for (uint32_t lid : ls.linksFromNode(me)) {
    const Link& l = ls.link(lid);
    const uint32_t nbr = l.other(myId);
    if (!maskHas(row, mask, nbr) || !l.isUp()) continue;
    const Metric overLink = l.metricFrom(myId) + (shortest - row.metric(nbr));
    if (overLink != shortest) continue;
    const std::string& nbrName = ls.nodeName(nbr);
    std::optional<MplsAction> act;
    if (swapLabel) {
      act = dsts.count({nbrName, area}) ? mpls(kPhp) : mpls(kSwap, swapLabel);
    }
    out.insert(nextHop(isV4 ? l.nhV4From(myId) : l.nhV6From(myId), l.ifFrom(myId),
                       static_cast<int32_t>(overLink), std::move(act), l.area, nbrName));
  }
  return true;
}

std::pair<Metric, SpfSolver::NhMap> SpfSolver::getNextHopsWithMetric(
    const std::string& me, const std::set<NodeAndArea>& dsts, bool perDst,
    const AreaLinkStates& als) const {
  // Decision.cpp:1177-1228
  NhMap nhs;
  Metric shortest = std::numeric_limits<Metric>::max();
  for (const auto& [area, ls] : als) {
    const SpfRow& row = ls.getSpfRow(me);
    Metric areaMin = std::numeric_limits<Metric>::max();
    std::vector<std::string> minNodes;
    for (const auto& [dst, _] : dsts) {  // getMinCostNodes: area ignored
      auto m = rowMetric(ls, row, dst);
      if (!m) continue;
      if (areaMin >= *m) {
        if (areaMin > *m) {
          areaMin = *m;
          minNodes.clear();
        }
        if (std::find(minNodes.begin(), minNodes.end(), dst) == minNodes.end())
          minNodes.push_back(dst);
      }
    }
    if (shortest < areaMin) continue;
    if (shortest > areaMin) {
      shortest = areaMin;
      nhs.clear();
    }
    for (const auto& dst : minNodes) {
      const std::string dstRef = perDst ? dst : "";
      if (dst == row.srcName) continue;  // the source has no first hops
      const uint32_t did = *ls.nodeId(dst);
      row.forEachNextHop(did, [&](uint32_t nb) {
        const std::string& nbName = ls.nodeName(nb);
        nhs[{nbName, dstRef}] = shortest - *ls.getMetricFromAToB(me, nbName);
      });
    }
  }
  return {shortest, std::move(nhs)};
}

NextHopSet SpfSolver::getNextHopsThrift(const std::string& me, const std::set<NodeAndArea>& dsts,
                                        bool isV4, bool perDst, Metric minMetric, const NhMap& nhs,
                                        std::optional<int32_t> swapLabel,
                                        const AreaLinkStates& als,
                                        const PrefixEntries* entries) const {
  // Decision.cpp:1230-1334
  if (nhs.empty()) throw std::logic_error("getNextHopsThrift: no nexthop nodes");
  NextHopSet out;
  const std::set<NodeAndArea> noDst{{"", ""}};
  for (const auto& [area, ls] : als) {
    auto myId = ls.nodeId(me);
    if (!myId) continue;
    for (uint32_t lid : ls.linksFromNode(me)) {
      const Link& l = ls.link(lid);
      for (const auto& [dst, dstArea] : perDst ? dsts : noDst) {
        if (!dstArea.empty() && area != dstArea) continue;
        const std::string& nbr = ls.nodeName(l.other(*myId));
        auto it = nhs.find({nbr, dst});
        if (it == nhs.end() || !l.isUp()) continue;
        if (!dst.empty() && dsts.count({nbr, area}) && nbr != dst) continue;
        const Metric overLink = l.metricFrom(*myId) + it->second;
        if (overLink != minMetric) continue;
        std::optional<MplsAction> act;
        if (swapLabel) act = dsts.count({nbr, area}) ? mpls(kPhp) : mpls(kSwap, swapLabel);
        if (!dst.empty()) {
          std::vector<int32_t> push;
          const auto& dpe = entries->at({dst, area});
          if (dpe->prependLabel) {
            push.push_back(*dpe->prependLabel);
            if (!isMplsLabelValid(push.back())) continue;
          }
          if (dst != nbr) {
            push.push_back(ls.getAdjacencyDatabases().at(dst).nodeLabel);
            if (!isMplsLabelValid(push.back())) continue;
          }
          if (!push.empty()) act = mpls(kPush, std::nullopt, std::move(push));
        }
        out.insert(nextHop(isV4 ? l.nhV4From(*myId) : l.nhV6From(*myId), l.ifFrom(*myId),
                           static_cast<int32_t>(overLink), std::move(act), l.area, nbr));
      }
    }
  }
  return out;
}

std::optional<RibUnicastEntry> SpfSolver::selectBestPathsSpf(
    const std::string& me, const Cidr& prefix, const BestRouteSelectionResult& r,
    const PrefixEntries& entries, bool isBgp, int32_t ft, const AreaLinkStates& als) {
  // Decision.cpp:904-963
  const bool isV4 = prefix.first.size() == 4;
  const bool perDst = ft == kFwdSrMpls;
  std::set<NodeAndArea> filteredCopy;
  const std::set<NodeAndArea>* fp = &r.allNodeAreas;
  if (r.hasNode(me) && perDst) {
    for (const auto& [na, e] : entries) {
      if (na.first == me && e->prependLabel) {
        filteredCopy = r.allNodeAreas;
        filteredCopy.erase(na);
        fp = &filteredCopy;
        break;
      }
    }
  }
  const std::set<NodeAndArea>& filtered = *fp;
  if (!perDst && als.size() == 1) {
    const auto& [area, ls] = *als.begin();
    if (ls.nodeId(me)) {
      NextHopSet nhs;
      if (!fastSpEcmp(me, ls, area, filtered, isV4, std::nullopt, nhs)) return std::nullopt;
      return addBestPaths(me, prefix, r, entries, isBgp, std::move(nhs));
    }
  }
  auto nhm = getNextHopsWithMetric(me, filtered, perDst, als);
  if (nhm.second.empty()) return std::nullopt;
  return addBestPaths(me, prefix, r, entries, isBgp,
                      getNextHopsThrift(me, r.allNodeAreas, isV4, perDst, nhm.first, nhm.second,
                                        std::nullopt, als, &entries));
}

std::optional<RibUnicastEntry> SpfSolver::selectBestPathsKsp2(
    const std::string& me, const Cidr& prefix, const BestRouteSelectionResult& r,
    const PrefixEntries& entries, bool isBgp, int32_t ft, const AreaLinkStates& als) {
  // Decision.cpp:965-1087
  if (ft != kFwdSrMpls) return std::nullopt;
  struct AreaPath {
    const LinkState* ls;
    Path path;
  };
  std::vector<AreaPath> paths;
  for (const auto& [area, ls] : als) {
    for (const auto& [node, bestArea] : r.allNodeAreas) {
      if (node == me && bestArea == area) continue;
      for (const auto& p : ls.getKthPathIds(me, node, 1)) paths.push_back({&ls, p});
    }
    const size_t firstPaths = paths.size();
    for (const auto& [node, bestArea] : r.allNodeAreas) {
      if (area != bestArea) continue;
      for (const auto& sp : ls.getKthPathIds(me, node, 2)) {
        bool add = true;
        for (size_t i = 0; i < firstPaths; ++i) {
          // link identity is per LinkState; paths of other areas never match
          if (paths[i].ls == &ls && LinkState::pathAInPathB(paths[i].path, sp)) {
            add = false;
            break;
          }
        }
        if (add) paths.push_back({&ls, sp});
      }
    }
  }
  if (paths.empty()) return std::nullopt;

  NextHopSet nexthops;
  for (const auto& ap : paths) {
    const LinkState& pls = *ap.ls;
    for (const auto& [area, ls] : als) {
      Metric cost = 0;
      std::list<int32_t> labels;
      uint32_t next = *pls.nodeId(me);
      for (uint32_t lid : ap.path) {
        const Link& l = pls.link(lid);
        cost += l.metricFrom(next);
        next = l.other(next);
        labels.push_front(ls.getAdjacencyDatabases().at(pls.nodeName(next)).nodeLabel);
      }
      labels.pop_back();  // PHP: the first hop's label is not pushed
      const auto& pe = entries.at({pls.nodeName(next), area});
      if (pe->prependLabel) labels.push_front(*pe->prependLabel);
      const Link& first = pls.link(ap.path.front());
      const uint32_t myId = *pls.nodeId(me);
      std::optional<MplsAction> act;
      if (!labels.empty())
        act = mpls(kPush, std::nullopt, std::vector<int32_t>(labels.begin(), labels.end()));
      nexthops.insert(nextHop(prefix.first.size() == 4 ? first.nhV4From(myId) : first.nhV6From(myId),
                              first.ifFrom(myId), static_cast<int32_t>(cost), std::move(act),
                              first.area, pls.nodeName(first.other(myId))));
    }
  }
  return addBestPaths(me, prefix, r, entries, isBgp, std::move(nexthops));
}

std::optional<RibUnicastEntry> SpfSolver::addBestPaths(const std::string& me, const Cidr& prefix,
                                                       const BestRouteSelectionResult& r,
                                                       const PrefixEntries& entries, bool isBgp,
                                                       NextHopSet&& nexthops) {
  // Decision.cpp:1089-1150 (+ getMinNextHopThreshold :824-838)
  std::optional<int64_t> minNh;
  for (const auto& na : r.allNodeAreas) {
    const auto& e = entries.at(na);
    if (e->minNexthop && (!minNh || *e->minNexthop > *minNh)) minNh = e->minNexthop;
  }
  if (minNh && *minNh > static_cast<int64_t>(nexthops.size())) return std::nullopt;
  if (r.hasNode(me)) {
    std::optional<int32_t> prepend;
    for (const auto& [na, e] : entries) {
      if (na.first == me && e->prependLabel) {
        prepend = e->prependLabel;
        break;
      }
    }
    if (!prepend) throw std::logic_error("self-advertised route without prepend label");
    auto it = staticMplsRoutes_.find(*prepend);
    if (it != staticMplsRoutes_.end())
      for (const auto& nh : it->second)
        nexthops.insert(nextHop(nh.address, std::nullopt, 0, std::nullopt, std::nullopt, std::nullopt));
  }
  RibUnicastEntry e;
  e.prefix = prefix;
  e.nexthops = std::move(nexthops);
  e.bestPrefixEntry = entries.at(r.bestNodeArea);
  e.bestArea = r.bestNodeArea.second;
  e.doNotInstall = isBgp && bgpDryRun_;
  return e;
}

// Device route selection (route_select_kernel) for every prefix of the
// PrefixState mirror: status / shortest metric / best advertisement / per-area
// first-hop masks land in selStatus_ .. selMask_. The kernel's area list is
// the mirror's area ids, then every other area of `als` (getMinCostNodes
// reads every area's SPF, Decision.cpp:1194-1197). Returns false (all
// prefixes on the host path) when the inputs are outside what it covers.
bool SpfSolver::selectOnDevice(const std::string& me, const AreaLinkStates& als,
                               const PrefixState& ps, bool diff) {
  deviceSelected_ = hostSelected_ = 0;
  lastDiffed_ = false;
  devPol_.reset();  // policy decisions belong to the selection they were made on
  // a selection that does not complete (host path) leaves no snapshot: the
  // routes built from it do not correspond to the previous one any more
  const bool hadPrev = havePrev_;
  havePrev_ = false;
  if (std::getenv("ORH_HOST_SELECT")) return false;  // A/B switch: host selection
  // below ORH_DEVICE_SELECT_MIN prefixes (default 1024) the launch and the
  // row uploads cost more than selecting on the host (C1: 100 prefixes)
  size_t minPrefixes = 1024;
  if (const char* e = std::getenv("ORH_DEVICE_SELECT_MIN")) minPrefixes = std::strtoull(e, nullptr, 10);
  if (ps.numPrefixIds() == 0 || ps.numPrefixIds() < minPrefixes || als.empty()) return false;
  orh_ctx* ctx = als.begin()->second.context();
  for (const auto& [_, ls] : als)
    if (ls.context() != ctx) return false;
  if (selCtx_ && selCtx_ != ctx) return false;
  // the kernel reads u32 distance rows: path metrics past 32 bits stay on the host
  for (const auto& [_, ls] : als)
    if (ls.getSpfRow(me).known && !ls.getSpfRow(me).dist64.empty()) return false;
  // getNextHopsWithMetric keys nexthops by neighbour name only (:1221): a
  // neighbour name shared by two areas couples their links, keep those
  // topologies on the host path
  if (als.size() > 1) {
    std::unordered_set<std::string> seen;
    for (const auto& [_, ls] : als) {
      auto myId = ls.nodeId(me);
      if (!myId) continue;
      std::unordered_set<std::string> mine;
      for (uint32_t lid : ls.linksFromNode(me)) mine.insert(ls.nodeName(ls.link(lid).other(*myId)));
      for (const auto& n : mine)
        if (!seen.insert(n).second) return false;
    }
  }
  std::vector<const LinkState*> order;  // kernel area index -> LinkState (or null)
  for (uint32_t a = 0; a < ps.numAreas(); ++a) {
    auto it = als.find(ps.area(a));
    order.push_back(it == als.end() ? nullptr : &it->second);
  }
  for (const auto& [area, ls] : als)
    if (!ps.areaId(area)) order.push_back(&ls);
  if (order.size() > 32) return false;
  selCtx_ = ctx;
  RouteProf prof;
  orh_prefix_set* set = ps.syncDevice(ctx);
  prof.mark(" select: sync");
  areaWork_.resize(order.size());
  std::vector<orh_select_area> sel(order.size());
  uint32_t words = 0;
  const uint32_t nNames = ps.numNames();
  for (size_t a = 0; a < order.size(); ++a) {
    AreaWork& w = areaWork_[a];
    sel[a] = orh_select_area{};
    w.words = 0;
    w.tmpl4.clear();
    w.linkOrder.clear();
    w.tmpl6.clear();
    const LinkState* ls = order[a];
    if (!ls) continue;
    sel[a].present = 1;
    const SpfRow& row = ls->getSpfRow(me);
    orh_graph* g = ls->deviceGraph();
    if (!row.known) continue;  // me's SpfResult holds only me: nothing reachable
    const uint32_t N = row.n;
    // names -> node ids of this area (incremental while both only grow)
    if (w.ls != ls || w.lsNodes != ls->numNodeIds() || w.psNames > nNames) {
      w.ls = ls;
      w.lsNodes = ls->numNodeIds();
      w.psNames = 0;
      w.nameNode.clear();
    }
    if (w.psNames != nNames) {
      w.nameNode.resize(nNames);
      for (uint32_t n = w.psNames; n < nNames; ++n) {
        auto id = ls->nodeId(ps.name(n));
        w.nameNode[n] = id && *id < N ? *id : ORH_NO_NODE;
      }
      if (nNames > w.dNameNodeCap) {
        if (w.dNameNode) orh_device_free(ctx, w.dNameNode);
        w.dNameNodeCap = std::max<size_t>(nNames, 2 * w.dNameNodeCap);
        w.dNameNode = nullptr;
        if (orh_device_alloc(ctx, w.dNameNodeCap * 4, reinterpret_cast<void**>(&w.dNameNode)) != ORH_OK)
          throw std::runtime_error("route select: device allocation failed");
      }
      if (orh_memcpy_h2d(ctx, w.dNameNode, w.nameNode.data(), nNames * 4ull) != ORH_OK)
        throw std::runtime_error(std::string("route select: ") + orh_last_error(ctx));
      w.psNames = nNames;
    }
    // me's rows of this area
    const size_t rowWords = static_cast<size_t>(N) * (1 + row.words);
    if (rowWords > w.dRowCap) {
      if (w.dRow) orh_device_free(ctx, w.dRow);
      w.dRow = nullptr;
      w.dRowCap = rowWords;
      if (orh_device_alloc(ctx, rowWords * 4, reinterpret_cast<void**>(&w.dRow)) != ORH_OK)
        throw std::runtime_error("route select: device allocation failed");
    }
    if (orh_memcpy_h2d(ctx, w.dRow, row.dist.data(), N * 4ull) != ORH_OK ||
        orh_memcpy_h2d(ctx, w.dRow + N, row.nh.data(), row.nh.size() * 4ull) != ORH_OK)
      throw std::runtime_error(std::string("route select: ") + orh_last_error(ctx));
    const uint8_t* dOvl = nullptr;
    if (orh_graph_device_flags(g, &dOvl) != ORH_OK)
      throw std::runtime_error(std::string("route select: ") + orh_last_error(ctx));
    w.words = row.words;
    w.wordOff = words;
    words += row.words;
    sel[a].d_dist = w.dRow;
    sel[a].d_nh = w.dRow + N;
    sel[a].d_overloaded = dOvl;
    sel[a].d_name_node = w.dNameNode;
    sel[a].words = w.words;
    sel[a].word_off = w.wordOff;
    // nexthop templates per first-hop bit: my up links whose metric equals
    // the distance to their neighbour (getNextHopsThrift's distOverLink ==
    // minMetric, Decision.cpp:1271-1276, for a neighbour on a shortest path)
    w.tmpl4.assign(row.nbrs.size(), {});
    w.tmpl6.assign(row.nbrs.size(), {});
    w.linkOrder.clear();
    const uint32_t myId = row.src;
    for (uint32_t lid : ls->linksFromNode(me)) {  // LinkSet iteration order
      const Link& l = ls->link(lid);
      const uint32_t nbr = l.other(myId);
      if (!l.isUp() || !row.reachable(nbr) || l.metricFrom(myId) != row.metric(nbr)) continue;
      auto k = std::lower_bound(row.nbrs.begin(), row.nbrs.end(), nbr) - row.nbrs.begin();
      if (k >= static_cast<ptrdiff_t>(row.nbrs.size()) || row.nbrs[k] != nbr) continue;
      const std::string& nbrName = ls->nodeName(nbr);
      w.linkOrder.emplace_back(static_cast<uint32_t>(k), static_cast<uint32_t>(w.tmpl6[k].size()));
      w.tmpl6[k].push_back(nextHop(l.nhV6From(myId), l.ifFrom(myId), 0, std::nullopt, l.area, nbrName));
      w.tmpl4[k].push_back(nextHop(l.nhV4From(myId), l.ifFrom(myId), 0, std::nullopt, l.area, nbrName));
    }
  }
  areaIter_.clear();
  for (const auto& [area, ls] : als)  // the reference's area loop order
    for (size_t a = 0; a < order.size(); ++a)
      if (order[a] == &ls) areaIter_.push_back(static_cast<uint32_t>(a));
  // digest of everything a materialised route depends on besides its
  // selection record: the area layout and every nexthop template
  uint64_t layout = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const auto* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) layout = (layout ^ b[i]) * 1099511628211ull;
  };
  // the insertion sequence too (a set iterates in the order its nexthops went
  // in): areas in AreaLinkStates order, my links in LinkSet order - a rehash
  // of my LinkSet can reorder the links with the templates unchanged
  for (uint32_t a : areaIter_) mix(&a, sizeof a);
  for (const AreaWork& w : areaWork_) {
    mix(&w.words, sizeof w.words);
    mix(&w.wordOff, sizeof w.wordOff);
    const void* ls = w.ls;
    mix(&ls, sizeof ls);
    const uint32_t nl = static_cast<uint32_t>(w.linkOrder.size());
    mix(&nl, sizeof nl);
    for (const auto& [b, j] : w.linkOrder) {
      mix(&b, sizeof b);
      mix(&j, sizeof j);
    }
    for (const auto* tm : {&w.tmpl6, &w.tmpl4}) {
      const uint32_t nb = static_cast<uint32_t>(tm->size());
      mix(&nb, sizeof nb);
      for (const auto& bit : *tm) {
        const uint32_t c = static_cast<uint32_t>(bit.size());
        mix(&c, sizeof c);
        for (const auto& t : bit) {
          mix(t.address.addr.data(), t.address.addr.size());
          if (t.address.ifName) mix(t.address.ifName->data(), t.address.ifName->size());
          if (t.area) mix(t.area->data(), t.area->size());
          if (t.neighborNodeName) mix(t.neighborNodeName->data(), t.neighborNodeName->size());
          mix("|", 1);
        }
      }
    }
  }
  prof.mark(" select: areas");
  // outputs: status [n] | metric [n] | best [n] | mask [n][words]
  const uint32_t n = ps.numPrefixIds();
  auto outOf = [&](uint8_t* base, uint32_t np) { return selOut(base, np, words); };
  const size_t n4 = (static_cast<size_t>(n) + 3) & ~static_cast<size_t>(3);
  const size_t bytes = n4 + 8ull * n + 4ull * n * std::max(words, 1u);
  if (bytes > dSelCap_) {
    if (dSel_) orh_device_free(ctx, dSel_);
    dSel_ = nullptr;
    dSelCap_ = std::max(bytes, dSelCap_ * 2);
    if (orh_device_alloc(ctx, dSelCap_, reinterpret_cast<void**>(&dSel_)) != ORH_OK)
      throw std::runtime_error("route select: device allocation failed");
  }
  orh_select_out out = outOf(dSel_, n);
  const auto meName = ps.nameId(me);
  uint32_t flags = (enableBestRouteSelection_ ? ORH_SELECT_BEST_ROUTE : 0u) |
      (enableV4_ ? ORH_SELECT_V4 : 0u);
  // a prefix shard selects (and copies back) its own block of prefix ids only
  const auto [pidLo, pidHi] = shardRange(n);
  if (orh_route_select_range(set, meName ? *meName : ORH_NO_NODE, flags, static_cast<uint32_t>(order.size()),
                             sel.data(), pidLo, pidHi, &out) != ORH_OK)
    throw std::runtime_error(std::string("orh_route_select: ") + orh_last_error(ctx));
  {
    uint32_t np = 0, live = 0;
    orh_prefix_info(set, &np, &live, nullptr);
    uint32_t areasWithRow = 0;
    for (const auto& sa : sel) areasWithRow += sa.d_dist ? 1 : 0;
    lastSelectBytes_ = 8ull * np + 20ull * live + 4ull * live * areasWithRow +
        static_cast<uint64_t>(np) * (9 + 4ull * words);
    if (np) lastSelectBytes_ = lastSelectBytes_ * (pidHi - pidLo) / np;  // the shard's share
  }
  prof.mark(" select: launch");
  const bool canDiff = diff && hadPrev && dSelPrev_ && prevWords_ == words && prevLayout_ == layout &&
                       prevN_ <= n && selStatus_.size() == prevN_;
  if (canDiff) {
    // only the records that differ from the snapshot come back
    const size_t rec = 4 + words;
    const size_t need = (static_cast<size_t>(n) * rec + 1) * 4;
    if (need > dDiffCap_) {
      if (dDiff_) orh_device_free(ctx, dDiff_);
      dDiff_ = nullptr;
      dDiffCap_ = std::max(need, dDiffCap_ * 2);
      if (orh_device_alloc(ctx, dDiffCap_, reinterpret_cast<void**>(&dDiff_)) != ORH_OK)
        throw std::runtime_error("route diff: device allocation failed");
    }
    const orh_select_out prev = outOf(dSelPrev_, prevN_);
    if (orh_route_diff(set, n, prevN_, &out, &prev, dDiff_ + 1, dDiff_) != ORH_OK)
      throw std::runtime_error(std::string("orh_route_diff: ") + orh_last_error(ctx));
    uint32_t k = 0;
    if (orh_memcpy_d2h(ctx, &k, dDiff_, 4) != ORH_OK)
      throw std::runtime_error(std::string("route diff copy-out: ") + orh_last_error(ctx));
    std::vector<uint32_t> recs(static_cast<size_t>(k) * rec);
    if (k && orh_memcpy_d2h(ctx, recs.data(), dDiff_ + 1, recs.size() * 4) != ORH_OK)
      throw std::runtime_error(std::string("route diff copy-out: ") + orh_last_error(ctx));
    selStatus_.resize(n, ORH_SEL_NONE);
    selMetric_.resize(n, 0);
    selBest_.resize(n, 0);
    selMask_.resize(static_cast<size_t>(n) * words, 0);
    changedPids_.resize(k);
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t* r = recs.data() + static_cast<size_t>(i) * rec;
      const uint32_t pid = r[0];
      changedPids_[i] = pid;
      selStatus_[pid] = static_cast<uint8_t>(r[1]);
      selMetric_[pid] = r[2];
      selBest_[pid] = r[3];
      std::copy(r + 4, r + 4 + words, selMask_.begin() + static_cast<size_t>(pid) * words);
    }
    lastDiffed_ = true;
  } else {
    selStatus_.resize(n);
    selMetric_.resize(n);
    selBest_.resize(n);
    selMask_.resize(static_cast<size_t>(n) * words);
    const size_t lo = pidLo, cnt = pidHi - pidLo;
    if (orh_memcpy_d2h(ctx, selStatus_.data() + lo, out.d_status + lo, cnt) != ORH_OK ||
        orh_memcpy_d2h(ctx, selMetric_.data() + lo, out.d_metric + lo, 4ull * cnt) != ORH_OK ||
        orh_memcpy_d2h(ctx, selBest_.data() + lo, out.d_best + lo, 4ull * cnt) != ORH_OK ||
        orh_memcpy_d2h(ctx, selMask_.data() + lo * words, out.d_mask + lo * words, 4ull * cnt * words) != ORH_OK)
      throw std::runtime_error(std::string("route select copy-out: ") + orh_last_error(ctx));
  }
  prof.mark(" select: copy-out");
  selWords_ = words;
  if (orh_last_select_ms(set, &lastSelectMs_) != ORH_OK) lastSelectMs_ = -1;
  // this selection is the snapshot the next one is compared with
  std::swap(dSel_, dSelPrev_);
  std::swap(dSelCap_, dSelPrevCap_);
  havePrev_ = shardWorld_ == 1;
  selGen_ = nextGeneration();  // process-unique: also names this solver
  prevN_ = n;
  prevWords_ = words;
  prevLayout_ = layout;
  return true;
}

template <class Act>
void SpfSolver::insertTemplates(const uint32_t* m, bool v4, int32_t metric,
                                const std::vector<std::vector<int32_t>>* wt,
                                std::vector<std::pair<const NextHopThrift*, int32_t>>* wts, NextHopSet& out,
                                Act&& act) const {
  // getNextHopsThrift's loops (Decision.cpp:1245-1246): areas in
  // AreaLinkStates order, then my links in LinkSet order; a link is a
  // nexthop when its neighbour's first-hop bit is set and it is tight
  for (uint32_t a : areaIter_) {
    const AreaWork& w = areaWork_[a];
    if (!w.words) continue;
    const auto& tmpl = v4 ? w.tmpl4 : w.tmpl6;
    for (const auto& [b, j] : w.linkOrder) {
      if (!((m[w.wordOff + b / 32] >> (b % 32)) & 1u)) continue;
      NextHopThrift nh = tmpl[b][j];
      nh.metric = metric;
      nh.mplsAction = act(nh);
      auto it = out.insert(std::move(nh)).first;
      if (wts) wts->emplace_back(&*it, (*wt)[a][b]);
    }
  }
}

RibUnicastEntry SpfSolver::materialize(uint32_t pid, const PrefixState& ps) const {
  // selectBestPathsSpf -> getNextHopsThrift -> addBestPaths (Decision.cpp
  // :904-963, :1230-1334, :1089-1150) for a device-selected IP / SP_ECMP
  // prefix: every set first-hop bit contributes its tight links, each with
  // metric = the shortest distance
  RibUnicastEntry e;
  e.prefix = ps.prefixOf(pid);
  const bool v4 = e.prefix.first.size() == 4;
  const int32_t metric = static_cast<int32_t>(selMetric_[pid]);
  const uint32_t* m = selMask_.data() + static_cast<size_t>(pid) * selWords_;
  // RibPolicy decided on the device: statement s sets every nexthop's weight
  // (RibPolicy.cpp:117-141); a weight of 0 drops the nexthop, and s only
  // applies when some nexthop keeps a weight (the kernel checked)
  const uint32_t s = devPol_.on ? devPol_.stmt[pid] : ORH_POL_NONE;
  // the nexthop set as the reference builds it: templates inserted in
  // getNextHopsThrift's order, and for a policy statement the set rebuilt
  // with its weights in the first set's iteration order
  auto buildSet = [&](NextHopSet& out) {
    if (s < ORH_POL_MAX_STMTS) {
      // the reference builds the route (weights 0), then the policy moves
      // the kept nexthops into a new set in the first set's iteration order
      // (RibPolicy.cpp:116-141): the same two sets here, so the result
      // iterates in the reference's order; weights from the device decision
      thread_local std::vector<std::pair<const NextHopThrift*, int32_t>> wts;
      wts.clear();
      NextHopSet built;
      insertTemplates(m, v4, metric, &devPol_.weight[s], &wts, built, noAction);
      while (!built.empty()) {
        auto node = built.extract(built.begin());  // node addresses are stable
        int32_t w = 0;
        for (const auto& [p, pw] : wts)
          if (p == &node.value()) w = pw;
        if (w <= 0) continue;
        node.value().weight = w;
        out.insert(std::move(node));
      }
    } else {
      insertTemplates(m, v4, metric, nullptr, nullptr, out, noAction);
    }
  };
  // Routes with the same first-hop mask, metric, family and policy statement
  // get the same set from the same insertion sequence: it is built once per
  // worker thread and then shared (NextHops), so it iterates exactly as the
  // set built in place - the reference's order (a30). C3: ~2,400 distinct
  // sets for 100k routes. A set depends on nothing else but the nexthop
  // templates and area layout (their digest, prevLayout_ of the selection
  // that produced the record) and the policy's weights (its generation), so
  // the cache lives across builds while those stay: a build after a
  // topology change elsewhere builds no set it had before.
  struct NhKey {  // mask words, metric, family + statement (inline: no allocation)
    uint32_t w[8];
    uint32_t n;
    bool operator==(const NhKey& o) const { return n == o.n && std::memcmp(w, o.w, n * 4) == 0; }
  };
  struct NhKeyHash {
    size_t operator()(const NhKey& k) const {
      uint64_t h = 0x9E3779B97F4A7C15ull ^ k.n;
      for (uint32_t i = 0; i < k.n; ++i) h = (h ^ k.w[i]) * 0x100000001B3ull;
      return static_cast<size_t>(h ^ (h >> 29));
    }
  };
  struct NhCache {
    uint64_t layout = 0, polGen = 0;
    uint32_t hits = 0, misses = 0;
    std::unordered_map<NhKey, NextHops, NhKeyHash> sets;  // shared with the routes
  };
  thread_local NhCache cache;
  const uint64_t polGen = s < ORH_POL_MAX_STMTS && devPol_.policy ? devPol_.policy->generation() : 0;
  if (cache.layout != prevLayout_ || (s < ORH_POL_MAX_STMTS && cache.polGen != polGen)) {
    cache.sets.clear();
    cache.layout = prevLayout_;
    cache.polGen = polGen;
    cache.hits = cache.misses = 0;
  }
  // off when the words do not fit the key, or once the sets turn out to be
  // mostly distinct (a miss builds the set and stores a copy)
  static const bool enabled = [] {  // ORH_NH_CACHE=0 (A/B): every set built in place
    const char* e = std::getenv("ORH_NH_CACHE");
    return !(e && e[0] == '0');
  }();
  const bool use = enabled && selWords_ + 2 <= 8 && cache.sets.size() < (1u << 16) &&
                   !(cache.misses >= 512 && cache.hits < cache.misses);
  if (use) {
    NhKey key;
    key.n = selWords_ + 2;
    std::memcpy(key.w, m, selWords_ * 4u);
    key.w[selWords_] = static_cast<uint32_t>(metric);
    key.w[selWords_ + 1] = (v4 ? 4u : 6u) | (s << 8);
    auto it = cache.sets.find(key);
    if (it != cache.sets.end()) {
      ++cache.hits;
      e.nexthops = it->second;
    } else {
      ++cache.misses;
      NextHopSet built;
      buildSet(built);
      e.nexthops = std::move(built);
      cache.sets.emplace(key, e.nexthops);
    }
  } else {
    NextHopSet built;
    buildSet(built);
    e.nexthops = std::move(built);
  }
  uint32_t cnt = 0;
  const AdvRef* advs = ps.advs(pid, &cnt);
  const AdvRef& best = advs[selBest_[pid]];
  e.bestPrefixEntry = *best.entry;
  e.bestArea = best.key->second;
  e.doNotInstall = false;  // BGP prefixes take the host path
  if (s == ORH_POL_HOST) {  // a tag set without a device id: matched on the host
    uint64_t inv = 0;
    if (devPol_.policy->applyAction(e, &inv)) ++devPol_.hostUpdated;
    if (inv) devPol_.hostInvalidated += inv;
  }
  return e;
}

bool SpfSolver::policyOnDevice(const PrefixState& ps, RibPolicy& policy) {
  devPol_.reset();
  const auto t0 = std::chrono::steady_clock::now();
  const auto& st = policy.statements();
  if (st.empty() || st.size() > ORH_POL_MAX_STMTS || !selCtx_ || !dSelPrev_ || prevN_ == 0) return false;
  const uint32_t S = static_cast<uint32_t>(st.size());
  const uint32_t words = selWords_, n = prevN_;
  orh_policy pol{};
  pol.n_stmts = S;
  pol.total_words = words;
  // set_weight per statement, area and first-hop bit: every template of a
  // bit is a link to one neighbour in one area, so they share the weight
  devPol_.weight.assign(S, {});
  std::vector<uint32_t> keep(static_cast<size_t>(S) * words, 0u);
  for (uint32_t s = 0; s < S; ++s) {
    devPol_.weight[s].resize(areaWork_.size());
    for (size_t a = 0; a < areaWork_.size(); ++a) {
      const AreaWork& w = areaWork_[a];
      auto& wa = devPol_.weight[s][a];
      wa.assign(w.tmpl6.size(), 0);
      for (size_t b = 0; b < w.tmpl6.size() && b < 32ull * w.words; ++b) {
        if (w.tmpl6[b].empty()) continue;
        const NextHopThrift& t = w.tmpl6[b].front();
        wa[b] = st[s].weightOf(t.area, t.neighborNodeName);
        if (wa[b] > 0) keep[s * words + w.wordOff + b / 32] |= 1u << (b % 32);
      }
    }
    if (!st[s].tagSet().empty()) pol.stmt_tags |= 1u << s;
    if (!st[s].prefixSet().empty()) pol.stmt_prefixes |= 1u << s;
  }
  // tag set id -> statements whose tag matcher it meets (id 0: no tags)
  const uint32_t nts = std::min<uint32_t>(ps.numTagSets(), ps.tagSetIdLimit() - 1) + 1;
  std::vector<uint32_t> tagStmts(nts, 0u);
  if (pol.stmt_tags) {
    for (uint32_t t = 1; t < nts; ++t)
      for (const auto& tag : ps.tagSet(t))
        for (uint32_t s = 0; s < S; ++s)
          if (st[s].tagSet().count(tag)) tagStmts[t] |= 1u << s;
  }
  // prefix ids named by the prefix matchers
  std::map<uint32_t, uint32_t> named;
  for (uint32_t s = 0; s < S; ++s)
    for (const Cidr& c : st[s].prefixSet())
      if (auto pid = ps.pidOf(c); pid && *pid < n) named[*pid] |= 1u << s;
  std::vector<uint32_t> pfxId, pfxStmts;
  for (const auto& [pid, mk] : named) {
    pfxId.push_back(pid);
    pfxStmts.push_back(mk);
  }
  pol.n_tagsets = nts;
  pol.h_tagset_stmts = tagStmts.data();
  pol.n_pfx = static_cast<uint32_t>(pfxId.size());
  pol.h_pfx_id = pfxId.data();
  pol.h_pfx_stmts = pfxStmts.data();
  pol.h_keep = keep.data();
  orh_ctx* ctx = selCtx_;
  // a device failure here leaves the decision to the host: the caller then
  // runs RibPolicy::applyPolicy over the built routes (same result)
  auto hostPath = [&](const char* what) {
    std::fprintf(stderr, "openr_amd: %s failed (%s); RibPolicy applied on the host\n", what, orh_last_error(ctx));
    devPol_.reset();
    return false;
  };
  const size_t need = n + 64;  // out bytes | invalidated (aligned)
  if (need > dPolOutCap_) {
    const size_t cap = std::max(need, 2 * dPolOutCap_);
    if (dPolOut_) orh_device_free(ctx, dPolOut_);
    dPolOut_ = nullptr;
    dPolOutCap_ = 0;
    if (orh_device_alloc(ctx, cap, reinterpret_cast<void**>(&dPolOut_)) != ORH_OK)
      return hostPath("route policy: device allocation");
    dPolOutCap_ = cap;
  }
  uint32_t* dInv = reinterpret_cast<uint32_t*>(dPolOut_ + ((n + 15) & ~size_t{15}));
  const orh_select_out sel = selOut(dSelPrev_, n, words);
  // a prefix shard decides (and counts the invalidated routes of) its own
  // block only
  const auto [lo, hi] = shardRange(n);
  if (orh_route_policy_range(ps.syncDevice(ctx), lo, hi, &sel, &pol, dPolOut_, dInv) != ORH_OK)
    return hostPath("orh_route_policy");
  devPol_.stmt.resize(n);
  uint32_t inv = 0;
  if (orh_memcpy_d2h(ctx, devPol_.stmt.data() + lo, dPolOut_ + lo, hi - lo) != ORH_OK ||
      orh_memcpy_d2h(ctx, &inv, dInv, 4) != ORH_OK)
    return hostPath("route policy copy-out");
  devPol_.deviceInvalidated = inv;
  devPol_.policy = &policy;
  devPol_.on = true;
  devPol_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return true;
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(const std::string& me,
                                                       const AreaLinkStates& als,
                                                       const PrefixState& ps) {
  return buildRouteDbImpl(me, als, ps, false);
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDbWithPolicy(const std::string& me,
                                                                 const AreaLinkStates& als,
                                                                 const PrefixState& ps, RibPolicy* policy,
                                                                 PolicyStats* stats) {
  PolicyStats local;
  PolicyStats& st = stats ? *stats : local;
  st = PolicyStats{};
  policyStats_ = &st;
  try {
    auto db = buildRouteDbImpl(me, als, ps, false, policy);
    policyStats_ = nullptr;
    return db;
  } catch (...) {
    policyStats_ = nullptr;
    throw;
  }
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDbImpl(const std::string& me,
                                                           const AreaLinkStates& als,
                                                           const PrefixState& ps, bool mplsOnly,
                                                           RibPolicy* policy) {
  // Decision.cpp:615-792 (mplsOnly: the MPLS routes alone, for buildRouteDelta)
  mplsKeyOk_ = false;
  bool exists = false;
  for (const auto& [_, ls] : als) exists |= ls.hasNode(me);
  if (!exists) return std::nullopt;
  if (!mplsOnly) ++routeBuildRuns_;

  // KSP2 prefixes need one fresh SPF per best node (getKthPaths k = 2): plan
  // them first and run them as one device batch (the memo then serves the
  // route build with the same paths and the same spf_runs count)
  RouteProf prof;
  bool hasKsp = false;
  if (ps.ksp2Entries() > 0 && !mplsOnly) {
    std::unordered_map<const LinkState*, std::vector<std::pair<std::string, std::string>>> plan;
    kspPlan_ = &plan;
    try {
      for (const auto& [prefix, entries] : ps.prefixes()) {
        bool ksp = false;
        for (const auto& [na, e] : entries) ksp |= e->forwardingAlgorithm == kAlgoKsp2EdEcmp;
        if (ksp) createRouteForPrefix(me, als, ps, prefix);
      }
    } catch (...) {
      kspPlan_ = nullptr;
      throw;
    }
    kspPlan_ = nullptr;
    for (auto& [ls, pairs] : plan) ls->prefetchKthPaths(pairs);
    hasKsp = !plan.empty();
  }

  // Every SPF row the prefixes read is memoized from here on (me's row per
  // area; KSP2 paths were prefetched above), so the per-prefix work reads
  // shared state only and runs on the host worker pool. KSP2 prefixes that
  // found paths in other areas may still trace lazily, so their presence
  // keeps the loop sequential.
  prof.mark("ksp2 plan");
  for (const auto& [_, ls] : als) ls.getSpfRow(me);
  prof.mark("spf(me)");
  DecisionRouteDb db;
  if (ps.prefixes().size() < kParallelMin) db.unicastRoutes.reserve(ps.prefixes().size());
  auto& pool = WorkerPool::instance();
  // per-prefix selection on the device; the host materialises the routes it
  // selected and runs the full reference logic for the prefixes it returns
  // as ORH_SEL_HOST (BGP, SR_MPLS / KSP2, minNexthop, self-advertised)
  const bool dev = !mplsOnly && selectOnDevice(me, als, ps);
  prof.mark("select (device)");
  // RibPolicy (buildRouteDbWithPolicy): decided on the device for the
  // device-selected routes and applied as they are materialised; host-path
  // routes take applyAction as they are built, static routes as they are
  // added; without a device decision, applyPolicy over the whole database
  const bool policyActive = !mplsOnly && policy && policy->isActive();
  const bool devPolicy = dev && policyActive && policyOnDevice(ps, *policy);
  auto hostPolicy = [&](RibUnicastEntry& r) {
    if (!devPolicy) return;
    uint64_t inv = 0;
    if (policy->applyAction(r, &inv)) ++devPol_.hostUpdated;
    if (inv) devPol_.hostInvalidated += inv;
  };
  if (devPolicy) prof.mark("policy (device)");
  bool labelsDone = false;  // node-label routes built by the pipelined path
  // node-label candidates per area (the candidate entry of every adjacency
  // database); computed on the pool beside the unicast routes when the
  // generic pool path runs, else in the node-label section below
  struct LabelArea {
    const std::string* area;
    const LinkState* ls;
    std::vector<const AdjacencyDatabase*> dbs;
    const AreaWork* tw = nullptr;
    const SpfRow* myRow = nullptr;
    std::vector<std::optional<RibMplsEntry>> cand;
  };
  std::vector<LabelArea> labAreas;
  std::vector<size_t> labOff{0};  // flat candidate index -> area
  bool labPre = false;
  auto labelPrepare = [&] {
    for (const auto& [area, ls] : als) {
      LabelArea la;
      la.area = &area;
      la.ls = &ls;
      for (const auto& [_, adjDb] : ls.getAdjacencyDatabases()) la.dbs.push_back(&adjDb);
      la.cand.resize(la.dbs.size());
      // one area with device-selection templates: the route to node v is its
      // first-hop mask in me's row, each bit's tight links with PHP when the
      // neighbour is v, else SWAP(label) (getNextHopsThrift, :1278-1287)
      if (dev && als.size() == 1)
        for (const auto& w : areaWork_)
          if (w.ls == &ls && w.words) la.tw = &w;
      la.myRow = la.tw ? &ls.getSpfRow(me) : nullptr;
      labOff.push_back(labOff.back() + la.dbs.size());
      labAreas.push_back(std::move(la));
    }
  };
  auto labelCompute = [&](LabelArea& la, size_t i) {
    const std::string& area = *la.area;
    const LinkState& ls = *la.ls;
    const AdjacencyDatabase& adjDb = *la.dbs[i];
    const int32_t label = adjDb.nodeLabel;
    if (label == 0 || !isMplsLabelValid(label)) return;
    RibMplsEntry entry{label, {}};
    if (adjDb.thisNodeName == me) {
      NextHopThrift nh;
      nh.address.addr = std::string(16, '\0');  // "::"
      nh.area = area;
      nh.mplsAction = mpls(kPopAndLookup);
      entry.nexthops.insert(std::move(nh));
    } else if (la.tw) {
      auto v = ls.nodeId(adjDb.thisNodeName);
      if (!v || !la.myRow->reachable(*v)) return;
      const int32_t metric = static_cast<int32_t>(la.myRow->metric(*v));
      const uint32_t* vm = la.myRow->nh.data() + static_cast<size_t>(*v) * la.tw->words;
      bool any = false;
      for (uint32_t k = 0; k < la.tw->words; ++k) any |= vm[k] != 0;
      if (any)  // one area: its words start at 0
        insertTemplates(vm, false, metric, nullptr, nullptr, entry.nexthops.edit(),
                        [&](const NextHopThrift& nh) -> std::optional<MplsAction> {
                          return *nh.neighborNodeName == adjDb.thisNodeName ? mpls(kPhp) : mpls(kSwap, label);
                        });
      if (!any) return;
    } else {
      const std::set<NodeAndArea> dst{{adjDb.thisNodeName, area}};
      if (als.size() == 1 && ls.nodeId(me)) {
        if (!fastSpEcmp(me, ls, area, dst, false, label, entry.nexthops.edit())) return;
      } else {
        auto nhm = getNextHopsWithMetric(me, dst, false, als);
        if (nhm.second.empty()) return;
        entry.nexthops = getNextHopsThrift(me, dst, false, false, nhm.first, nhm.second, label, als, nullptr);
      }
    }
    la.cand[i] = std::move(entry);
  };
  std::vector<const Cidr*> keys;
  // static unicast routes go to the shard of their prefix id (shard 0 when
  // PrefixState lacks the prefix)
  auto ownsStatic = [&](const Cidr& prefix) {
    if (shardWorld_ <= 1) return true;
    auto pid = ps.pidOf(prefix);
    return pid ? ownsPid(*pid, ps.numPrefixIds()) : shardRank_ == 0;
  };
  uint64_t devPolOnDevice = 0, devPolUpdated = 0;
  if (dev) {
    const uint32_t n = ps.numPrefixIds();
    // a prefix shard materialises its own block of prefix ids [pidLo, pidHi)
    const auto [pidLo, pidHi] = shardRange(n);
    const uint32_t nOwn = pidHi - pidLo;
    // the selection counts (and the device policy's, read after the build)
    // in one pass over the pool: C5's 1M ids were two sequential passes
    {
      const size_t W = 4 * pool.size();  // chunks, claimed dynamically
      std::vector<std::array<uint64_t, 4>> cnt(W, std::array<uint64_t, 4>{});
      auto countRange = [&](size_t w, size_t b, size_t e) {
        uint64_t h = 0, d = 0, od = 0, up = 0;
        for (size_t i = b; i < e; ++i) {
          const uint32_t pid = pidLo + static_cast<uint32_t>(i);
          if (!ps.prefixLive(pid)) continue;
          const uint8_t st = selStatus_[pid];
          if (st == ORH_SEL_HOST) ++h; else ++d;
          if (devPolicy && st == ORH_SEL_ROUTE && devPol_.stmt[pid] != ORH_POL_HOST) {
            ++od;
            up += devPol_.stmt[pid] < ORH_POL_MAX_STMTS;
          }
        }
        cnt[w] = {h, d, od, up};
      };
      if (nOwn >= kParallelMin && W > 1) pool.parallelFor(nOwn, countRange, W);
      else countRange(0, 0, nOwn);
      uint64_t s[4] = {0, 0, 0, 0};
      for (const auto& c : cnt)
        for (int k = 0; k < 4; ++k) s[k] += c[k];
      hostSelected_ = s[0];
      deviceSelected_ = s[1];
      devPolOnDevice = s[2];
      devPolUpdated = s[3];
    }
    using RouteMap = decltype(db.unicastRoutes);
    // the unicast routes of [pidLo, pidHi) into db, and `extra(k)` for k in
    // [0, nExtra) (node-label candidates) in the same pool pass. Two passes
    // (ORH_ROUTE_TWO_PHASE=0, A/B: one pass into per-worker maps, then
    // spliced): the routes are built over contiguous prefix-id ranges into a
    // flat slot array (no hashing, no map nodes), each worker listing its
    // slots per output shard; then each shard's routes move into its map,
    // shard by shard on the pool - one insertion per route instead of an
    // insertion and a splice (C5: build 51-54 -> 42-45 ms,
    // profiles/r05/ze_route_two_phase_ab.txt)
    auto fillRoutes = [&](size_t nExtra, auto&& extra) {
      static const bool twoPhase = [] {
        const char* e = std::getenv("ORH_ROUTE_TWO_PHASE");
        return !(e && e[0] == '0');
      }();
      if (!twoPhase) {
        std::vector<RouteMap> parts(pool.size());
        pool.parallelFor(nOwn + nExtra, [&](size_t w, size_t b, size_t e) {
          for (size_t i = b; i < e; ++i) {
            if (i >= nOwn) {
              extra(i - nOwn);
              continue;
            }
            const uint32_t pid = pidLo + static_cast<uint32_t>(i);
            if (!ps.prefixLive(pid)) continue;
            if (selStatus_[pid] == ORH_SEL_ROUTE) {
              RibUnicastEntry r = materialize(pid, ps);
              Cidr k = r.prefix;
              parts[w].shard(RouteMap::shardOf(k)).emplace(std::move(k), std::move(r));
            } else if (selStatus_[pid] == ORH_SEL_HOST) {
              if (auto r = createRouteForPrefix(me, als, ps, ps.prefixOf(pid))) {
                hostPolicy(*r);
                Cidr k = r->prefix;
                parts[w].shard(RouteMap::shardOf(k)).emplace(std::move(k), std::move(*r));
              }
            }
          }
        });
        prof.mark("unicast + labels (pool)");
        mergeParts(db.unicastRoutes, parts, pool);
        prof.mark("unicast merge");
        return;
      }
      constexpr size_t kS = RouteMap::kShards;
      // the pass in chunks claimed dynamically, several per thread, so a
      // pool thread held up by a busy core (threads are pinned) leaves its
      // remaining chunks to the others (ORH_FILL_CHUNKS: chunks per thread,
      // 1 = one per thread, A/B)
      static const size_t perThread = [] {
        const char* e = std::getenv("ORH_FILL_CHUNKS");
        return e && std::atoi(e) > 0 ? static_cast<size_t>(std::atoi(e)) : size_t{4};
      }();
      const size_t W = pool.size() * perThread;  // chunk (list) count
      RouteSlots& slots = routeSlots_;
      slots.reserve(nOwn);
      slots.lists.resize(W * kS);
      for (auto& l : slots.lists) l.clear();
      // a slot is listed right after it is constructed: on an exception the
      // listed slots are exactly the live ones, destroyed before rethrowing
      auto dropListed = [&] {
        for (auto& l : slots.lists) {
          for (uint32_t i : l) slots.at(i)->~RibUnicastEntry();
          l.clear();
        }
      };
      try {
      pool.parallelFor(nOwn + nExtra, [&](size_t w, size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) {
          if (i >= nOwn) {
            extra(i - nOwn);
            continue;
          }
          const uint32_t pid = pidLo + static_cast<uint32_t>(i);
          if (!ps.prefixLive(pid)) continue;
          RibUnicastEntry* slot = slots.at(i);
          if (selStatus_[pid] == ORH_SEL_ROUTE) {
            new (slot) RibUnicastEntry(materialize(pid, ps));
          } else if (selStatus_[pid] == ORH_SEL_HOST) {
            auto r = createRouteForPrefix(me, als, ps, ps.prefixOf(pid));
            if (!r) continue;
            hostPolicy(*r);
            new (slot) RibUnicastEntry(std::move(*r));
          } else {
            continue;
          }
          slots.lists[w * kS + RouteMap::shardOf(slot->prefix)].push_back(static_cast<uint32_t>(i));
        }
      }, W);
      } catch (...) {
        dropListed();
        throw;
      }
      prof.mark("unicast + labels (pool)");
      std::atomic<bool> dup{false};
      // per list, the slots already moved out and destroyed (a list is
      // consumed in order by the one thread that owns its shard): if the
      // merge throws (bad_alloc in reserve / emplace), exactly the rest are
      // destroyed before rethrowing
      std::vector<uint32_t> done(W * kS, 0u);
      // shards claimed one at a time (dynamic chunks): shard sizes vary, and
      // kS / threads leaves a static split uneven. ORH_MERGE_DYN=0: static (A/B)
      static const size_t mergeChunks = [] {
        const char* e = std::getenv("ORH_MERGE_DYN");
        return (e && e[0] == '0') ? size_t{0} : kS;
      }();
      try {
      pool.parallelFor(kS, [&](size_t, size_t b, size_t e) {
        for (size_t sh = b; sh < e; ++sh) {
          size_t n = 0;
          for (size_t w = 0; w < W; ++w) n += slots.lists[w * kS + sh].size();
          auto& dst = db.unicastRoutes.shard(sh);
          dst.reserve(dst.size() + n);
          for (size_t w = 0; w < W; ++w) {
            const auto& list = slots.lists[w * kS + sh];
            for (size_t q = 0; q < list.size(); ++q) {
              // a shard's slots are ~1/64 of the slot array apart: the
              // slots a few routes ahead are fetched while this one inserts
              constexpr size_t kAhead = 6;
              if (q + kAhead < list.size()) {
                const char* ahead = reinterpret_cast<const char*>(slots.at(list[q + kAhead]));
                __builtin_prefetch(ahead);
                __builtin_prefetch(ahead + 64);
              }
              const uint32_t i = list[q];
              RibUnicastEntry* r = slots.at(i);
              Cidr k = r->prefix;
              if (!dst.emplace(std::move(k), std::move(*r)).second) dup = true;
              r->~RibUnicastEntry();
              ++done[w * kS + sh];
            }
          }
        }
      }, mergeChunks);
      } catch (...) {
        for (size_t l = 0; l < slots.lists.size(); ++l) {
          auto& list = slots.lists[l];
          for (size_t q = done[l]; q < list.size(); ++q) slots.at(list[q])->~RibUnicastEntry();
          list.clear();
        }
        throw;
      }
      for (auto& l : slots.lists) l.clear();
      if (dup) throw std::logic_error("duplicate unicast route");
      prof.mark("unicast merge");
    };
    auto one = [&](uint32_t pid, RouteMap::Shard& out) {
      if (!ps.prefixLive(pid)) return;
      if (selStatus_[pid] == ORH_SEL_ROUTE) {
        RibUnicastEntry e = materialize(pid, ps);
        Cidr k = e.prefix;
        out.emplace(std::move(k), std::move(e));
      } else if (selStatus_[pid] == ORH_SEL_HOST) {
        if (auto r = createRouteForPrefix(me, als, ps, ps.prefixOf(pid))) {
          hostPolicy(*r);
          Cidr k = r->prefix;
          out.emplace(std::move(k), std::move(*r));
        }
      }
    };
    // one area with nexthop templates: unicast routes and node-label
    // candidates in one pool pass, then the two output maps are assembled
    // concurrently (their insertion is the sequential part of the build);
    // node labels belong to shard 0
    const AreaWork* tw = nullptr;
    if (als.size() == 1)
      for (const auto& w : areaWork_)
        if (w.ls == &als.begin()->second && w.words) tw = &w;
    if (!hasKsp && tw && nOwn >= kParallelMin && pool.size() > 1) {
      const auto& [area, ls] = *als.begin();
      const SpfRow& myRow = ls.getSpfRow(me);
      std::vector<const AdjacencyDatabase*> dbs;
      if (shardRank_ == 0) {
        dbs.reserve(ls.getAdjacencyDatabases().size());
        for (const auto& [_, adjDb] : ls.getAdjacencyDatabases()) dbs.push_back(&adjDb);
      }
      std::vector<std::optional<RibMplsEntry>> cand(dbs.size());
      auto label = [&, &area = area, &ls = ls](size_t i) {
        const AdjacencyDatabase& adjDb = *dbs[i];
        const int32_t lbl = adjDb.nodeLabel;
        if (lbl == 0 || !isMplsLabelValid(lbl)) return;
        RibMplsEntry entry{lbl, {}};
        if (adjDb.thisNodeName == me) {  // POP_AND_LOOKUP (Decision.cpp:690-703)
          NextHopThrift nh;
          nh.address.addr = std::string(16, '\0');
          nh.area = area;
          nh.mplsAction = mpls(kPopAndLookup);
          entry.nexthops.insert(std::move(nh));
        } else {
          auto v = ls.nodeId(adjDb.thisNodeName);
          if (!v || !myRow.reachable(*v)) return;
          const int32_t metric = static_cast<int32_t>(myRow.metric(*v));
          const uint32_t* vm = myRow.nh.data() + static_cast<size_t>(*v) * tw->words;
          bool any = false;
          for (uint32_t k = 0; k < tw->words; ++k) any |= vm[k] != 0;
          if (!any) return;
          // the row's words are the only area's: wordOff 0
          insertTemplates(vm, false, metric, nullptr, nullptr, entry.nexthops.edit(),
                          [&](const NextHopThrift& nh) -> std::optional<MplsAction> {
                            return *nh.neighborNodeName == adjDb.thisNodeName ? mpls(kPhp) : mpls(kSwap, lbl);
                          });
        }
        cand[i] = std::move(entry);
      };
      fillRoutes(dbs.size(), label);
      for (const auto& [prefix, nhs] : staticUnicastRoutes_) {
        if (db.unicastRoutes.count(prefix) || !ownsStatic(prefix)) continue;
        RibUnicastEntry se;
        se.prefix = prefix;
        se.nexthops.insert(nhs.begin(), nhs.end());
        hostPolicy(se);
        db.unicastRoutes.emplace(prefix, std::move(se));
      }
      prof.mark("unicast statics");
      // duplicate labels: the smaller node name wins among the nodes with a
      // route (:675-688); labels are resolved shard by shard on the pool
      if (!dbs.empty()) {
        std::vector<std::vector<uint32_t>> byLabelShard(MplsRouteMap::kShards);
        for (size_t i = 0; i < dbs.size(); ++i) {
          const int32_t lbl = dbs[i]->nodeLabel;
          if (lbl == 0 || !isMplsLabelValid(lbl) || !cand[i]) continue;
          byLabelShard[MplsRouteMap::shardOf(lbl)].push_back(static_cast<uint32_t>(i));
        }
        // per shard: candidates sorted by (label, node name), the first of
        // each label wins - no per-shard map of winners to allocate; shards
        // claimed one at a time
        pool.parallelFor(MplsRouteMap::kShards, [&](size_t, size_t b, size_t e) {
          for (size_t sh = b; sh < e; ++sh) {
            auto& list = byLabelShard[sh];
            std::sort(list.begin(), list.end(), [&](uint32_t x, uint32_t y) {
              const int32_t lx = dbs[x]->nodeLabel, ly = dbs[y]->nodeLabel;
              return lx != ly ? lx < ly : dbs[x]->thisNodeName < dbs[y]->thisNodeName;
            });
            auto& dst = db.mplsRoutes.shard(sh);
            dst.reserve(dst.size() + list.size() + 1);
            for (size_t q = 0; q < list.size(); ++q) {
              const uint32_t i = list[q];
              if (q && dbs[list[q - 1]]->nodeLabel == dbs[i]->nodeLabel) continue;
              dst.emplace(dbs[i]->nodeLabel, std::move(*cand[i]));
            }
          }
        }, MplsRouteMap::kShards);
        prof.mark("label map");
      }
      labelsDone = true;
    } else if (!hasKsp && nOwn >= kParallelMin && pool.size() > 1) {
      // the node-label candidates (shard 0) are computed in the same pass
      if (shardRank_ == 0) {
        labelPrepare();
        labPre = true;
      }
      const size_t nLab = labOff.back();
      auto label = [&](size_t f) {
        const size_t a = static_cast<size_t>(std::upper_bound(labOff.begin(), labOff.end(), f) - labOff.begin()) - 1;
        labelCompute(labAreas[a], f - labOff[a]);
      };
      fillRoutes(nLab, label);
    } else {
      for (uint32_t pid = pidLo; pid < pidHi; ++pid) {
        if (!ps.prefixLive(pid)) continue;
        one(pid, db.unicastRoutes.shard(RouteMap::shardOf(ps.prefixOf(pid))));
      }
    }
  } else if (!mplsOnly) {
    keys.reserve(ps.prefixes().size());
    const uint32_t n = ps.numPrefixIds();
    for (const auto& [prefix, _] : ps.prefixes())
      if (shardWorld_ == 1 || ownsPid(*ps.pidOf(prefix), n)) keys.push_back(&prefix);
  }
  if (dev) {
    // routes built above
  } else if (!hasKsp && keys.size() >= kParallelMin && pool.size() > 1) {
    // each worker fills a map of the output type; the merge splices nodes
    // (no entry is copied or moved)
    std::vector<decltype(db.unicastRoutes)> parts(pool.size());
    pool.parallelFor(keys.size(), [&](size_t w, size_t b, size_t e) {
      for (size_t i = b; i < e; ++i)
        if (auto r = createRouteForPrefix(me, als, ps, *keys[i])) {
          Cidr k = r->prefix;
          parts[w].emplace(std::move(k), std::move(*r));
        }
    });
    prof.mark("unicast (pool)");
    mergeParts(db.unicastRoutes, parts, pool);
  } else {
    for (const Cidr* prefix : keys) {
      if (auto r = createRouteForPrefix(me, als, ps, *prefix)) {
        if (!db.unicastRoutes.emplace(*prefix, std::move(*r)).second)
          throw std::logic_error("duplicate unicast route");
      }
    }
  }
  if (!labelsDone && !mplsOnly) {
    for (const auto& [prefix, nhs] : staticUnicastRoutes_) {
      if (db.unicastRoutes.count(prefix) || !ownsStatic(prefix)) continue;
      RibUnicastEntry e;
      e.prefix = prefix;
      e.nexthops.insert(nhs.begin(), nhs.end());
      hostPolicy(e);
      db.unicastRoutes.emplace(prefix, std::move(e));
    }
    prof.mark("unicast merge");
  }
  if (policyActive) {
    uint64_t updated = 0, onDevice = 0;
    if (devPolicy) {
      onDevice = devPolOnDevice;  // counted with the selection (devPolicy implies dev)
      updated = devPolUpdated;
      updated += devPol_.hostUpdated;
      policy->addInvalidated(devPol_.deviceInvalidated + devPol_.hostInvalidated);
    } else {  // RibPolicy::applyPolicy over the whole database on the host
      const uint64_t inv0 = policy->invalidatedRoutes();
      updated = policy->applyPolicy(db.unicastRoutes).updatedRoutes.size();
      if (policyStats_) policyStats_->invalidated = policy->invalidatedRoutes() - inv0;
    }
    if (policyStats_) {
      policyStats_->updated = updated;
      policyStats_->onDevice = onDevice;
      if (devPolicy) {
        policyStats_->invalidated = devPol_.deviceInvalidated + devPol_.hostInvalidated;
        policyStats_->deviceMs = devPol_.ms;
      }
    }
    devPol_.on = false;  // later materialisations (other builds) select anew
    prof.mark("policy (host part)");
  }
  // node-label routes; duplicate labels resolve to the smaller node name.
  // The candidate entry of every adjacency database is computed on the
  // worker pool, then the duplicate resolution walks them in the reference's
  // iteration order (Decision.cpp:655-744).
  std::unordered_map<int32_t, std::pair<std::string, RibMplsEntry>> labelToNode;
  if (!labelsDone && shardRank_ == 0 && !labPre) {
    labelPrepare();
    const size_t nLab = labOff.back();
    if (nLab >= kParallelMin && pool.size() > 1) {
      pool.parallelFor(nLab, [&](size_t, size_t b, size_t e) {
        for (size_t f = b; f < e; ++f) {
          const size_t a = static_cast<size_t>(std::upper_bound(labOff.begin(), labOff.end(), f) - labOff.begin()) - 1;
          labelCompute(labAreas[a], f - labOff[a]);
        }
      });
    } else {
      for (auto& la : labAreas)
        for (size_t i = 0; i < la.dbs.size(); ++i) labelCompute(la, i);
    }
  }
  for (auto& la : labAreas) {
    if (labelsDone || shardRank_ != 0) break;
    const auto& dbs = la.dbs;
    auto& cand = la.cand;
    // winner per label: (node name, candidate index); entries move once
    std::unordered_map<int32_t, std::pair<const std::string*, size_t>> win;
    win.reserve(dbs.size());
    for (size_t i = 0; i < dbs.size(); ++i) {
      const AdjacencyDatabase& adjDb = *dbs[i];
      const int32_t label = adjDb.nodeLabel;
      if (label == 0 || !isMplsLabelValid(label)) continue;
      auto lt = labelToNode.find(label);  // an earlier area's winner
      const std::string* held = nullptr;
      auto it = win.find(label);
      if (it != win.end()) held = it->second.first;
      else if (lt != labelToNode.end()) held = &lt->second.first;
      if (held && *held < adjDb.thisNodeName) continue;
      if (!cand[i]) continue;
      if (lt != labelToNode.end()) labelToNode.erase(lt);
      win[label] = {&adjDb.thisNodeName, i};
    }
    if (als.size() == 1) {  // one area: the winners are the routes
      for (auto& [label, w] : win) db.mplsRoutes.emplace(label, std::move(*cand[w.second]));
      continue;
    }
    for (auto& [label, w] : win)
      labelToNode.emplace(label, std::make_pair(*w.first, std::move(*cand[w.second])));
  }
  for (auto& [label, ne] : labelToNode) db.mplsRoutes.emplace(label, std::move(ne.second));
  prof.mark("node labels");

  // adjacency-label routes for all my links, up or not (:749-775)
  for (const auto& [_, ls] : als) {
    if (shardRank_ != 0) break;
    auto myId = ls.nodeId(me);
    if (!myId) continue;
    for (uint32_t lid : ls.linksFromNode(me)) {
      const Link& l = ls.link(lid);
      const int32_t label = l.adjLabelFrom(*myId);
      if (label == 0 || !isMplsLabelValid(label)) continue;
      RibMplsEntry e{label, {}};
      e.nexthops.insert(nextHop(l.nhV6From(*myId), l.ifFrom(*myId),
                                static_cast<int32_t>(l.metricFrom(*myId)), mpls(kPhp), l.area,
                                ls.nodeName(l.other(*myId))));
      if (!db.mplsRoutes.emplace(label, std::move(e)).second)
        throw std::logic_error("duplicate mpls route");
    }
  }
  for (const auto& [label, nhs] : staticMplsRoutes_) {
    if (shardRank_ != 0) break;
    RibMplsEntry e{label, {}};
    e.nexthops.insert(nhs.begin(), nhs.end());
    if (!db.mplsRoutes.emplace(label, std::move(e)).second)
      throw std::logic_error("duplicate mpls route");
  }
  prof.mark("adj + static mpls");
  mplsKey_ = mplsInputs(als);
  mplsMe_ = me;
  mplsStatic_ = staticEpoch_;
  mplsKeyOk_ = true;
  return db;
}

std::vector<std::pair<const LinkState*, uint64_t>> SpfSolver::mplsInputs(const AreaLinkStates& als) const {
  std::vector<std::pair<const LinkState*, uint64_t>> k;
  for (const auto& [_, ls] : als) k.emplace_back(&ls, ls.stateStamp());
  return k;
}

std::optional<DecisionRouteUpdate> SpfSolver::buildRouteDelta(const std::string& me,
                                                              const AreaLinkStates& als,
                                                              const PrefixState& ps,
                                                              const DecisionRouteDb& current,
                                                              uint64_t selGen, uint64_t psStamp,
                                                              RibPolicy* policy) {
  if (!havePrev_ || selGen != selGen_ || shardWorld_ != 1 || ps.ksp2Entries() > 0) return std::nullopt;
  bool exists = false;
  for (const auto& [_, ls] : als) exists |= ls.hasNode(me);
  if (!exists) return std::nullopt;
  std::vector<Cidr> deleted;
  if (!ps.forEachDeletedSince(psStamp, [&](const Cidr& c) { deleted.push_back(c); })) return std::nullopt;
  RouteProf prof;
  for (const auto& [_, ls] : als) ls.getSpfRow(me);
  prof.mark("spf(me)");
  if (!selectOnDevice(me, als, ps, true) || !lastDiffed_) return std::nullopt;  // the caller builds in full
  prof.mark("select + diff (device)");
  ++routeBuildRuns_;
  const uint32_t n = ps.numPrefixIds();
  // prefixes to rebuild: changed selection records, prefixes changed since
  // psStamp, and the host-path prefixes (their inputs are not in the record)
  std::vector<uint8_t> want(n, 0);
  for (uint32_t pid : changedPids_) want[pid] = 1;
  auto& pool = WorkerPool::instance();
  pool.parallelFor(n, [&](size_t, size_t b, size_t e) {
    for (size_t pid = b; pid < e; ++pid)
      if (selStatus_[pid] == ORH_SEL_HOST || ps.pidStamp(static_cast<uint32_t>(pid)) > psStamp) want[pid] = 1;
  });
  std::vector<uint32_t> todo;
  for (uint32_t pid = 0; pid < n; ++pid)
    if (want[pid] && ps.prefixLive(pid)) todo.push_back(pid);
  uint64_t nDev = 0, nHost = 0;
  for (uint32_t pid : todo) (selStatus_[pid] == ORH_SEL_HOST ? nHost : nDev) += 1;
  deviceSelected_ = nDev;
  hostSelected_ = nHost;
  prof.mark("candidates");
  const bool applyPolicy = policy && policy->isActive();
  // the policy decided on the device for the materialised routes (as in
  // buildRouteDbWithPolicy); host-path and static routes take applyAction
  const bool devPolicy = applyPolicy && policyOnDevice(ps, *policy);
  // the full rebuild counts the policy's invalidated routes over the whole
  // DB (RibPolicy.cpp:149-150 via Decision.cpp:1895); without the device's
  // count of every selected route the delta cannot, so the caller rebuilds
  if (applyPolicy && !devPolicy) return std::nullopt;
  if (devPolicy) prof.mark("policy (device)");
  auto staticRoute = [&](const Cidr& p) -> std::optional<RibUnicastEntry> {
    auto it = staticUnicastRoutes_.find(p);
    if (it == staticUnicastRoutes_.end()) return std::nullopt;
    RibUnicastEntry e;
    e.prefix = p;
    e.nexthops.insert(it->second.begin(), it->second.end());
    return e;
  };
  struct alignas(128) Part {  // one per worker, no shared cache lines
    std::vector<RibUnicastEntry> upd;
    std::vector<Cidr> del;
    uint64_t invalidated{0};
    double tBuild{0}, tPolicy{0}, tFind{0}, tCmp{0}, tPush{0}, tCpu{0};  // ORH_ROUTE_PROF
    size_t n{0};
  };
  using Clock = std::chrono::steady_clock;
  auto ms = [](Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  auto cpuMs = [] {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
  };
  // chunks claimed dynamically: host-path prefixes (BGP, SR-MPLS, ...) cost
  // far more than materialised ones and cluster by prefix id
  const size_t nChunks = std::min<size_t>(8 * pool.size(), std::max<size_t>(todo.size() + deleted.size(), 1));
  std::vector<Part> parts(nChunks);
  // the new route of one prefix (createRouteForPrefixOrGetStaticRoute, then
  // the policy), compared with current's entry (calculateUpdate)
  auto one = [&](const Cidr& prefix, std::optional<RibUnicastEntry> r, Part& out, bool policyDone) {
    if (!r) {
      r = staticRoute(prefix);
      policyDone = false;
    }
    const auto t1 = prof.on ? Clock::now() : Clock::time_point{};
    if (r && applyPolicy && !policyDone) policy->applyAction(*r, &out.invalidated);
    const auto t2 = prof.on ? Clock::now() : Clock::time_point{};
    auto it = current.unicastRoutes.find(prefix);
    const auto t3 = prof.on ? Clock::now() : Clock::time_point{};
    bool differs = false;
    if (r) differs = it == current.unicastRoutes.end() || it->second != *r;
    const auto t4 = prof.on ? Clock::now() : Clock::time_point{};
    if (r) {
      if (differs) out.upd.push_back(std::move(*r));
    } else if (it != current.unicastRoutes.end()) {
      out.del.push_back(prefix);
    }
    if (prof.on) {
      const auto t5 = Clock::now();
      out.tPolicy += ms(t1, t2);
      out.tFind += ms(t2, t3);
      out.tCmp += ms(t3, t4);
      out.tPush += ms(t4, t5);
    }
  };
  // items: the prefix ids to rebuild, then the withdrawn prefixes (their
  // routes go, or fall back to a static route, unless a live id carries them)
  const size_t nItems = todo.size() + deleted.size();
  pool.parallelFor(nItems, [&](size_t w, size_t b, size_t e) {
    const double c0 = prof.on ? cpuMs() : 0.0;
    parts[w].upd.reserve(parts[w].upd.size() + (e - b));  // no regrowth (and its page faults) per route
    for (size_t i = b; i < e; ++i) {
      if (i >= todo.size()) {
        const Cidr& c = deleted[i - todo.size()];
        if (!ps.pidOf(c)) one(c, std::nullopt, parts[w], false);
        continue;
      }
      const uint32_t pid = todo[i];
      const Cidr& prefix = ps.prefixOf(pid);
      const auto t0 = prof.on ? Clock::now() : Clock::time_point{};
      std::optional<RibUnicastEntry> r;
      bool policyDone = false;
      if (selStatus_[pid] == ORH_SEL_ROUTE) {
        r = materialize(pid, ps);
        policyDone = devPolicy;
      } else if (selStatus_[pid] == ORH_SEL_HOST) {
        r = createRouteForPrefix(me, als, ps, prefix);
      }
      if (prof.on) {
        parts[w].tBuild += ms(t0, Clock::now());
        ++parts[w].n;
      }
      one(prefix, std::move(r), parts[w], policyDone);
    }
    if (prof.on) parts[w].tCpu += cpuMs() - c0;
  }, nChunks);
  if (prof.on) {
    double b = 0, pl = 0, f = 0, c = 0, pu = 0, cpu = 0;
    size_t nn = 0, busy = 0;
    for (const auto& p : parts) {
      b += p.tBuild;
      pl += p.tPolicy;
      f += p.tFind;
      c += p.tCmp;
      pu += p.tPush;
      cpu += p.tCpu;
      nn += p.n;
      busy += p.n > 0;
    }
    std::fprintf(stderr,
                 "route-prof delta: %zu routes on %zu workers; thread-ms build %.3f policy %.3f find %.3f "
                 "compare %.3f push %.3f; thread cpu-ms %.3f\n",
                 nn, busy, b, pl, f, c, pu, cpu);
  }
  prof.mark("unicast (pool)");
  DecisionRouteUpdate delta;
  uint64_t invalidated = 0;
  for (auto& p : parts) {
    for (auto& r : p.upd) {
      Cidr k = r.prefix;
      if (!delta.unicastRoutesToUpdate.emplace(std::move(k), std::move(r)).second)
        throw std::logic_error("buildRouteDelta: duplicate unicast route");  // RouteUpdate.h:39 CHECK
    }
    for (auto& c : p.del) delta.unicastRoutesToDelete.push_back(std::move(c));
    invalidated += p.invalidated;
  }
  // the device counted every selected route, as the reference's full rebuild
  // counts every route it applies the policy to (RibPolicy.cpp:149-150)
  if (devPolicy) {
    // routes whose tag set has no device id (ORH_POL_HOST) take applyAction as
    // they materialise: the ones not rebuilt above are materialised to count
    pool.parallelFor(n, [&](size_t, size_t b, size_t e) {
      for (size_t pid = b; pid < e; ++pid)
        if (!want[pid] && selStatus_[pid] == ORH_SEL_ROUTE && devPol_.stmt[pid] == ORH_POL_HOST &&
            ps.prefixLive(static_cast<uint32_t>(pid)))
          (void)materialize(static_cast<uint32_t>(pid), ps);
    });
    invalidated += devPol_.deviceInvalidated + devPol_.hostInvalidated;
    // and every static route the full DB holds that no item above rebuilt:
    // its prefix has no live id, or a live id with no route, and was not
    // withdrawn since psStamp (buildRouteDbImpl applies the policy to each)
    std::unordered_set<Cidr, CidrHash> gone;
    if (!staticUnicastRoutes_.empty()) gone.insert(deleted.begin(), deleted.end());
    for (const auto& [prefix, nhs] : staticUnicastRoutes_) {
      const auto pid = ps.pidOf(prefix);
      const bool live = pid && ps.prefixLive(*pid);
      if (live ? (want[*pid] || selStatus_[*pid] != ORH_SEL_NONE) : gone.count(prefix) != 0) continue;
      auto r = staticRoute(prefix);
      policy->applyAction(*r, &invalidated);
    }
  }
  if (policy) policy->addInvalidated(invalidated);
  devPol_.on = false;
  // MPLS routes: unchanged inputs (no topology or static change since the
  // build current holds) keep them; else rebuilt and compared in full
  if (mplsKeyOk_ && mplsMe_ == me && mplsStatic_ == staticEpoch_ && mplsKey_ == mplsInputs(als)) {
    prof.mark("mpls (kept)");
    return delta;
  }
  auto mdb = buildRouteDbImpl(me, als, ps, true);
  {  // compared shard by shard (same key -> shard map); lists in iteration order
    constexpr size_t kS = MplsRouteMap::kShards;
    std::vector<std::vector<RibMplsEntry>> upd(kS);
    std::vector<std::vector<int32_t>> del(kS);
    pool.parallelFor(kS, [&](size_t, size_t b, size_t e) {
      for (size_t sh = b; sh < e; ++sh) {
        const auto& cur = current.mplsRoutes.shard(sh);
        if (mdb) {
          for (auto& [label, entry] : mdb->mplsRoutes.shard(sh)) {
            auto it = cur.find(label);
            if (it == cur.end() || it->second != entry) upd[sh].push_back(std::move(entry));
          }
        }
        for (const auto& [label, _] : cur)
          if (!mdb || !mdb->mplsRoutes.shard(sh).count(label)) del[sh].push_back(label);
      }
    });
    for (size_t sh = 0; sh < kS; ++sh) {
      for (auto& e : upd[sh]) delta.mplsRoutesToUpdate.push_back(std::move(e));
      delta.mplsRoutesToDelete.insert(delta.mplsRoutesToDelete.end(), del[sh].begin(), del[sh].end());
    }
  }
  prof.mark("mpls");
  return delta;
}

}  // namespace openr_amd
