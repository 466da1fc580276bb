// TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle_types.h header).
// Restates openr/decision/Decision.cpp (SpfSolverImpl), PrefixState.cpp and
// the Util.cpp helpers the route build uses; each function cites its source.
#include "oracle_decision.h"

#include <algorithm>
#include <limits>
#include <list>
#include <stdexcept>

namespace oracle {

// ---- PrefixState (PrefixState.cpp:17-56) -----------------------------------
std::unordered_set<Cidr, CidrHash> PrefixState::updatePrefix(const std::string& node,
                                                             const std::string& area,
                                                             const PrefixEntry& e) {
  std::unordered_set<Cidr, CidrHash> changed;
  Cidr key{e.prefixAddr, e.prefixLen};
  auto [it, inserted] = prefixes_[key].emplace(NodeAndArea{node, area}, e);
  if (!inserted && it->second == e) return changed;
  if (!inserted) it->second = e;
  changed.insert(key);
  return changed;
}

std::unordered_set<Cidr, CidrHash> PrefixState::deletePrefix(const std::string& node,
                                                             const std::string& area,
                                                             const Cidr& prefix) {
  std::unordered_set<Cidr, CidrHash> changed;
  auto it = prefixes_.find(prefix);
  if (it != prefixes_.end() && it->second.erase(NodeAndArea{node, area})) {
    changed.insert(prefix);
    if (it->second.empty()) prefixes_.erase(it);
  }
  return changed;
}

// ---- Util helpers -----------------------------------------------------------
std::set<NodeAndArea> selectBestPrefixMetrics(const PrefixEntries& entries) {
  // Util.h:491-526: lexicographic max of (path_pref, source_pref, -distance)
  using T = std::tuple<int32_t, int32_t, int32_t>;
  T best{std::numeric_limits<int32_t>::min(), std::numeric_limits<int32_t>::min(),
         std::numeric_limits<int32_t>::min()};
  std::set<NodeAndArea> keys;
  for (const auto& [k, e] : entries) {
    // distance * -1 in int32 (wrapping negation)
    T t{e.metrics.path_preference, e.metrics.source_preference,
        static_cast<int32_t>(0u - static_cast<uint32_t>(e.metrics.distance))};
    if (t < best) continue;
    if (t > best) {
      best = t;
      keys.clear();
    }
    keys.insert(k);
  }
  return keys;
}

NodeAndArea selectBestNodeArea(const std::set<NodeAndArea>& all, const std::string& me) {
  NodeAndArea best = *all.begin();  // Util.cpp:902-913
  for (const auto& na : all) {
    if (na.first == me) {
      best = na;
      break;
    }
  }
  return best;
}

std::pair<int32_t, int32_t> getPrefixForwardingTypeAndAlgorithm(
    const PrefixEntries& entries, const std::set<NodeAndArea>& best) {
  // Util.cpp:452-480: minimum enum value over the best entries
  if (entries.empty()) return {FT_IP, FA_SP_ECMP};
  std::pair<int32_t, int32_t> r{FT_SR_MPLS, FA_KSP2_ED_ECMP};
  for (const auto& [k, e] : entries) {
    if (!best.count(k)) continue;
    r.first = std::min(r.first, e.forwardingType);
    r.second = std::min(r.second, e.forwardingAlgorithm);
    if (r.first == FT_IP && r.second == FA_SP_ECMP) return r;
  }
  return r;
}

static MplsAction mplsAction(int32_t code, std::optional<int32_t> swap = std::nullopt,
                             std::optional<std::vector<int32_t>> push = std::nullopt) {
  // createMplsAction + checkMplsAction (Util.cpp:482-512, :793-803)
  MplsAction a{code, swap, push};
  if (code == PUSH && (!push || push->empty())) throw std::logic_error("bad PUSH");
  if (code == SWAP && (!swap || !isMplsLabelValid(*swap))) throw std::logic_error("bad SWAP");
  if (push)
    for (auto l : *push)
      if (!isMplsLabelValid(l)) throw std::logic_error("bad push label");
  return a;
}

static NextHopThrift nextHop(const BinaryAddress& addr, std::optional<std::string> ifName,
                             int32_t metric, std::optional<MplsAction> action,
                             std::optional<std::string> area,
                             std::optional<std::string> nbr) {
  NextHopThrift nh;  // createNextHop (Util.cpp:775-789); metric narrows to i32
  nh.address.addr = addr.addr;
  nh.address.ifName = std::move(ifName);
  nh.metric = metric;
  nh.mplsAction = std::move(action);
  nh.area = std::move(area);
  nh.neighborNodeName = std::move(nbr);
  return nh;
}

// ---- MetricVectorUtils (Util.cpp:938-1094) ---------------------------------
static CompareResult invert(CompareResult r) {
  switch (r) {
    case CompareResult::WINNER: return CompareResult::LOOSER;
    case CompareResult::TIE_WINNER: return CompareResult::TIE_LOOSER;
    case CompareResult::TIE: return CompareResult::TIE;
    case CompareResult::TIE_LOOSER: return CompareResult::TIE_WINNER;
    case CompareResult::LOOSER: return CompareResult::WINNER;
    default: return CompareResult::ERROR;
  }
}
static bool decisive(CompareResult r) {
  return r == CompareResult::WINNER || r == CompareResult::LOOSER ||
      r == CompareResult::ERROR;
}
static CompareResult compareMetrics(const std::vector<int64_t>& l,
                                    const std::vector<int64_t>& r, bool tb) {
  if (l.size() != r.size()) return CompareResult::ERROR;
  for (size_t i = 0; i < l.size(); ++i) {
    if (l[i] > r[i]) return tb ? CompareResult::TIE_WINNER : CompareResult::WINNER;
    if (l[i] < r[i]) return tb ? CompareResult::TIE_LOOSER : CompareResult::LOOSER;
  }
  return CompareResult::TIE;
}
static CompareResult loner(const MetricEntity& e) {
  if (e.op == 1 /*WIN_IF_PRESENT*/)
    return e.isBestPathTieBreaker ? CompareResult::TIE_WINNER : CompareResult::WINNER;
  if (e.op == 2 /*WIN_IF_NOT_PRESENT*/)
    return e.isBestPathTieBreaker ? CompareResult::TIE_LOOSER : CompareResult::LOOSER;
  return CompareResult::TIE;
}
static void maybeUpdate(CompareResult& t, CompareResult u) {
  if (decisive(u) || t == CompareResult::TIE) t = u;
}
CompareResult compareMetricVectors(MetricVector l, MetricVector r) {
  if (l.version != r.version) return CompareResult::ERROR;
  auto byPrio = [](const MetricEntity& a, const MetricEntity& b) {
    return a.priority > b.priority;
  };
  // sortMetricVector sorts only when not already sorted (non-stable sort)
  if (!std::is_sorted(l.metrics.begin(), l.metrics.end(), byPrio))
    std::sort(l.metrics.begin(), l.metrics.end(), byPrio);
  if (!std::is_sorted(r.metrics.begin(), r.metrics.end(), byPrio))
    std::sort(r.metrics.begin(), r.metrics.end(), byPrio);
  CompareResult res = CompareResult::TIE;
  size_t i = 0, j = 0;
  while (!decisive(res) && i < l.metrics.size() && j < r.metrics.size()) {
    const auto& a = l.metrics[i];
    const auto& b = r.metrics[j];
    if (a.type == b.type) {
      if (a.isBestPathTieBreaker != b.isBestPathTieBreaker) {
        maybeUpdate(res, CompareResult::ERROR);
      } else {
        maybeUpdate(res, compareMetrics(a.metric, b.metric, a.isBestPathTieBreaker));
      }
      ++i;
      ++j;
    } else if (a.priority > b.priority) {
      maybeUpdate(res, loner(a));
      ++i;
    } else if (a.priority < b.priority) {
      maybeUpdate(res, invert(loner(b)));
      ++j;
    } else {
      maybeUpdate(res, CompareResult::ERROR);
    }
  }
  while (!decisive(res) && i < l.metrics.size()) maybeUpdate(res, loner(l.metrics[i++]));
  while (!decisive(res) && j < r.metrics.size())
    maybeUpdate(res, invert(loner(r.metrics[j++])));
  return res;
}

// ---- SpfSolverImpl ------------------------------------------------------------
void SpfSolver::updateStaticUnicastRoutes(
    const std::vector<std::pair<Cidr, std::vector<NextHopThrift>>>& upd,
    const std::vector<Cidr>& del) {  // Decision.cpp:370-394
  for (const auto& [p, nhs] : upd) staticUnicastRoutes_[p] = nhs;
  for (const auto& p : del) staticUnicastRoutes_.erase(p);
}

void SpfSolver::updateStaticMplsRoutes(
    const std::vector<std::pair<int32_t, std::vector<NextHopThrift>>>& upd,
    const std::vector<int32_t>& del) {  // Decision.cpp:396-419
  for (const auto& [l, nhs] : upd) staticMplsRoutes_[l] = nhs;
  for (auto l : del) staticMplsRoutes_.erase(l);
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefixOrGetStaticRoute(
    const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
    const Cidr& prefix) {  // Decision.cpp:421-443
  if (auto r = createRouteForPrefix(me, als, ps, prefix)) return r;
  auto it = staticUnicastRoutes_.find(prefix);
  if (it != staticUnicastRoutes_.end()) {
    RibUnicastEntry e;
    e.prefix = prefix;
    e.nexthops.insert(it->second.begin(), it->second.end());
    return e;
  }
  return std::nullopt;
}

std::optional<RibUnicastEntry> SpfSolver::createRouteForPrefix(const std::string& me,
                                                               const AreaLinkStates& als,
                                                               const PrefixState& ps,
                                                               const Cidr& prefix) {
  // Decision.cpp:445-613
  auto search = ps.prefixes().find(prefix);
  if (search == ps.prefixes().end()) return std::nullopt;

  PrefixEntries entries = search->second;  // copy, then drop unreachable
  for (const auto& [area, ls] : als) {
    const auto& spf = ls.getSpfResult(me);
    for (auto it = entries.begin(); it != entries.end();) {
      const auto& [node, parea] = it->first;
      if (area != parea || spf.count(node)) {
        ++it;
      } else {
        it = entries.erase(it);
      }
    }
  }
  if (entries.empty()) return std::nullopt;
  if (isV4(prefix) && !enableV4_) return std::nullopt;

  bool hasBGP = false, hasNonBGP = false, missingMv = false, hasSelfPrependLabel = true;
  for (const auto& [na, e] : entries) {
    const bool bgp = e.type == BGP;
    hasBGP |= bgp;
    hasNonBGP |= !bgp;
    if (na.first == me) hasSelfPrependLabel &= e.prependLabel.has_value();
    if (bgp && !e.mv) missingMv = true;
  }
  if (hasBGP) {
    if (hasNonBGP && !enableBestRouteSelection_) return std::nullopt;
    if (missingMv) return std::nullopt;
  }

  const auto best = selectBestRoutes(me, prefix, entries, hasBGP, als);
  if (!best.success) return std::nullopt;
  if (best.allNodeAreas.empty()) return std::nullopt;

  if (best.hasNode(me) && !hasSelfPrependLabel) return std::nullopt;

  const auto [ft, fa] = getPrefixForwardingTypeAndAlgorithm(entries, best.allNodeAreas);
  if (fa == FA_SP_ECMP) return selectBestPathsSpf(me, prefix, best, entries, hasBGP, ft, als);
  if (fa == FA_KSP2_ED_ECMP)
    return selectBestPathsKsp2(me, prefix, best, entries, hasBGP, ft, als);
  return std::nullopt;
}

std::optional<DecisionRouteDb> SpfSolver::buildRouteDb(const std::string& me,
                                                       const AreaLinkStates& als,
                                                       const PrefixState& ps) {
  // Decision.cpp:615-792
  bool exists = false;
  for (const auto& [_, ls] : als) exists |= ls.hasNode(me);
  if (!exists) return std::nullopt;
  ++routeBuildRuns;

  DecisionRouteDb db;
  for (const auto& [prefix, _] : ps.prefixes()) {
    if (auto r = createRouteForPrefix(me, als, ps, prefix)) {
      if (!db.unicastRoutes.emplace(prefix, std::move(*r)).second)
        throw std::logic_error("duplicate unicast route");
    }
  }
  for (const auto& [prefix, nhs] : staticUnicastRoutes_) {
    if (db.unicastRoutes.count(prefix)) continue;
    RibUnicastEntry e;
    e.prefix = prefix;
    e.nexthops.insert(nhs.begin(), nhs.end());
    db.unicastRoutes.emplace(prefix, std::move(e));
  }

  // node-label routes (:655-744); duplicate labels: smaller node name wins,
  // except that my own label always (re)claims its slot
  std::unordered_map<int32_t, std::pair<std::string, RibMplsEntry>> labelToNode;
  for (const auto& [area, ls] : als) {
    for (const auto& [_, adjDb] : ls.getAdjacencyDatabases()) {
      const int32_t label = adjDb.nodeLabel;
      if (label == 0) continue;
      if (!isMplsLabelValid(label)) continue;
      auto it = labelToNode.find(label);
      if (it != labelToNode.end() && it->second.first < adjDb.thisNodeName) continue;
      if (adjDb.thisNodeName == me) {
        NextHopThrift nh;
        nh.address.addr = std::string(16, '\0');  // "::"
        nh.area = area;
        nh.mplsAction = mplsAction(POP_AND_LOOKUP);
        RibMplsEntry e{label, {}};
        e.nexthops.insert(nh);
        labelToNode.erase(label);
        labelToNode.emplace(label, std::make_pair(adjDb.thisNodeName, std::move(e)));
        continue;
      }
      std::set<NodeAndArea> dst{{adjDb.thisNodeName, area}};
      auto metricNhs = getNextHopsWithMetric(me, dst, false, als);
      if (metricNhs.second.empty()) continue;  // no route to label
      RibMplsEntry e{label,
                     getNextHopsThrift(me, dst, false, false, metricNhs.first,
                                       metricNhs.second, label, als, {})};
      labelToNode.erase(label);
      labelToNode.emplace(label, std::make_pair(adjDb.thisNodeName, std::move(e)));
    }
  }
  for (auto& [_, ne] : labelToNode) db.mplsRoutes.emplace(ne.second.label, ne.second);

  // adjacency-label routes for all my links, up or not (:749-775)
  for (const auto& [_, ls] : als) {
    for (const auto& link : ls.linksFromNode(me)) {
      const int32_t label = link->getAdjLabelFromNode(me);
      if (label == 0 || !isMplsLabelValid(label)) continue;
      RibMplsEntry e{label, {}};
      e.nexthops.insert(nextHop(link->getNhV6FromNode(me), link->getIfaceFromNode(me),
                                static_cast<int32_t>(link->getMetricFromNode(me)),
                                mplsAction(PHP), link->getArea(),
                                link->getOtherNodeName(me)));
      if (!db.mplsRoutes.emplace(label, std::move(e)).second)
        throw std::logic_error("duplicate mpls route");
    }
  }
  for (const auto& [label, nhs] : staticMplsRoutes_) {  // :780-784
    RibMplsEntry e{label, {}};
    e.nexthops.insert(nhs.begin(), nhs.end());
    if (!db.mplsRoutes.emplace(label, std::move(e)).second)
      throw std::logic_error("duplicate mpls route");
  }
  return db;
}

BestRouteSelectionResult SpfSolver::selectBestRoutes(const std::string& me,
                                                     const Cidr& prefix,
                                                     const PrefixEntries& entries,
                                                     bool isBgp, const AreaLinkStates& als) {
  BestRouteSelectionResult r;  // Decision.cpp:794-822
  if (enableBestRouteSelection_) {
    r.allNodeAreas = selectBestPrefixMetrics(entries);
    r.bestNodeArea = selectBestNodeArea(r.allNodeAreas, me);
    r.success = true;
  } else if (isBgp) {
    r = runBestPathSelectionBgp(me, prefix, entries, als);
  } else {
    for (const auto& [na, _] : entries) r.allNodeAreas.insert(na);
    r.bestNodeArea = *r.allNodeAreas.begin();
    r.success = true;
  }
  return maybeFilterDrainedNodes(std::move(r), als);
}

std::optional<int64_t> SpfSolver::getMinNextHopThreshold(
    const BestRouteSelectionResult& r, const PrefixEntries& entries) const {
  std::optional<int64_t> mx;  // Decision.cpp:824-838
  for (const auto& na : r.allNodeAreas) {
    const auto& e = entries.at(na);
    if (e.minNexthop && (!mx || *e.minNexthop > *mx)) mx = e.minNexthop;
  }
  return mx;
}

BestRouteSelectionResult SpfSolver::maybeFilterDrainedNodes(
    BestRouteSelectionResult&& r, const AreaLinkStates& als) const {
  BestRouteSelectionResult f = r;  // Decision.cpp:840-862
  for (auto it = f.allNodeAreas.begin(); it != f.allNodeAreas.end();) {
    if (als.at(it->second).isNodeOverloaded(it->first)) {
      it = f.allNodeAreas.erase(it);
    } else {
      ++it;
    }
  }
  if (!f.allNodeAreas.empty() && f.bestNodeArea != r.bestNodeArea) {
    f.bestNodeArea = *f.allNodeAreas.begin();
  }
  return f.allNodeAreas.empty() ? r : f;
}

BestRouteSelectionResult SpfSolver::runBestPathSelectionBgp(const std::string& me,
                                                            const Cidr& prefix,
                                                            const PrefixEntries& entries,
                                                            const AreaLinkStates& als) {
  BestRouteSelectionResult r;  // Decision.cpp:864-902
  std::optional<MetricVector> bestVector;
  for (const auto& [na, e] : entries) {
    const MetricVector& mv = e.mv.value();
    const CompareResult c =
        bestVector ? compareMetricVectors(mv, *bestVector) : CompareResult::WINNER;
    switch (c) {
      case CompareResult::WINNER:
        r.allNodeAreas.clear();
        [[fallthrough]];
      case CompareResult::TIE_WINNER:
        bestVector = mv;
        r.bestNodeArea = na;
        [[fallthrough]];
      case CompareResult::TIE_LOOSER:
        r.allNodeAreas.insert(na);
        break;
      case CompareResult::TIE:
      case CompareResult::ERROR:
        return r;  // success stays false: route skipped
      default:
        break;
    }
  }
  r.success = true;
  return maybeFilterDrainedNodes(std::move(r), als);
}

std::optional<RibUnicastEntry> SpfSolver::selectBestPathsSpf(
    const std::string& me, const Cidr& prefix, const BestRouteSelectionResult& r,
    const PrefixEntries& entries, bool isBgp, int32_t ft, const AreaLinkStates& als) {
  // Decision.cpp:904-963
  const bool v4 = isV4(prefix);
  const bool perDst = ft == FT_SR_MPLS;
  auto filtered = r.allNodeAreas;
  if (r.hasNode(me) && perDst) {
    for (const auto& [na, e] : entries) {
      if (na.first == me && e.prependLabel) {
        filtered.erase(na);
        break;
      }
    }
  }
  auto nhm = getNextHopsWithMetric(me, filtered, perDst, als);
  if (nhm.second.empty()) return std::nullopt;
  return addBestPaths(me, prefix, r, entries, isBgp,
                      getNextHopsThrift(me, r.allNodeAreas, v4, perDst, nhm.first,
                                        nhm.second, std::nullopt, als, entries));
}

std::optional<RibUnicastEntry> SpfSolver::selectBestPathsKsp2(
    const std::string& me, const Cidr& prefix, const BestRouteSelectionResult& r,
    const PrefixEntries& entries, bool isBgp, int32_t ft, const AreaLinkStates& als) {
  // Decision.cpp:965-1087
  if (ft != FT_SR_MPLS) return std::nullopt;
  NextHopSet nexthops;
  std::vector<Path> paths;
  for (const auto& [area, ls] : als) {
    for (const auto& [node, bestArea] : r.allNodeAreas) {
      if (node == me && bestArea == area) continue;
      for (const auto& p : ls.getKthPaths(me, node, 1)) paths.push_back(p);
    }
    const size_t firstPaths = paths.size();
    for (const auto& [node, bestArea] : r.allNodeAreas) {
      if (area != bestArea) continue;
      for (const auto& sp : ls.getKthPaths(me, node, 2)) {
        bool add = true;
        for (size_t i = 0; i < firstPaths; ++i) {
          if (LinkState::pathAInPathB(paths[i], sp)) {
            add = false;
            break;
          }
        }
        if (add) paths.push_back(sp);
      }
    }
  }
  if (paths.empty()) return std::nullopt;

  for (const auto& path : paths) {
    for (const auto& [area, ls] : als) {
      Metric cost = 0;
      std::list<int32_t> labels;
      std::string next = me;
      for (const auto& link : path) {
        cost += link->getMetricFromNode(next);
        next = link->getOtherNodeName(next);
        labels.push_front(ls.getAdjacencyDatabases().at(next).nodeLabel);
      }
      labels.pop_back();  // PHP: drop the first hop's label
      const auto& pe = entries.at({next, area});
      if (pe.prependLabel) labels.push_front(*pe.prependLabel);
      const auto& first = path.front();
      std::optional<MplsAction> act;
      if (!labels.empty())
        act = mplsAction(PUSH, std::nullopt,
                         std::vector<int32_t>(labels.begin(), labels.end()));
      nexthops.insert(nextHop(isV4(prefix) ? first->getNhV4FromNode(me)
                                           : first->getNhV6FromNode(me),
                              first->getIfaceFromNode(me), static_cast<int32_t>(cost), act,
                              first->getArea(), first->getOtherNodeName(me)));
    }
  }
  return addBestPaths(me, prefix, r, entries, isBgp, std::move(nexthops));
}

std::optional<RibUnicastEntry> SpfSolver::addBestPaths(const std::string& me,
                                                       const Cidr& prefix,
                                                       const BestRouteSelectionResult& r,
                                                       const PrefixEntries& entries,
                                                       bool isBgp, NextHopSet&& nexthops) {
  // Decision.cpp:1089-1150
  auto minNh = getMinNextHopThreshold(r, entries);
  if (minNh && *minNh > static_cast<int64_t>(nexthops.size())) return std::nullopt;
  if (r.hasNode(me)) {
    std::optional<int32_t> prepend;
    for (const auto& [na, e] : entries) {
      if (na.first == me && e.prependLabel) {
        prepend = e.prependLabel;
        break;
      }
    }
    if (!prepend) throw std::logic_error("self route without prepend label");
    auto it = staticMplsRoutes_.find(*prepend);
    if (it != staticMplsRoutes_.end()) {
      for (const auto& nh : it->second) {
        nexthops.insert(nextHop(nh.address, std::nullopt, 0, std::nullopt, std::nullopt,
                                std::nullopt));
      }
    }
  }
  RibUnicastEntry e;
  e.prefix = prefix;
  e.nexthops = std::move(nexthops);
  e.bestPrefixEntry = entries.at(r.bestNodeArea);
  e.bestArea = r.bestNodeArea.second;
  e.doNotInstall = isBgp && bgpDryRun_;
  return e;
}

std::pair<Metric, std::unordered_set<std::string>> SpfSolver::getMinCostNodes(
    const SpfResult& spf, const std::set<NodeAndArea>& dsts) {
  Metric best = std::numeric_limits<Metric>::max();  // Decision.cpp:1152-1175
  std::unordered_set<std::string> nodes;
  for (const auto& [dst, _] : dsts) {  // area deliberately ignored
    auto it = spf.find(dst);
    if (it == spf.end()) continue;
    const Metric d = it->second.metric();
    if (best >= d) {
      if (best > d) {
        best = d;
        nodes.clear();
      }
      nodes.insert(dst);
    }
  }
  return {best, std::move(nodes)};
}

std::pair<Metric, std::unordered_map<SpfSolver::NhKey, Metric, PairStrHash>>
SpfSolver::getNextHopsWithMetric(const std::string& me, const std::set<NodeAndArea>& dsts,
                                 bool perDst, const AreaLinkStates& als) const {
  // Decision.cpp:1177-1228
  std::unordered_map<NhKey, Metric, PairStrHash> nhs;
  Metric shortest = std::numeric_limits<Metric>::max();
  for (const auto& [area, ls] : als) {
    const auto& spf = ls.getSpfResult(me);
    auto mc = getMinCostNodes(spf, dsts);
    if (shortest < mc.first) continue;
    if (shortest > mc.first) {
      shortest = mc.first;
      nhs.clear();
    }
    if (mc.second.empty()) continue;
    for (const auto& dst : mc.second) {
      const std::string dstRef = perDst ? dst : "";
      for (const auto& nh : spf.at(dst).nextHops()) {
        nhs[{nh, dstRef}] = shortest - *ls.getMetricFromAToB(me, nh);
      }
    }
  }
  return {shortest, std::move(nhs)};
}

NextHopSet SpfSolver::getNextHopsThrift(
    const std::string& me, const std::set<NodeAndArea>& dsts, bool v4, bool perDst,
    Metric minMetric, const std::unordered_map<NhKey, Metric, PairStrHash>& nhs,
    std::optional<int32_t> swapLabel, const AreaLinkStates& als,
    const PrefixEntries& entries) const {
  // Decision.cpp:1230-1334
  if (nhs.empty()) throw std::logic_error("empty nexthop nodes");
  NextHopSet out;
  const std::set<NodeAndArea> noDst{{"", ""}};
  for (const auto& [area, ls] : als) {
    for (const auto& link : ls.linksFromNode(me)) {
      for (const auto& [dst, dstArea] : perDst ? dsts : noDst) {
        if (!dstArea.empty() && area != dstArea) continue;
        const std::string nbr = link->getOtherNodeName(me);
        auto it = nhs.find({nbr, dst});
        if (it == nhs.end() || !link->isUp()) continue;
        if (!dst.empty() && dsts.count({nbr, area}) && nbr != dst) continue;
        const Metric overLink = link->getMetricFromNode(me) + it->second;
        if (overLink != minMetric) continue;

        std::optional<MplsAction> act;
        if (swapLabel) {
          const bool nhIsDst = dsts.count({nbr, area}) != 0;
          act = nhIsDst ? mplsAction(PHP) : mplsAction(SWAP, swapLabel);
        }
        if (!dst.empty()) {
          std::vector<int32_t> push;
          const auto& dpe = entries.at({dst, area});
          if (dpe.prependLabel) {
            push.push_back(*dpe.prependLabel);
            if (!isMplsLabelValid(push.back())) continue;
          }
          if (dst != nbr) {
            push.push_back(ls.getAdjacencyDatabases().at(dst).nodeLabel);
            if (!isMplsLabelValid(push.back())) continue;
          }
          if (!push.empty()) act = mplsAction(PUSH, std::nullopt, std::move(push));
        }
        out.insert(nextHop(v4 ? link->getNhV4FromNode(me) : link->getNhV6FromNode(me),
                           link->getIfaceFromNode(me), static_cast<int32_t>(overLink), act,
                           link->getArea(), nbr));
      }
    }
  }
  return out;
}

}  // namespace oracle
