// TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle_types.h header).
//
// Restatement of the route-computation half of the Decision module:
//   PrefixState                 openr/decision/PrefixState.{h,cpp}
//   RibUnicastEntry / RibMplsEntry / DecisionRouteDb
//                               openr/decision/RibEntry.h, Decision.h:78-119
//   SpfSolver::SpfSolverImpl    openr/decision/Decision.cpp:161-1391
//   MetricVectorUtils           openr/common/Util.cpp:915-1094
#pragma once

#include <set>
#include <unordered_map>
#include <unordered_set>

#include "oracle_link_state.h"

namespace oracle {

using PrefixEntries = std::unordered_map<NodeAndArea, PrefixEntry, PairStrHash>;

class PrefixState {  // PrefixState.h:22-70
 public:
  std::unordered_set<Cidr, CidrHash> updatePrefix(const std::string& node,
                                                  const std::string& area,
                                                  const PrefixEntry& e);
  std::unordered_set<Cidr, CidrHash> deletePrefix(const std::string& node,
                                                  const std::string& area,
                                                  const Cidr& prefix);
  const std::unordered_map<Cidr, PrefixEntries, CidrHash>& prefixes() const {
    return prefixes_;
  }

 private:
  std::unordered_map<Cidr, PrefixEntries, CidrHash> prefixes_;
};

using NextHopSet = std::unordered_set<NextHopThrift, NextHopHash>;

struct RibUnicastEntry {  // RibEntry.h:38-99
  Cidr prefix;
  NextHopSet nexthops;
  std::optional<PrefixEntry> bestPrefixEntry;
  std::string bestArea;
  bool doNotInstall{false};
};

// RibEntry.h:65-69 (bestArea is not compared) and RibEntry.h:28-31
inline bool operator==(const RibUnicastEntry& a, const RibUnicastEntry& b) {
  if (!(a.prefix == b.prefix && a.doNotInstall == b.doNotInstall)) return false;
  if (a.bestPrefixEntry.has_value() != b.bestPrefixEntry.has_value()) return false;
  if (a.bestPrefixEntry && !(*a.bestPrefixEntry == *b.bestPrefixEntry)) return false;
  return a.nexthops == b.nexthops;
}

struct RibMplsEntry {  // RibEntry.h:101-144
  int32_t label{0};
  NextHopSet nexthops;
};

inline bool operator==(const RibMplsEntry& a, const RibMplsEntry& b) {  // RibEntry.h:123-126
  return a.label == b.label && a.nexthops == b.nexthops;
}

struct DecisionRouteUpdate {  // RouteUpdate.h:23-41
  std::unordered_map<Cidr, RibUnicastEntry, CidrHash> unicastRoutesToUpdate;
  std::vector<Cidr> unicastRoutesToDelete;
  std::vector<RibMplsEntry> mplsRoutesToUpdate;
  std::vector<int32_t> mplsRoutesToDelete;
};

struct DecisionRouteDb {  // Decision.h:78-119
  std::unordered_map<Cidr, RibUnicastEntry, CidrHash> unicastRoutes;
  std::unordered_map<int32_t, RibMplsEntry> mplsRoutes;

  // Decision.cpp:108-143
  DecisionRouteUpdate calculateUpdate(DecisionRouteDb&& newDb) const {
    DecisionRouteUpdate delta;
    for (auto& kv : newDb.unicastRoutes) {
      auto search = unicastRoutes.find(kv.first);
      if (search == unicastRoutes.end() || !(search->second == kv.second)) {
        auto key = kv.second.prefix;
        delta.unicastRoutesToUpdate.emplace(std::move(key), std::move(kv.second));
      }
    }
    for (auto& kv : unicastRoutes)
      if (!newDb.unicastRoutes.count(kv.first)) delta.unicastRoutesToDelete.emplace_back(kv.first);
    for (const auto& kv : newDb.mplsRoutes) {
      auto search = mplsRoutes.find(kv.first);
      if (search == mplsRoutes.end() || !(search->second == kv.second))
        delta.mplsRoutesToUpdate.emplace_back(kv.second);
    }
    for (const auto& kv : mplsRoutes)
      if (!newDb.mplsRoutes.count(kv.first)) delta.mplsRoutesToDelete.emplace_back(kv.first);
    return delta;
  }

  // Decision.cpp:146-160
  void update(const DecisionRouteUpdate& u) {
    for (const auto& prefix : u.unicastRoutesToDelete) unicastRoutes.erase(prefix);
    for (const auto& kv : u.unicastRoutesToUpdate) unicastRoutes.insert_or_assign(kv.second.prefix, kv.second);
    for (auto label : u.mplsRoutesToDelete) mplsRoutes.erase(label);
    for (const auto& e : u.mplsRoutesToUpdate) mplsRoutes.insert_or_assign(e.label, e);
  }
};

struct BestRouteSelectionResult {  // Decision.h:51-76
  bool success{false};
  std::set<NodeAndArea> allNodeAreas;
  NodeAndArea bestNodeArea;
  bool hasNode(const std::string& n) const {
    for (auto& na : allNodeAreas)
      if (na.first == n) return true;
    return false;
  }
};

using AreaLinkStates = std::unordered_map<std::string, LinkState>;

class SpfSolver {
 public:
  SpfSolver(const std::string& myNodeName, bool enableV4, bool enableOrderedFib = false,
            bool bgpDryRun = false, bool enableBestRouteSelection = false)
      : myNodeName_(myNodeName),
        enableV4_(enableV4),
        enableOrderedFib_(enableOrderedFib),
        bgpDryRun_(bgpDryRun),
        enableBestRouteSelection_(enableBestRouteSelection) {}

  void updateStaticUnicastRoutes(
      const std::vector<std::pair<Cidr, std::vector<NextHopThrift>>>& upd,
      const std::vector<Cidr>& del);
  void updateStaticMplsRoutes(
      const std::vector<std::pair<int32_t, std::vector<NextHopThrift>>>& upd,
      const std::vector<int32_t>& del);

  std::optional<DecisionRouteDb> buildRouteDb(const std::string& me,
                                              const AreaLinkStates& als,
                                              const PrefixState& ps);
  std::optional<RibUnicastEntry> createRouteForPrefixOrGetStaticRoute(
      const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
      const Cidr& prefix);

 private:
  std::optional<RibUnicastEntry> createRouteForPrefix(const std::string& me,
                                                      const AreaLinkStates& als,
                                                      const PrefixState& ps,
                                                      const Cidr& prefix);
  BestRouteSelectionResult selectBestRoutes(const std::string& me, const Cidr& prefix,
                                            const PrefixEntries& entries, bool isBgp,
                                            const AreaLinkStates& als);
  BestRouteSelectionResult runBestPathSelectionBgp(const std::string& me,
                                                   const Cidr& prefix,
                                                   const PrefixEntries& entries,
                                                   const AreaLinkStates& als);
  BestRouteSelectionResult maybeFilterDrainedNodes(BestRouteSelectionResult&& r,
                                                   const AreaLinkStates& als) const;
  std::optional<int64_t> getMinNextHopThreshold(const BestRouteSelectionResult& r,
                                                const PrefixEntries& entries) const;
  std::optional<RibUnicastEntry> selectBestPathsSpf(
      const std::string& me, const Cidr& prefix, const BestRouteSelectionResult& r,
      const PrefixEntries& entries, bool isBgp, int32_t fwdType,
      const AreaLinkStates& als);
  std::optional<RibUnicastEntry> selectBestPathsKsp2(
      const std::string& me, const Cidr& prefix, const BestRouteSelectionResult& r,
      const PrefixEntries& entries, bool isBgp, int32_t fwdType,
      const AreaLinkStates& als);
  std::optional<RibUnicastEntry> addBestPaths(const std::string& me, const Cidr& prefix,
                                              const BestRouteSelectionResult& r,
                                              const PrefixEntries& entries, bool isBgp,
                                              NextHopSet&& nexthops);

 public:
  using NhKey = std::pair<std::string, std::string>;  // (nexthop node, dst or "")
  static std::pair<Metric, std::unordered_set<std::string>> getMinCostNodes(
      const SpfResult& spf, const std::set<NodeAndArea>& dsts);
  std::pair<Metric, std::unordered_map<NhKey, Metric, PairStrHash>> getNextHopsWithMetric(
      const std::string& me, const std::set<NodeAndArea>& dsts, bool perDestination,
      const AreaLinkStates& als) const;
  NextHopSet getNextHopsThrift(const std::string& me, const std::set<NodeAndArea>& dsts,
                               bool isV4, bool perDestination, Metric minMetric,
                               const std::unordered_map<NhKey, Metric, PairStrHash>& nhs,
                               std::optional<int32_t> swapLabel,
                               const AreaLinkStates& als,
                               const PrefixEntries& entries) const;

  // fb303 counter restatements
  uint64_t routeBuildRuns{0};

 private:
  std::unordered_map<int32_t, std::vector<NextHopThrift>> staticMplsRoutes_;
  std::unordered_map<Cidr, std::vector<NextHopThrift>, CidrHash> staticUnicastRoutes_;
  std::string myNodeName_;
  bool enableV4_, enableOrderedFib_, bgpDryRun_, enableBestRouteSelection_;
};

// Util.h:491-526 / Util.cpp:452-480 / Util.cpp:902-913
std::set<NodeAndArea> selectBestPrefixMetrics(const PrefixEntries& entries);
NodeAndArea selectBestNodeArea(const std::set<NodeAndArea>& all, const std::string& me);
std::pair<int32_t, int32_t> getPrefixForwardingTypeAndAlgorithm(
    const PrefixEntries& entries, const std::set<NodeAndArea>& best);

enum class CompareResult { WINNER, TIE_WINNER, TIE, TIE_LOOSER, LOOSER, ERROR };
CompareResult compareMetricVectors(MetricVector l, MetricVector r);

}  // namespace oracle
