// Drop-in SpfSolver (the pimpl seam of openr/decision/Decision.h:200-251)
// and PrefixState (openr/decision/PrefixState.h:22-70) over device SPF rows.
//
// buildRouteDb follows SpfSolver::SpfSolverImpl (Decision.cpp:615-792): per
// prefix reachability filter, best-route selection, SP_ECMP or KSP2
// nexthops, MPLS node-label and adjacency-label routes, static routes. The
// shortest-path inputs are the SpfRow of `me` per area, computed on the GPU
// by LinkState::getSpfResult; first-hop sets are bitmasks, so the per-prefix
// getMinCostNodes / getNextHopsWithMetric step is a min-reduction plus a
// mask OR instead of string-set unions.
#pragma once

#include <set>

#include "link_state.h"

namespace openr_amd {

using PrefixEntries = std::unordered_map<NodeAndArea, PrefixEntry, StrPairHash>;

class PrefixState {
 public:
  std::vector<Cidr> updatePrefix(const std::string& node, const std::string& area,
                                 const PrefixEntry& e);
  std::vector<Cidr> deletePrefix(const std::string& node, const std::string& area,
                                 const Cidr& prefix);
  const std::unordered_map<Cidr, PrefixEntries, CidrHash>& prefixes() const { return prefixes_; }
  // advertisements with forwardingAlgorithm KSP2_ED_ECMP (lets buildRouteDb
  // skip its KSP2 planning pass when there are none)
  size_t ksp2Entries() const { return ksp2Entries_; }

 private:
  std::unordered_map<Cidr, PrefixEntries, CidrHash> prefixes_;
  size_t ksp2Entries_{0};
};

// unordered_map<string, LinkState>; nodes are stable so LinkState can stay
// non-movable (it owns a device graph)
using AreaLinkStates = std::unordered_map<std::string, LinkState>;

struct BestRouteSelectionResult {
  bool success{false};
  std::set<NodeAndArea> allNodeAreas;
  NodeAndArea bestNodeArea;
  bool hasNode(const std::string& n) const {
    for (const auto& na : allNodeAreas)
      if (na.first == n) return true;
    return false;
  }
};

class SpfSolver {
 public:
  SpfSolver(const std::string& myNodeName, bool enableV4, bool enableOrderedFib = false,
            bool bgpDryRun = false, bool enableBestRouteSelection = false);

  void updateStaticUnicastRoutes(
      const std::vector<std::pair<Cidr, std::vector<NextHopThrift>>>& upd,
      const std::vector<Cidr>& del);
  void updateStaticMplsRoutes(
      const std::vector<std::pair<int32_t, std::vector<NextHopThrift>>>& upd,
      const std::vector<int32_t>& del);

  std::optional<DecisionRouteDb> buildRouteDb(const std::string& me, const AreaLinkStates& als,
                                              const PrefixState& ps);
  std::optional<RibUnicastEntry> createRouteForPrefixOrGetStaticRoute(
      const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
      const Cidr& prefix);

  uint64_t routeBuildRuns() const { return routeBuildRuns_; }

 private:
  using NhKey = std::pair<std::string, std::string>;
  using NhMap = std::unordered_map<NhKey, Metric, StrPairHash>;

  std::optional<RibUnicastEntry> createRouteForPrefix(const std::string& me,
                                                      const AreaLinkStates& als,
                                                      const PrefixState& ps, const Cidr& prefix);
  BestRouteSelectionResult selectBestRoutes(const std::string& me,
                                            const PrefixEntries& entries, bool isBgp,
                                            const AreaLinkStates& als) const;
  BestRouteSelectionResult runBestPathSelectionBgp(const PrefixEntries& entries,
                                                   const AreaLinkStates& als) const;
  BestRouteSelectionResult filterDrained(BestRouteSelectionResult&& r,
                                         const AreaLinkStates& als) const;
  std::optional<RibUnicastEntry> selectBestPathsSpf(const std::string& me, const Cidr& prefix,
                                                    const BestRouteSelectionResult& r,
                                                    const PrefixEntries& entries, bool isBgp,
                                                    int32_t fwdType, const AreaLinkStates& als);
  std::optional<RibUnicastEntry> selectBestPathsKsp2(const std::string& me, const Cidr& prefix,
                                                     const BestRouteSelectionResult& r,
                                                     const PrefixEntries& entries, bool isBgp,
                                                     int32_t fwdType, const AreaLinkStates& als);
  std::optional<RibUnicastEntry> addBestPaths(const std::string& me, const Cidr& prefix,
                                              const BestRouteSelectionResult& r,
                                              const PrefixEntries& entries, bool isBgp,
                                              NextHopSet&& nexthops);
  std::pair<Metric, NhMap> getNextHopsWithMetric(const std::string& me,
                                                 const std::set<NodeAndArea>& dsts, bool perDst,
                                                 const AreaLinkStates& als) const;
  NextHopSet getNextHopsThrift(const std::string& me, const std::set<NodeAndArea>& dsts,
                               bool isV4, bool perDst, Metric minMetric, const NhMap& nhs,
                               std::optional<int32_t> swapLabel, const AreaLinkStates& als,
                               const PrefixEntries* entries) const;
  // single-area, IP-forwarded SP_ECMP: min-reduction + mask OR on the row
  bool fastSpEcmp(const std::string& me, const LinkState& ls, const std::string& area,
                  const std::set<NodeAndArea>& dsts, bool isV4, std::optional<int32_t> swapLabel,
                  NextHopSet& out) const;

  std::unordered_map<int32_t, std::vector<NextHopThrift>> staticMplsRoutes_;
  std::unordered_map<Cidr, std::vector<NextHopThrift>, CidrHash> staticUnicastRoutes_;
  std::string myNodeName_;
  bool enableV4_, enableOrderedFib_, bgpDryRun_, enableBestRouteSelection_;
  uint64_t routeBuildRuns_{0};
  // set during buildRouteDb's KSP2 planning pass (see buildRouteDb)
  std::unordered_map<const LinkState*, std::vector<std::pair<std::string, std::string>>>* kspPlan_{
      nullptr};
};

}  // namespace openr_amd
