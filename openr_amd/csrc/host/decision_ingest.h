// KvStore -> Decision ingest: Decision::processPublication
// (openr/decision/Decision.cpp:1682-1824) over the drop-in LinkState /
// PrefixState, so publications turn straight into device-mirror deltas (the
// next SPF or route build flushes the changed CSR rows and dirty prefixes).
//
// A publication arrives as thrift Compact bytes (thrift::Publication,
// Types.thrift:897-936; values are Compact-encoded AdjacencyDatabase /
// PrefixDatabase, Types.thrift:144-180, :431-460) or as decoded structs.
// Keys: "adj:<node>" adjacency databases, "prefix:<node>:<area>:[<addr>/<len>]"
// prefix databases (Constants.h:209-212, PrefixKey Types.cpp:43-77),
// "fibtime:<node>" Fib programming times. DecisionPendingUpdates follows
// Decision.cpp:40-100 (perf events are not carried).
#pragma once

#include <optional>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "rib_policy.h"
#include "spf_solver.h"

namespace openr_amd {

struct KvValue {  // thrift::Value (Types.thrift:555-605)
  int64_t version{0};
  std::string originatorId;
  std::optional<std::string> value;  // unset: a TTL refresh
  int64_t ttl{0};
  int64_t ttlVersion{0};
  std::optional<int64_t> hash;
};

struct Publication {  // thrift::Publication (Types.thrift:897-936), the fields Decision reads
  std::unordered_map<std::string, KvValue> keyVals;
  std::vector<std::string> expiredKeys;
  std::string area;
};

Publication publicationFromCompact(const std::string& bytes);
std::string publicationToCompact(const Publication& pub);  // encoder (tests, tools)

// PrefixKey::fromStr (Types.cpp:57-77): node, area and masked prefix of a
// "prefix:" key; nullopt when the key does not parse
struct PrefixKeyParts {
  std::string node, area;
  Cidr prefix;
};
std::optional<PrefixKeyParts> parsePrefixKey(const std::string& key);
// getNodeNameFromKey (Util.cpp:891-899): the second ':'-separated field
std::string nodeNameFromKey(const std::string& key);

class DecisionPendingUpdates {  // Decision.h:128-200
 public:
  explicit DecisionPendingUpdates(std::string myNodeName) : me_(std::move(myNodeName)) {}
  bool needsFullRebuild() const { return fullRebuild_; }
  bool needsRouteUpdate() const { return fullRebuild_ || !updatedPrefixes_.empty(); }
  const std::unordered_set<Cidr, CidrHash>& updatedPrefixes() const { return updatedPrefixes_; }
  uint32_t count() const { return count_; }
  void applyLinkStateChange(const std::string& node, const LinkStateChange& c) {
    fullRebuild_ |= c.topologyChanged || c.nodeLabelChanged || (c.linkAttributesChanged && node == me_);
    ++count_;
  }
  void applyPrefixStateChange(const std::vector<Cidr>& changed) {
    updatedPrefixes_.insert(changed.begin(), changed.end());
    ++count_;
  }
  void reset() {
    count_ = 0;
    fullRebuild_ = false;
    updatedPrefixes_.clear();
  }

 private:
  std::string me_;
  uint32_t count_{0};
  bool fullRebuild_{false};
  std::unordered_set<Cidr, CidrHash> updatedPrefixes_;
};

struct IngestStats {  // fb303 decision.adj_db_update / prefix_db_update / error counters
  uint64_t adjDbUpdates{0}, prefixDbUpdates{0}, errors{0}, ttlRefreshes{0};
};

// Decision::processPublication. areaLinkStates gains the publication's area
// on first sight (on the context of `lane`, see laneContext); orderedFib
// computes hold TTLs from `me`'s hop counts (Decision.cpp:1715-1723).
void processPublication(const Publication& pub, const std::string& me, bool orderedFib,
                        AreaLinkStates& areaLinkStates, PrefixState& prefixState,
                        DecisionPendingUpdates& pending,
                        std::unordered_map<std::string, int64_t>& fibTimes, IngestStats& stats,
                        unsigned lane = 0);

// Decision's route database and Decision::rebuildRoutes (Decision.cpp:1865-1930):
// a full rebuild (buildRouteDb, RibPolicy, calculateUpdate against the
// previous database) when the pending updates need one, else only the
// updated prefixes (createRouteForPrefixOrGetStaticRoute, here batched over
// one device selection pass); the database takes the update either way.
class DecisionRib {
 public:
  DecisionRouteUpdate rebuildRoutes(SpfSolver& solver, const std::string& me,
                                    const AreaLinkStates& als, const PrefixState& ps,
                                    bool fullRebuild, const std::vector<Cidr>& updatedPrefixes,
                                    RibPolicy* policy);
  DecisionRouteUpdate rebuildRoutes(SpfSolver& solver, const std::string& me,
                                    const AreaLinkStates& als, const PrefixState& ps,
                                    DecisionPendingUpdates& pending, RibPolicy* policy);
  const DecisionRouteDb& routeDb() const { return routeDb_; }
  // full rebuilds that ran as a delta against routeDb_ (SpfSolver::
  // buildRouteDelta) / as a whole build (tests, A/B)
  uint64_t deltaRebuilds() const { return deltaRebuilds_; }
  uint64_t wholeRebuilds() const { return wholeRebuilds_; }

 private:
  DecisionRouteDb routeDb_;
  // what routeDb_ was last made from: the solver's selection snapshot, the
  // prefix state (instance and stamp), the policy and its state, the static
  // routes. Every one is a process-unique generation (nextGeneration()), not
  // an address: an object freed and another allocated in its place cannot
  // pass for it
  uint64_t selGen_{0}, psId_{0}, psStamp_{0}, staticEpoch_{0}, policyId_{0};
  bool policyActive_{false};
  uint64_t deltaRebuilds_{0}, wholeRebuilds_{0};
};

}  // namespace openr_amd
