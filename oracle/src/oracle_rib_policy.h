// TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle_types.h header).
//
// Restatement of openr/decision/RibPolicy.{h,cpp} (RibPolicy.cpp:19-247) with
// the reference's containers: unordered sets for the prefix and tag
// matchers, a fresh unordered_set<NextHopThrift> per transformed route, the
// statements tried in order, the invalidated-routes stat as a counter.
#pragma once

#include <chrono>
#include <map>
#include <unordered_set>

#include "oracle_decision.h"

namespace oracle {

struct RibRouteActionWeight {  // OpenrCtrl.thrift RibRouteActionWeight
  int32_t default_weight{0};
  std::map<std::string, int32_t> area_to_weight;
  std::map<std::string, int32_t> neighbor_to_weight;
};

struct RibPolicyStatementSpec {  // thrift::RibPolicyStatement (matcher + action)
  std::string name;
  std::optional<std::vector<Cidr>> prefixes;
  std::optional<std::vector<std::string>> tags;
  std::optional<RibRouteActionWeight> set_weight;
};

class RibPolicyStatement {  // RibPolicy.h RibPolicyStatement
 public:
  explicit RibPolicyStatement(const RibPolicyStatementSpec& stmt);  // throws std::invalid_argument
  bool match(const RibUnicastEntry& route) const;
  bool applyAction(RibUnicastEntry& route, uint64_t& invalidatedStat) const;

 private:
  std::string name_;
  std::unordered_set<Cidr, CidrHash> prefixSet_;
  std::unordered_set<std::string> tagSet_;
  RibRouteActionWeight action_;
};

class RibPolicy {  // RibPolicy.h RibPolicy
 public:
  RibPolicy(const std::vector<RibPolicyStatementSpec>& statements, int64_t ttlSecs);
  std::chrono::milliseconds getTtlDuration() const;
  bool isActive() const;
  bool match(const RibUnicastEntry& route) const;
  bool applyAction(RibUnicastEntry& route);
  struct PolicyChange {
    std::vector<Cidr> updatedRoutes, deletedRoutes;
  };
  PolicyChange applyPolicy(std::unordered_map<Cidr, RibUnicastEntry, CidrHash>& unicastEntries);
  // fb303 "decision.rib_policy.invalidated_routes" (RibPolicy.cpp:149-150)
  uint64_t invalidatedRoutes() const { return invalidated_; }

 private:
  std::vector<RibPolicyStatement> policyStatements_;
  std::chrono::steady_clock::time_point validUntilTs_;
  uint64_t invalidated_{0};
};

}  // namespace oracle
