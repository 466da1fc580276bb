// Drop-in RibPolicy (openr/decision/RibPolicy.{h,cpp}): UCMP weights applied
// to the unicast routes of a built DecisionRouteDb.
//
// A statement matches a route when every populated matcher matches (prefix
// set: the route's prefix; tag set: any tag of the route's best prefix
// entry) and at least one matcher is populated (RibPolicy.cpp:73-105). Its
// set_weight action gives each nexthop the neighbour weight, else the area
// weight, else the default weight; weight 0 drops the nexthop, and a route
// whose nexthops would all be dropped is kept unchanged
// (RibPolicy.cpp:108-161). A policy applies the first matching statement per
// route and only while its TTL has not expired (RibPolicy.cpp:215-247).
#pragma once

#include <chrono>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "host_types.h"

namespace openr_amd {

struct RibRouteActionWeight {  // OpenrCtrl.thrift RibRouteActionWeight
  int32_t defaultWeight{0};
  std::map<std::string, int32_t> areaToWeight;
  std::map<std::string, int32_t> neighborToWeight;
};

struct RibPolicyStatementSpec {  // thrift::RibPolicyStatement
  std::string name;
  std::optional<std::vector<Cidr>> prefixes;      // matcher.prefixes
  std::optional<std::vector<std::string>> tags;   // matcher.tags
  std::optional<RibRouteActionWeight> setWeight;  // action.set_weight
};

class RibPolicyStatement {
 public:
  explicit RibPolicyStatement(const RibPolicyStatementSpec& spec);  // throws std::invalid_argument
  bool match(const RibUnicastEntry& route) const;
  bool applyAction(RibUnicastEntry& route, uint64_t* invalidated = nullptr) const;
  const std::string& name() const { return name_; }
  // the set_weight action for one nexthop: neighbour weight, else area
  // weight, else the default weight (RibPolicy.cpp:118-134)
  int32_t weightOf(const std::optional<std::string>& area,
                   const std::optional<std::string>& neighbor) const;
  const std::set<Cidr>& prefixSet() const { return prefixSet_; }
  const std::set<std::string>& tagSet() const { return tagSet_; }

 private:
  std::string name_;
  RibRouteActionWeight action_;
  std::set<Cidr> prefixSet_;
  std::set<std::string> tagSet_;
  uint64_t id_{nextGeneration()};  // names the statement in the nexthop memo
};

class RibPolicy {
 public:
  struct PolicyChange {
    std::vector<Cidr> updatedRoutes;
    std::vector<Cidr> deletedRoutes;
  };

  RibPolicy(const std::vector<RibPolicyStatementSpec>& statements, int64_t ttlSecs);
  bool isActive() const { return getTtlDuration().count() > 0; }
  std::chrono::milliseconds getTtlDuration() const;
  bool match(const RibUnicastEntry& route) const;
  bool applyAction(RibUnicastEntry& route);
  // the same, counting invalidated routes into *invalidated (thread-safe for
  // distinct routes and counters)
  bool applyAction(RibUnicastEntry& route, uint64_t* invalidated) const;
  PolicyChange applyPolicy(UnicastRouteMap& routes);
  // the same over a DecisionRouteUpdate's routes (Decision.cpp:1912-1924)
  PolicyChange applyPolicy(std::unordered_map<Cidr, RibUnicastEntry, CidrHash>& routes);
  const std::vector<RibPolicyStatement>& statements() const { return statements_; }
  // decision.rib_policy.invalidated_routes (RibPolicy.cpp:150-153)
  uint64_t invalidatedRoutes() const { return invalidated_; }
  void addInvalidated(uint64_t n) { invalidated_ += n; }
  // process-unique id of this policy (caches record it, not the address)
  uint64_t generation() const { return generation_; }

 private:
  uint64_t generation_{nextGeneration()};
  std::chrono::steady_clock::time_point validUntil_;
  std::vector<RibPolicyStatement> statements_;
  uint64_t invalidated_{0};
};

}  // namespace openr_amd
