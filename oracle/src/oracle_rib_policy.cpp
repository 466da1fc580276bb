// TEST INFRASTRUCTURE ONLY — CPU oracle: RibPolicy (see oracle_rib_policy.h).
#include "oracle_rib_policy.h"

#include <stdexcept>

namespace oracle {

// RibPolicy.cpp:19-49: an action and a matcher are mandatory (thrift
// OpenrError there, std::invalid_argument here)
RibPolicyStatement::RibPolicyStatement(const RibPolicyStatementSpec& stmt) : name_(stmt.name) {
  if (!stmt.set_weight)
    throw std::invalid_argument("Missing policy_statement.action.set_weight attribute");
  if (!stmt.prefixes && !stmt.tags)
    throw std::invalid_argument(
        "Missing policy_statement.matcher.prefixes or policy_statement.matcher.tags attribute");
  action_ = *stmt.set_weight;
  if (stmt.prefixes)
    for (const auto& p : *stmt.prefixes) prefixSet_.insert(p);
  if (stmt.tags)
    for (const auto& t : *stmt.tags) tagSet_.insert(t);
}

// RibPolicy.cpp:72-105
bool RibPolicyStatement::match(const RibUnicastEntry& route) const {
  if (tagSet_.empty() && prefixSet_.empty()) return false;
  bool tagMatch = false;
  if (tagSet_.empty()) {
    tagMatch = true;
  } else {
    // route.bestPrefixEntry is a PrefixEntry value there: no entry = no tags
    for (const auto& tag : tagSet_) {
      if (route.bestPrefixEntry && route.bestPrefixEntry->tags.count(tag)) {
        tagMatch = true;
        break;
      }
    }
  }
  bool prefixMatch = false;
  if (prefixSet_.empty()) {
    prefixMatch = true;
  } else {
    prefixMatch = prefixSet_.count(route.prefix) > 0;
  }
  return tagMatch && prefixMatch;
}

// RibPolicy.cpp:107-158
bool RibPolicyStatement::applyAction(RibUnicastEntry& route, uint64_t& invalidatedStat) const {
  if (!match(route)) return false;
  const RibRouteActionWeight& weightAction = action_;
  NextHopSet newNexthops;
  for (const auto& nh : route.nexthops) {
    // precedence: neighbour weight, area weight, default weight
    int32_t newWeight = weightAction.default_weight;
    if (nh.area) {
      auto it = weightAction.area_to_weight.find(*nh.area);
      if (it != weightAction.area_to_weight.end()) newWeight = it->second;
    }
    if (nh.neighborNodeName) {
      auto it = weightAction.neighbor_to_weight.find(*nh.neighborNodeName);
      if (it != weightAction.neighbor_to_weight.end()) newWeight = it->second;
    }
    if (newWeight > 0) {
      NextHopThrift newNh = nh;
      newNh.weight = newWeight;
      newNexthops.emplace(std::move(newNh));
    }
  }
  // every nexthop weighted 0: the route keeps its nexthops (and is counted)
  if (newNexthops.empty()) {
    ++invalidatedStat;
    return false;
  }
  route.nexthops = std::move(newNexthops);
  return true;
}

// RibPolicy.cpp:164-178
RibPolicy::RibPolicy(const std::vector<RibPolicyStatementSpec>& statements, int64_t ttlSecs)
    : validUntilTs_(std::chrono::steady_clock::now() + std::chrono::seconds(ttlSecs)) {
  if (statements.empty()) throw std::invalid_argument("Missing policy.statements attribute");
  for (const auto& s : statements) policyStatements_.emplace_back(RibPolicyStatement(s));
}

// RibPolicy.cpp:197-206
std::chrono::milliseconds RibPolicy::getTtlDuration() const {
  return std::chrono::duration_cast<std::chrono::milliseconds>(validUntilTs_ -
                                                               std::chrono::steady_clock::now());
}

bool RibPolicy::isActive() const { return getTtlDuration().count() > 0; }

// RibPolicy.cpp:208-226
bool RibPolicy::match(const RibUnicastEntry& route) const {
  for (const auto& statement : policyStatements_)
    if (statement.match(route)) return true;
  return false;
}

bool RibPolicy::applyAction(RibUnicastEntry& route) {
  for (const auto& statement : policyStatements_)
    if (statement.applyAction(route, invalidated_)) return true;
  return false;
}

// RibPolicy.cpp:228-246
RibPolicy::PolicyChange RibPolicy::applyPolicy(
    std::unordered_map<Cidr, RibUnicastEntry, CidrHash>& unicastEntries) {
  PolicyChange change;
  if (!isActive()) return change;
  for (auto iter = unicastEntries.begin(); iter != unicastEntries.end(); ++iter) {
    if (applyAction(iter->second)) change.updatedRoutes.push_back(iter->second.prefix);
  }
  return change;
}

}  // namespace oracle
