// Drop-in RibPolicy (see rib_policy.h).
#include "rib_policy.h"

#include "parallel.h"

#include <stdexcept>

namespace openr_amd {

RibPolicyStatement::RibPolicyStatement(const RibPolicyStatementSpec& spec)
    : name_(spec.name) {
  // RibPolicy.cpp:20-36: an action and at least one matcher are mandatory
  if (!spec.setWeight)
    throw std::invalid_argument("Missing policy_statement.action.set_weight attribute");
  if (!spec.prefixes && !spec.tags)
    throw std::invalid_argument(
        "Missing policy_statement.matcher.prefixes or policy_statement.matcher.tags attribute");
  action_ = *spec.setWeight;
  if (spec.prefixes) prefixSet_.insert(spec.prefixes->begin(), spec.prefixes->end());
  if (spec.tags) tagSet_.insert(spec.tags->begin(), spec.tags->end());
}

bool RibPolicyStatement::match(const RibUnicastEntry& route) const {  // RibPolicy.cpp:73-105
  if (tagSet_.empty() && prefixSet_.empty()) return false;
  bool tagMatch = tagSet_.empty();
  if (!tagMatch && route.bestPrefixEntry) {
    for (const auto& tag : tagSet_) {
      if (route.bestPrefixEntry->tags.count(tag)) {
        tagMatch = true;
        break;
      }
    }
  }
  const bool prefixMatch = prefixSet_.empty() || prefixSet_.count(route.prefix) > 0;
  return tagMatch && prefixMatch;
}

int32_t RibPolicyStatement::weightOf(const std::optional<std::string>& area,
                                     const std::optional<std::string>& neighbor) const {
  // precedence: neighbour weight, then area weight, then default weight
  int32_t w = action_.defaultWeight;
  if (area) {
    auto it = action_.areaToWeight.find(*area);
    if (it != action_.areaToWeight.end()) w = it->second;
  }
  if (neighbor) {
    auto it = action_.neighborToWeight.find(*neighbor);
    if (it != action_.neighborToWeight.end()) w = it->second;
  }
  return w;
}

bool RibPolicyStatement::applyAction(RibUnicastEntry& route, uint64_t* invalidated) const {
  if (!match(route)) return false;  // RibPolicy.cpp:108-161
  // the outcome depends on the nexthop set and this statement only: the
  // routes sharing a set (NextHops) share its result, per thread. A memo
  // entry holds its input set, so that set's address is not reused while
  // it is a key; statements are named by a process-unique id
  struct Key {
    const void* set;
    uint64_t stmt;
    bool operator==(const Key& o) const { return set == o.set && stmt == o.stmt; }
  };
  struct KeyHash {
    size_t operator()(const Key& k) const {
      return std::hash<const void*>()(k.set) ^ (std::hash<uint64_t>()(k.stmt) * 0x9E3779B97F4A7C15ull);
    }
  };
  struct Memo {
    NextHops in, out;
    bool kept;
  };
  thread_local std::unordered_map<Key, Memo, KeyHash> memo;
  const bool shared = route.nexthops.id() != nullptr;
  if (shared) {
    auto it = memo.find(Key{route.nexthops.id(), id_});
    if (it != memo.end()) {
      if (!it->second.kept) {
        if (invalidated) ++*invalidated;
        return false;
      }
      route.nexthops = it->second.out;
      return true;
    }
    if (memo.size() >= 4096) memo.clear();
  }
  const NextHops in = shared ? route.nexthops : NextHops{};
  auto weightOf = [&](const NextHopThrift& nh) { return this->weightOf(nh.area, nh.neighborNodeName); };
  bool any = false;
  for (const auto& nh : route.nexthops) {
    if (weightOf(nh) > 0) {
      any = true;
      break;
    }
  }
  if (!any) {  // every nexthop dropped: keep the route as it was
    if (invalidated) ++*invalidated;
    if (shared) memo.emplace(Key{in.id(), id_}, Memo{in, NextHops{}, false});
    return false;
  }
  // the kept nexthops move into a new set as nodes (no copies of their
  // strings, no allocations), in the old set's iteration order - the
  // reference's insertion sequence into newNexthops (RibPolicy.cpp:116-141),
  // so the new set iterates as the reference's does (the weight is part of
  // the hash, NetworkUtil.cpp:57-66)
  NextHopSet src = route.nexthops.take();  // moved out, or copied when shared
  NextHopSet out;  // grown as the reference's is (no reserve: the bucket count shapes the order)
  while (!src.empty()) {
    auto node = src.extract(src.begin());
    const int32_t w = weightOf(node.value());
    if (w <= 0) continue;
    node.value().weight = w;
    out.insert(std::move(node));
  }
  route.nexthops = std::move(out);
  if (shared) memo.emplace(Key{in.id(), id_}, Memo{in, route.nexthops, true});
  return true;
}

RibPolicy::RibPolicy(const std::vector<RibPolicyStatementSpec>& statements, int64_t ttlSecs)
    : validUntil_(std::chrono::steady_clock::now() + std::chrono::seconds(ttlSecs)) {
  if (statements.empty()) throw std::invalid_argument("Missing policy.statements attribute");
  for (const auto& s : statements) statements_.emplace_back(s);
}

std::chrono::milliseconds RibPolicy::getTtlDuration() const {
  return std::chrono::duration_cast<std::chrono::milliseconds>(validUntil_ -
                                                               std::chrono::steady_clock::now());
}

bool RibPolicy::match(const RibUnicastEntry& route) const {
  for (const auto& s : statements_)
    if (s.match(route)) return true;
  return false;
}

bool RibPolicy::applyAction(RibUnicastEntry& route) { return applyAction(route, &invalidated_); }

bool RibPolicy::applyAction(RibUnicastEntry& route, uint64_t* invalidated) const {
  for (const auto& s : statements_)
    if (s.applyAction(route, invalidated)) return true;
  return false;
}

RibPolicy::PolicyChange RibPolicy::applyPolicy(UnicastRouteMap& routes) {
  PolicyChange change;  // RibPolicy.cpp:229-247
  if (!isActive()) return change;
  // shard by shard (on the worker pool for large databases: C5 applies the
  // policy to 1M routes); updated prefixes in the map's iteration order
  constexpr size_t kS = UnicastRouteMap::kShards;
  std::vector<std::vector<Cidr>> updated(kS);
  std::vector<uint64_t> invalidated(kS, 0);
  auto shard = [&](size_t s) {
    for (auto& [prefix, route] : routes.shard(s))
      if (applyAction(route, &invalidated[s])) updated[s].push_back(route.prefix);
  };
  auto& pool = WorkerPool::instance();
  if (routes.size() >= 4096 && pool.size() > 1) {
    pool.parallelFor(kS, [&](size_t, size_t b, size_t e) {
      for (size_t s = b; s < e; ++s) shard(s);
    });
  } else {
    for (size_t s = 0; s < kS; ++s) shard(s);
  }
  for (size_t s = 0; s < kS; ++s) {
    change.updatedRoutes.insert(change.updatedRoutes.end(), updated[s].begin(), updated[s].end());
    invalidated_ += invalidated[s];
  }
  return change;
}

RibPolicy::PolicyChange RibPolicy::applyPolicy(std::unordered_map<Cidr, RibUnicastEntry, CidrHash>& routes) {
  PolicyChange change;
  if (!isActive()) return change;
  for (auto& [prefix, route] : routes)
    if (applyAction(route, &invalidated_)) change.updatedRoutes.push_back(route.prefix);
  return change;
}

}  // namespace openr_amd
