// TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle_types.h header).
//
// Restatement of openr/decision/LinkState.{h,cpp}: HoldableValue, Link, the
// per-area LinkState graph store, DijkstraQ and runSpf / getKthPaths. The
// containers are the reference's own choices (string-keyed unordered maps,
// shared_ptr<Link> sets hashed with the folly pair hash, a binary heap
// re-made on every strict decrease) so that (a) iteration-order-dependent
// results (KSP2 parallel-link ties) come out identically and (b) the CPU
// timing is a faithful baseline for the reference algorithm.
#pragma once

#include <limits>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "oracle_types.h"

namespace oracle {

using Metric = uint64_t;  // LinkStateMetric, LinkState.h:22

// LinkState.h:36-58, LinkState.cpp:54-125
template <class T>
class HoldableValue {
 public:
  explicit HoldableValue(T v) : val_(v) {}
  void set(T v) {  // operator=
    val_ = v;
    held_.reset();
    ttl_ = 0;
  }
  const T& value() const { return held_ ? *held_ : val_; }
  bool hasHold() const { return held_.has_value(); }
  bool decrementTtl() {
    if (held_ && --ttl_ == 0) {
      held_.reset();
      return true;
    }
    return false;
  }
  bool updateValue(T v, Metric upTtl, Metric downTtl);

 private:
  bool bringingUp(T v) const;
  T val_;
  std::optional<T> held_;
  Metric ttl_{0};
};

class Link {  // LinkState.h:82-175
 public:
  Link(const std::string& area, const std::string& n1, const std::string& if1,
       const std::string& n2, const std::string& if2);
  Link(const std::string& area, const std::string& n1, const Adjacency& a1,
       const std::string& n2, const Adjacency& a2);

  const std::string& getArea() const { return area_; }
  const std::string& getOtherNodeName(const std::string& n) const;
  const std::string& firstNodeName() const { return ordered_.first.first; }
  const std::string& secondNodeName() const { return ordered_.second.first; }
  const std::string& getIfaceFromNode(const std::string& n) const;
  Metric getMetricFromNode(const std::string& n) const;
  int32_t getAdjLabelFromNode(const std::string& n) const;
  bool getOverloadFromNode(const std::string& n) const;
  const BinaryAddress& getNhV4FromNode(const std::string& n) const;
  const BinaryAddress& getNhV6FromNode(const std::string& n) const;
  void setNhV4FromNode(const std::string& n, const BinaryAddress& a);
  void setNhV6FromNode(const std::string& n, const BinaryAddress& a);
  bool setMetricFromNode(const std::string& n, Metric m, Metric up, Metric down);
  void setAdjLabelFromNode(const std::string& n, int32_t l);
  bool setOverloadFromNode(const std::string& n, bool o, Metric up, Metric down);
  void setHoldUpTtl(Metric t) { holdUpTtl_ = t; }
  bool isUp() const;
  bool decrementHolds();
  bool hasHolds() const;
  bool operator<(const Link& o) const;
  bool operator==(const Link& o) const;

 private:
  int side(const std::string& n) const;  // 1, 2; throws std::invalid_argument
  std::string area_, n1_, n2_, if1_, if2_;
  HoldableValue<Metric> metric1_{1}, metric2_{1};
  HoldableValue<bool> overload1_{false}, overload2_{false};
  int32_t adjLabel1_{0}, adjLabel2_{0};
  BinaryAddress nhV41_, nhV42_, nhV61_, nhV62_;
  Metric holdUpTtl_{0};
  std::pair<std::pair<std::string, std::string>, std::pair<std::string, std::string>>
      ordered_;

 public:
  const size_t hash;
};

using LinkPtr = std::shared_ptr<Link>;
struct LinkPtrHash {
  size_t operator()(const LinkPtr& l) const { return l->hash; }
};
struct LinkPtrEq {
  bool operator()(const LinkPtr& a, const LinkPtr& b) const { return *a == *b; }
};
struct LinkPtrLess {
  bool operator()(const LinkPtr& a, const LinkPtr& b) const { return *a < *b; }
};
using LinkSet = std::unordered_set<LinkPtr, LinkPtrHash, LinkPtrEq>;
using Path = std::vector<LinkPtr>;

class NodeSpfResult {  // LinkState.h:203-257
 public:
  struct PathLink {
    LinkPtr link;
    std::string prevNode;
  };
  explicit NodeSpfResult(Metric m) : metric_(m) {}
  void reset(Metric m) {
    metric_ = m;
    pathLinks_.clear();
    nextHops_.clear();
  }
  const std::vector<PathLink>& pathLinks() const { return pathLinks_; }
  const std::unordered_set<std::string>& nextHops() const { return nextHops_; }
  Metric metric() const { return metric_; }
  void addPath(const LinkPtr& l, const std::string& prev) {
    pathLinks_.push_back({l, prev});
  }
  void addNextHops(const std::unordered_set<std::string>& s) {
    nextHops_.insert(s.begin(), s.end());
  }
  void addNextHop(const std::string& s) { nextHops_.insert(s); }

 private:
  Metric metric_;
  std::vector<PathLink> pathLinks_;
  std::unordered_set<std::string> nextHops_;
};

using SpfResult = std::unordered_map<std::string, NodeSpfResult>;

struct LinkStateChange {  // LinkState.h:306-325
  bool topologyChanged{false};
  bool linkAttributesChanged{false};
  bool nodeLabelChanged{false};
};

class LinkState {  // LinkState.h:177-469
 public:
  explicit LinkState(const std::string& area) : area_(area) {}

  const SpfResult& getSpfResult(const std::string& node, bool useLinkMetric = true) const;
  const std::vector<Path>& getKthPaths(const std::string& src, const std::string& dst,
                                       size_t k) const;
  LinkStateChange decrementHolds();
  LinkStateChange updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric up = 0,
                                          Metric down = 0);
  LinkStateChange deleteAdjacencyDatabase(const std::string& node);
  std::optional<Metric> getMetricFromAToB(const std::string& a, const std::string& b,
                                          bool useLinkMetric = true) const;
  std::optional<Metric> getHopsFromAToB(const std::string& a, const std::string& b) const {
    return getMetricFromAToB(a, b, false);
  }
  Metric getMaxHopsToNode(const std::string& node) const;
  const std::string& getArea() const { return area_; }
  bool hasNode(const std::string& n) const { return adjacencyDatabases_.count(n) != 0; }
  const LinkSet& linksFromNode(const std::string& n) const;
  bool isNodeOverloaded(const std::string& n) const;
  bool hasHolds() const;
  size_t numLinks() const { return allLinks_.size(); }
  size_t numNodes() const { return linkMap_.size(); }
  const std::unordered_map<std::string, AdjacencyDatabase>& getAdjacencyDatabases() const {
    return adjacencyDatabases_;
  }
  static bool pathAInPathB(const Path& a, const Path& b);

  // not memoized: the fresh run getKthPaths uses for k >= 2
  SpfResult runSpf(const std::string& src, bool useLinkMetric,
                   const LinkSet& ignore = {}) const;

  mutable uint64_t spfRuns{0};  // fb303 "decision.spf_runs"

 private:
  std::optional<Path> traceOnePath(const std::string& src, const std::string& dst,
                                   const SpfResult& res, LinkSet& visited) const;
  void addLink(const LinkPtr& l);
  void removeLink(const LinkPtr& l);
  void removeNode(const std::string& n);
  bool updateNodeOverloaded(const std::string& n, bool o, Metric up, Metric down);
  LinkPtr maybeMakeLink(const std::string& node, const Adjacency& adj) const;
  std::vector<LinkPtr> getOrderedLinkSet(const AdjacencyDatabase& db) const;
  std::vector<LinkPtr> orderedLinksFromNode(const std::string& n) const;

  std::string area_;
  // memo keys only affect lookup, never results (LinkState.h:279-301)
  mutable std::map<std::pair<std::string, bool>, SpfResult> spfResults_;
  mutable std::map<std::tuple<std::string, std::string, size_t>, std::vector<Path>>
      kthPathResults_;
  std::unordered_map<std::string, LinkSet> linkMap_;
  LinkSet allLinks_;
  std::unordered_map<std::string, HoldableValue<bool>> nodeOverloads_;
  std::unordered_map<std::string, AdjacencyDatabase> adjacencyDatabases_;
};

}  // namespace oracle
