// TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle_types.h header).
// Restates openr/decision/LinkState.cpp; each function cites the lines it
// follows.
#include "oracle_link_state.h"

#include <algorithm>
#include <stdexcept>

namespace oracle {

// ---- HoldableValue (LinkState.cpp:87-121) --------------------------------
template <>
bool HoldableValue<bool>::bringingUp(bool v) const {
  return val_ && !v;  // overloaded -> not overloaded
}
template <>
bool HoldableValue<Metric>::bringingUp(Metric v) const {
  return v < val_;  // metric decrease
}

template <class T>
bool HoldableValue<T>::updateValue(T v, Metric upTtl, Metric downTtl) {
  if (v == val_) {
    return false;
  }
  if (hasHold()) {
    // a second change while held falls back to a fast update
    held_.reset();
    ttl_ = 0;
  } else {
    ttl_ = bringingUp(v) ? upTtl : downTtl;
    if (ttl_ != 0) {
      held_ = val_;
    }
  }
  val_ = v;
  return !hasHold();
}
template class HoldableValue<bool>;
template class HoldableValue<Metric>;

// ---- Link (LinkState.cpp:127-361) -----------------------------------------
static size_t linkHash(const std::pair<std::pair<std::string, std::string>,
                                       std::pair<std::string, std::string>>& o) {
  PairStrHash h;
  return hash128to64(h(o.first), h(o.second));
}

Link::Link(const std::string& area, const std::string& n1, const std::string& if1,
           const std::string& n2, const std::string& if2)
    : area_(area),
      n1_(n1),
      n2_(n2),
      if1_(if1),
      if2_(if2),
      ordered_(std::minmax(std::make_pair(n1, if1), std::make_pair(n2, if2))),
      hash(linkHash(ordered_)) {}

Link::Link(const std::string& area, const std::string& n1, const Adjacency& a1,
           const std::string& n2, const Adjacency& a2)
    : Link(area, n1, a1.ifName, n2, a2.ifName) {
  metric1_.set(static_cast<Metric>(static_cast<int64_t>(a1.metric)));
  metric2_.set(static_cast<Metric>(static_cast<int64_t>(a2.metric)));
  overload1_.set(a1.isOverloaded);
  overload2_.set(a2.isOverloaded);
  adjLabel1_ = a1.adjLabel;
  adjLabel2_ = a2.adjLabel;
  nhV41_ = a1.nextHopV4;
  nhV42_ = a2.nextHopV4;
  nhV61_ = a1.nextHopV6;
  nhV62_ = a2.nextHopV6;
}

int Link::side(const std::string& n) const {
  if (n == n1_) return 1;
  if (n == n2_) return 2;
  throw std::invalid_argument(n);
}

const std::string& Link::getOtherNodeName(const std::string& n) const {
  return side(n) == 1 ? n2_ : n1_;
}
const std::string& Link::getIfaceFromNode(const std::string& n) const {
  return side(n) == 1 ? if1_ : if2_;
}
Metric Link::getMetricFromNode(const std::string& n) const {
  return side(n) == 1 ? metric1_.value() : metric2_.value();
}
int32_t Link::getAdjLabelFromNode(const std::string& n) const {
  return side(n) == 1 ? adjLabel1_ : adjLabel2_;
}
bool Link::getOverloadFromNode(const std::string& n) const {
  return side(n) == 1 ? overload1_.value() : overload2_.value();
}
const BinaryAddress& Link::getNhV4FromNode(const std::string& n) const {
  return side(n) == 1 ? nhV41_ : nhV42_;
}
const BinaryAddress& Link::getNhV6FromNode(const std::string& n) const {
  return side(n) == 1 ? nhV61_ : nhV62_;
}
void Link::setNhV4FromNode(const std::string& n, const BinaryAddress& a) {
  (side(n) == 1 ? nhV41_ : nhV42_) = a;
}
void Link::setNhV6FromNode(const std::string& n, const BinaryAddress& a) {
  (side(n) == 1 ? nhV61_ : nhV62_) = a;
}
bool Link::setMetricFromNode(const std::string& n, Metric m, Metric up, Metric down) {
  return (side(n) == 1 ? metric1_ : metric2_).updateValue(m, up, down);
}
void Link::setAdjLabelFromNode(const std::string& n, int32_t l) {
  (side(n) == 1 ? adjLabel1_ : adjLabel2_) = l;
}
bool Link::setOverloadFromNode(const std::string& n, bool o, Metric up, Metric down) {
  const bool wasUp = isUp();
  (side(n) == 1 ? overload1_ : overload2_).updateValue(o, up, down);
  return wasUp != isUp();  // only simplex-free up/down transitions count
}
bool Link::isUp() const {  // LinkState.cpp:233-236
  return holdUpTtl_ == 0 && !overload1_.value() && !overload2_.value();
}
bool Link::decrementHolds() {  // LinkState.cpp:238-249
  bool expired = false;
  if (holdUpTtl_ != 0) expired |= (--holdUpTtl_ == 0);
  expired |= metric1_.decrementTtl();
  expired |= metric2_.decrementTtl();
  expired |= overload1_.decrementTtl();
  expired |= overload2_.decrementTtl();
  return expired;
}
bool Link::hasHolds() const {
  return holdUpTtl_ != 0 || metric1_.hasHold() || metric2_.hasHold() ||
      overload1_.hasHold() || overload2_.hasHold();
}
bool Link::operator<(const Link& o) const {  // LinkState.cpp:347-353
  if (hash != o.hash) return hash < o.hash;
  return ordered_ < o.ordered_;
}
bool Link::operator==(const Link& o) const {
  return hash == o.hash && ordered_ == o.ordered_;
}

// ---- LinkState graph store ------------------------------------------------
bool LinkState::pathAInPathB(const Path& a, const Path& b) {  // LinkState.h:395-410
  if (a.size() > b.size()) return false;
  for (size_t i = 0; i + a.size() <= b.size(); ++i) {
    size_t k = 0;
    while (k < a.size() && *a[k] == *b[i + k]) ++k;
    if (k == a.size()) return true;
  }
  return false;
}

std::optional<Path> LinkState::traceOnePath(const std::string& src, const std::string& dst,
                                            const SpfResult& res,
                                            LinkSet& visited) const {  // :398-419
  if (src == dst) return Path{};
  for (const auto& pl : res.at(dst).pathLinks()) {
    // a link is consumed on first touch, even if the branch then fails
    if (visited.insert(pl.link).second) {
      auto p = traceOnePath(src, pl.prevNode, res, visited);
      if (p) {
        p->push_back(pl.link);
        return p;
      }
    }
  }
  return std::nullopt;
}

void LinkState::addLink(const LinkPtr& l) {  // :421-426
  if (!linkMap_[l->firstNodeName()].insert(l).second ||
      !linkMap_[l->secondNodeName()].insert(l).second || !allLinks_.insert(l).second) {
    throw std::logic_error("duplicate link insert");
  }
}

void LinkState::removeLink(const LinkPtr& l) {  // :429-434
  if (!linkMap_.at(l->firstNodeName()).erase(l) ||
      !linkMap_.at(l->secondNodeName()).erase(l) || !allLinks_.erase(l)) {
    throw std::logic_error("missing link on remove");
  }
}

void LinkState::removeNode(const std::string& n) {  // :436-455
  auto it = linkMap_.find(n);
  if (it == linkMap_.end()) return;
  for (const auto& l : it->second) {
    linkMap_.at(l->getOtherNodeName(n)).erase(l);
    allLinks_.erase(l);
  }
  linkMap_.erase(it);
  nodeOverloads_.erase(n);
}

const LinkSet& LinkState::linksFromNode(const std::string& n) const {  // :457-465
  static const LinkSet kEmpty;
  auto it = linkMap_.find(n);
  return it == linkMap_.end() ? kEmpty : it->second;
}

std::vector<LinkPtr> LinkState::orderedLinksFromNode(const std::string& n) const {
  std::vector<LinkPtr> v;  // :467-478
  auto it = linkMap_.find(n);
  if (it != linkMap_.end()) {
    v.assign(it->second.begin(), it->second.end());
    std::sort(v.begin(), v.end(), LinkPtrLess{});
  }
  return v;
}

bool LinkState::updateNodeOverloaded(const std::string& n, bool o, Metric up,
                                     Metric down) {  // :480-493
  auto it = nodeOverloads_.find(n);
  if (it != nodeOverloads_.end()) return it->second.updateValue(o, up, down);
  nodeOverloads_.emplace(n, HoldableValue<bool>{o});
  return false;  // a new node's overload bit is not a topology change
}

bool LinkState::isNodeOverloaded(const std::string& n) const {  // :495-498
  auto it = nodeOverloads_.find(n);
  return it != nodeOverloads_.end() && it->second.value();
}

LinkStateChange LinkState::decrementHolds() {  // :500-514
  LinkStateChange c;
  for (auto& l : allLinks_) c.topologyChanged |= l->decrementHolds();
  for (auto& kv : nodeOverloads_) c.topologyChanged |= kv.second.decrementTtl();
  if (c.topologyChanged) {
    spfResults_.clear();
    kthPathResults_.clear();
  }
  return c;
}

bool LinkState::hasHolds() const {  // :516-529
  for (auto& l : allLinks_)
    if (l->hasHolds()) return true;
  for (auto& kv : nodeOverloads_)
    if (kv.second.hasHold()) return true;
  return false;
}

LinkPtr LinkState::maybeMakeLink(const std::string& node, const Adjacency& adj) const {
  // :531-547 — only bidirectional adjacencies (names and ifnames match) form links
  auto it = adjacencyDatabases_.find(adj.otherNodeName);
  if (it == adjacencyDatabases_.end()) return nullptr;
  for (const auto& other : it->second.adjacencies) {
    if (other.otherNodeName == node && adj.otherIfName == other.ifName &&
        adj.ifName == other.otherIfName) {
      return std::make_shared<Link>(area_, node, adj, adj.otherNodeName, other);
    }
  }
  return nullptr;
}

std::vector<LinkPtr> LinkState::getOrderedLinkSet(const AdjacencyDatabase& db) const {
  std::vector<LinkPtr> v;  // :549-562
  for (const auto& a : db.adjacencies) {
    if (auto l = maybeMakeLink(db.thisNodeName, a)) v.push_back(l);
  }
  std::sort(v.begin(), v.end(), LinkPtrLess{});
  return v;
}

LinkStateChange LinkState::updateAdjacencyDatabase(const AdjacencyDatabase& db,
                                                   Metric up, Metric down) {
  // :564-719
  LinkStateChange change;
  const std::string node = db.thisNodeName;
  AdjacencyDatabase prior = std::move(adjacencyDatabases_[node]);
  adjacencyDatabases_[node] = db;

  auto oldLinks = orderedLinksFromNode(node);
  auto newLinks = getOrderedLinkSet(db);

  change.topologyChanged |= updateNodeOverloaded(node, db.isOverloaded, up, down);
  change.nodeLabelChanged = prior.nodeLabel != db.nodeLabel;

  auto ni = newLinks.begin();
  auto oi = oldLinks.begin();
  while (ni != newLinks.end() || oi != oldLinks.end()) {
    if (ni != newLinks.end() && (oi == oldLinks.end() || **ni < **oi)) {
      (*ni)->setHoldUpTtl(up);  // link up (held if up != 0)
      change.topologyChanged |= (*ni)->isUp();
      addLink(*ni);
      ++ni;
      continue;
    }
    if (oi != oldLinks.end() && (ni == newLinks.end() || **oi < **ni)) {
      change.topologyChanged |= (*oi)->isUp();  // link down
      removeLink(*oi);
      ++oi;
      continue;
    }
    Link& nl = **ni;
    Link& ol = **oi;
    if (nl.getMetricFromNode(node) != ol.getMetricFromNode(node)) {
      change.topologyChanged |=
          ol.setMetricFromNode(node, nl.getMetricFromNode(node), up, down);
    }
    if (nl.getOverloadFromNode(node) != ol.getOverloadFromNode(node)) {
      change.topologyChanged |=
          ol.setOverloadFromNode(node, nl.getOverloadFromNode(node), up, down);
    }
    if (nl.getAdjLabelFromNode(node) != ol.getAdjLabelFromNode(node)) {
      change.linkAttributesChanged = true;
      ol.setAdjLabelFromNode(node, nl.getAdjLabelFromNode(node));
    }
    if (nl.getNhV4FromNode(node) != ol.getNhV4FromNode(node)) {
      change.linkAttributesChanged = true;
      ol.setNhV4FromNode(node, nl.getNhV4FromNode(node));
    }
    if (nl.getNhV6FromNode(node) != ol.getNhV6FromNode(node)) {
      change.linkAttributesChanged = true;
      ol.setNhV6FromNode(node, nl.getNhV6FromNode(node));
    }
    ++ni;
    ++oi;
  }
  if (change.topologyChanged) {
    spfResults_.clear();
    kthPathResults_.clear();
  }
  return change;
}

LinkStateChange LinkState::deleteAdjacencyDatabase(const std::string& node) {
  LinkStateChange c;  // :721-738
  auto it = adjacencyDatabases_.find(node);
  if (it != adjacencyDatabases_.end()) {
    removeNode(node);
    adjacencyDatabases_.erase(it);
    spfResults_.clear();
    kthPathResults_.clear();
    c.topologyChanged = true;
  }
  return c;
}

std::optional<Metric> LinkState::getMetricFromAToB(const std::string& a,
                                                   const std::string& b,
                                                   bool useLinkMetric) const {
  if (a == b) return 0;  // :740-751
  const auto& r = getSpfResult(a, useLinkMetric);
  auto it = r.find(b);
  if (it == r.end()) return std::nullopt;
  return it->second.metric();
}

Metric LinkState::getMaxHopsToNode(const std::string& node) const {  // :753-760
  Metric mx = 0;
  for (const auto& kv : getSpfResult(node, false)) mx = std::max(mx, kv.second.metric());
  return mx;
}

const std::vector<Path>& LinkState::getKthPaths(const std::string& src,
                                                const std::string& dst,
                                                size_t k) const {  // :762-791
  if (k < 1) throw std::invalid_argument("k must be >= 1");
  auto key = std::make_tuple(src, dst, k);
  auto it = kthPathResults_.find(key);
  if (it != kthPathResults_.end()) return it->second;

  LinkSet ignore;
  for (size_t i = 1; i < k; ++i) {
    for (const auto& p : getKthPaths(src, dst, i)) {
      for (const auto& l : p) ignore.insert(l);
    }
  }
  std::vector<Path> paths;
  SpfResult fresh;
  const SpfResult* res;
  if (ignore.empty()) {
    res = &getSpfResult(src, true);
  } else {
    fresh = runSpf(src, true, ignore);
    res = &fresh;
  }
  if (res->count(dst)) {
    LinkSet visited;
    auto p = traceOnePath(src, dst, *res, visited);
    while (p && !p->empty()) {
      paths.push_back(std::move(*p));
      p = traceOnePath(src, dst, *res, visited);
    }
  }
  return kthPathResults_.emplace(key, std::move(paths)).first->second;
}

const SpfResult& LinkState::getSpfResult(const std::string& node,
                                         bool useLinkMetric) const {  // :793-803
  auto key = std::make_pair(node, useLinkMetric);
  auto it = spfResults_.find(key);
  if (it == spfResults_.end()) {
    it = spfResults_.emplace(key, runSpf(node, useLinkMetric)).first;
  }
  return it->second;
}

// ---- DijkstraQ (LinkState.h:475-535) ---------------------------------------
namespace {
struct QNode {
  QNode(const std::string& n, Metric m) : name(n), result(m) {}
  std::string name;
  NodeSpfResult result;
};
using QNodePtr = std::shared_ptr<QNode>;

class DijkstraQ {
 public:
  void insert(const std::string& n, Metric d) {
    heap_.push_back(std::make_shared<QNode>(n, d));
    byName_[n] = heap_.back();
    std::push_heap(heap_.begin(), heap_.end(), greater);
  }
  QNodePtr get(const std::string& n) {
    auto it = byName_.find(n);
    return it == byName_.end() ? nullptr : it->second;
  }
  QNodePtr extractMin() {
    if (heap_.empty()) return nullptr;
    auto m = heap_.front();
    byName_.erase(m->name);
    std::pop_heap(heap_.begin(), heap_.end(), greater);
    heap_.pop_back();
    return m;
  }
  void reMake() { std::make_heap(heap_.begin(), heap_.end(), greater); }

 private:
  // min-heap on (metric, name)
  static bool greater(const QNodePtr& a, const QNodePtr& b) {
    if (a->result.metric() != b->result.metric())
      return a->result.metric() > b->result.metric();
    return a->name > b->name;
  }
  std::vector<QNodePtr> heap_;
  std::unordered_map<std::string, QNodePtr> byName_;
};
}  // namespace

SpfResult LinkState::runSpf(const std::string& src, bool useLinkMetric,
                            const LinkSet& ignore) const {  // :808-882
  SpfResult result;
  ++spfRuns;
  DijkstraQ q;
  q.insert(src, 0);
  while (auto node = q.extractMin()) {
    auto rc = result.emplace(node->name, std::move(node->result));
    const std::string& v = rc.first->first;
    const Metric dv = rc.first->second.metric();
    const auto& nhv = rc.first->second.nextHops();
    if (isNodeOverloaded(v) && v != src) {
      continue;  // recorded, but no transit through a drained node
    }
    for (const auto& link : linksFromNode(v)) {
      const std::string& u = link->getOtherNodeName(v);
      if (!link->isUp() || result.count(u) || ignore.count(link)) continue;
      const Metric w = useLinkMetric ? link->getMetricFromNode(v) : 1;
      auto un = q.get(u);
      if (!un) {
        q.insert(u, dv + w);
        un = q.get(u);
      }
      if (un->result.metric() >= dv + w) {
        if (un->result.metric() > dv + w) {
          un->result.reset(dv + w);
          q.reMake();
        }
        un->result.addPath(link, v);
        un->result.addNextHops(nhv);
        if (un->result.nextHops().empty()) un->result.addNextHop(u);  // direct nbr
      }
    }
  }
  return result;
}

}  // namespace oracle
