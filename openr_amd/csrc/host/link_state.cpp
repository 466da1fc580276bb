// Drop-in LinkState over libopenr_hip (see link_state.h).
#include "link_state.h"

#include "parallel.h"

#include <set>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string_view>

namespace openr_amd {

namespace {

void check(orh_ctx* ctx, int rc, const char* what) {
  if (rc != ORH_OK) {
    throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) +
                             "): " + (ctx ? orh_last_error(ctx) : ""));
  }
}

uint32_t toDeviceMetric(Metric m) {
  // the device keeps 32-bit link metrics (path sums are 64-bit on the exact
  // path); thrift adjacency metrics are i32, so only negative values (which
  // widen past 2^32) are out of range
  if (m > 0xFFFFFFFFull) {
    throw std::domain_error("libopenr_hip: link metric " + std::to_string(m) +
                            " is outside [0, 2^32-1] (negative adjacency metrics are "
                            "not supported by the device SPF)");
  }
  return static_cast<uint32_t>(m);
}

// ORH_KSP_PROF=1: phase times of prefetchKthPaths / fillRows on stderr
struct KspProf {
  bool on = std::getenv("ORH_KSP_PROF") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "ksp-prof %-20s %8.3f ms\n", what,
                 std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

}  // namespace

orh_ctx* defaultContext() {
  static std::once_flag once;
  static orh_ctx* ctx = nullptr;
  static int rc = ORH_OK;
  std::call_once(once, [] {
    int dev = 0;
    if (const char* e = std::getenv("ORH_DEVICE")) dev = std::atoi(e);
    rc = orh_create(dev, 0, &ctx);
  });
  if (!ctx) {
    throw std::runtime_error("libopenr_hip: no usable HIP device (orh_create rc=" +
                             std::to_string(rc) + "); the Decision SPF path requires a GPU");
  }
  return ctx;
}

orh_ctx* laneContext(unsigned lane) {
  if (lane == 0) return defaultContext();
  if (lane >= kMaxLanes) throw std::invalid_argument("laneContext: lane out of range");
  static std::mutex mu;
  static orh_ctx* lanes[kMaxLanes] = {};
  std::lock_guard<std::mutex> lock(mu);
  if (!lanes[lane]) {
    int dev = 0;
    if (const char* e = std::getenv("ORH_DEVICE")) dev = std::atoi(e);
    const int rc = orh_create(dev, 0, &lanes[lane]);
    if (rc != ORH_OK)
      throw std::runtime_error("libopenr_hip: orh_create for lane " + std::to_string(lane) +
                               " failed (rc=" + std::to_string(rc) + ")");
  }
  return lanes[lane];
}

// ---- HoldableValue (LinkState.cpp:87-121) ---------------------------------
template <>
bool Holdable<bool>::update(bool v, Metric upTtl, Metric downTtl) {
  if (v == val_) return false;
  if (hasHold()) {
    held_.reset();
    ttl_ = 0;
  } else {
    ttl_ = (val_ && !v) ? upTtl : downTtl;  // clearing overload brings the link up
    if (ttl_ != 0) held_ = val_;
  }
  val_ = v;
  return !hasHold();
}

template <>
bool Holdable<Metric>::update(Metric v, Metric upTtl, Metric downTtl) {
  if (v == val_) return false;
  if (hasHold()) {
    held_.reset();
    ttl_ = 0;
  } else {
    ttl_ = (v < val_) ? upTtl : downTtl;  // a lower metric brings traffic up
    if (ttl_ != 0) held_ = val_;
  }
  val_ = v;
  return !hasHold();
}

bool Link::less(const Link& o) const {
  if (hash != o.hash) return hash < o.hash;
  return std::tie(on1, oif1, on2, oif2) < std::tie(o.on1, o.oif1, o.on2, o.oif2);
}

// ---- construction -------------------------------------------------------
uint64_t LinkState::nextStamp() { return nextGeneration(); }

LinkState::LinkState(const std::string& area, orh_ctx* ctx)
    : area_(area), stamp_(nextStamp()), ctx_(ctx ? ctx : defaultContext()),
      store_(std::make_shared<LinkStateStore>()), ids_(store_->ids), names_(store_->names),
      links_(store_->links), freeLinks_(store_->freeLinks), nLinks_(store_->nLinks),
      nodeLinks_(store_->nodeLinks), nodeOverloads_(store_->nodeOverloads),
      adjacencyDatabases_(store_->adjacencyDatabases) {
  check(ctx_, orh_graph_create(ctx_, &graph_), "orh_graph_create");
  store_->views.push_back(this);
}

LinkState::LinkState(LinkState& primary, orh_ctx* ctx)
    : area_(primary.area_), stamp_(nextStamp()), ctx_(ctx ? ctx : defaultContext()), replica_(true),
      store_(primary.store_), ids_(store_->ids), names_(store_->names), links_(store_->links),
      freeLinks_(store_->freeLinks), nLinks_(store_->nLinks), nodeLinks_(store_->nodeLinks),
      nodeOverloads_(store_->nodeOverloads), adjacencyDatabases_(store_->adjacencyDatabases) {
  if (primary.replica_) throw std::invalid_argument("LinkState: a replica of a replica");
  check(ctx_, orh_graph_create(ctx_, &graph_), "orh_graph_create");
  store_->views.push_back(this);  // structDirty_: the whole store uploads at first use
}

LinkState::~LinkState() {
  auto& v = store_->views;
  v.erase(std::remove(v.begin(), v.end(), this), v.end());
  if (graph_) orh_graph_destroy(graph_);
}

void LinkState::mutating() const {
  if (replica_) throw std::logic_error("LinkState: a device replica is updated through its primary");
}
void LinkState::markStruct() {
  for (LinkState* w : store_->views) w->structDirty_ = true;
}
void LinkState::markRow(uint32_t v) {
  for (LinkState* w : store_->views) w->rowsDirty_.insert(v);
}
void LinkState::markLink(uint32_t id) {
  for (LinkState* w : store_->views) w->patchLinks_.insert(id);
}
void LinkState::markNode(uint32_t v) {
  for (LinkState* w : store_->views) w->patchNodes_.insert(v);
}
void LinkState::newStamps() {
  for (LinkState* w : store_->views) w->stamp_ = nextStamp();
}

uint32_t LinkState::ensureNode(const std::string& n) {
  auto it = ids_.find(n);
  if (it != ids_.end()) return it->second;
  const uint32_t id = static_cast<uint32_t>(names_.size());
  ids_.emplace(n, id);
  names_.push_back(n);
  nodeLinks_.push_back(std::make_unique<LinkSet>(0, LinkIdHash{&links_}));
  markStruct();
  return id;
}

std::optional<uint32_t> LinkState::nodeId(const std::string& n) const {
  auto it = ids_.find(n);
  if (it == ids_.end()) return std::nullopt;
  return it->second;
}

LinkSet& LinkState::setOf(uint32_t v) { return *nodeLinks_[v]; }

size_t LinkState::numNodes() const {
  size_t n = 0;  // nodes with a link set entry (linkMap_ keys)
  for (const auto& s : nodeLinks_) n += s->empty() ? 0 : 1;
  return n;
}

std::vector<uint32_t> LinkState::linksFromNode(const std::string& n) const {
  auto id = nodeId(n);
  if (!id) return {};
  return std::vector<uint32_t>(nodeLinks_[*id]->begin(), nodeLinks_[*id]->end());
}

bool LinkState::isNodeOverloaded(const std::string& n) const {
  auto it = nodeOverloads_.find(n);
  return it != nodeOverloads_.end() && it->second.value();
}

std::optional<Link> LinkState::maybeMakeLink(const std::string& node, const Adjacency& adj) {
  // bidirectional only (LinkState.cpp:531-547)
  auto it = adjacencyDatabases_.find(adj.otherNodeName);
  if (it == adjacencyDatabases_.end()) return std::nullopt;
  for (const auto& o : it->second.adjacencies) {
    if (o.otherNodeName != node || adj.otherIfName != o.ifName || adj.ifName != o.otherIfName)
      continue;
    Link l;
    l.area = area_;
    l.n1 = ensureNode(node);
    l.n2 = ensureNode(adj.otherNodeName);
    l.if1 = adj.ifName;
    l.if2 = o.ifName;
    l.metric1.reset(static_cast<Metric>(static_cast<int64_t>(adj.metric)));
    l.metric2.reset(static_cast<Metric>(static_cast<int64_t>(o.metric)));
    l.overload1.reset(adj.isOverloaded);
    l.overload2.reset(o.isOverloaded);
    l.adjLabel1 = adj.adjLabel;
    l.adjLabel2 = o.adjLabel;
    l.nhV41 = adj.nextHopV4;
    l.nhV42 = o.nextHopV4;
    l.nhV61 = adj.nextHopV6;
    l.nhV62 = o.nextHopV6;
    const auto a = std::make_pair(node, adj.ifName);
    const auto b = std::make_pair(adj.otherNodeName, o.ifName);
    const auto& lo = (b < a) ? b : a;
    const auto& hi = (b < a) ? a : b;
    l.on1 = lo.first;
    l.oif1 = lo.second;
    l.on2 = hi.first;
    l.oif2 = hi.second;
    l.hash = linkHash(l.on1, l.oif1, l.on2, l.oif2);
    return l;
  }
  return std::nullopt;
}

bool LinkState::linkAlive(uint32_t id) const { return id < links_.size() && links_[id].alive; }

uint32_t LinkState::addLink(Link&& l) {  // LinkState.cpp:421-426
  uint32_t id;
  if (!freeLinks_.empty()) {
    id = freeLinks_.back();
    freeLinks_.pop_back();
    links_[id] = std::move(l);
  } else {
    id = static_cast<uint32_t>(links_.size());
    links_.push_back(std::move(l));
  }
  Link& k = links_[id];
  k.alive = true;
  // the reference inserts into firstNodeName()'s set, then secondNodeName()'s
  const uint32_t first = k.on1 == names_[k.n1] && k.oif1 == k.if1 ? k.n1 : k.n2;
  const uint32_t second = k.other(first);
  if (!setOf(first).insert(id).second || !setOf(second).insert(id).second)
    throw std::logic_error("LinkState: duplicate link");
  ++nLinks_;
  markRow(first);
  markRow(second);
  return id;
}

void LinkState::removeLink(uint32_t id) {  // LinkState.cpp:429-434
  Link& k = links_[id];
  const uint32_t first = k.on1 == names_[k.n1] && k.oif1 == k.if1 ? k.n1 : k.n2;
  setOf(first).erase(id);
  setOf(k.other(first)).erase(id);
  k.alive = false;
  freeLinks_.push_back(id);
  --nLinks_;
  markRow(first);
  markRow(k.other(first));
}

void LinkState::removeNode(uint32_t v) {  // LinkState.cpp:436-455
  std::vector<uint32_t> ids(setOf(v).begin(), setOf(v).end());
  for (uint32_t id : ids) {
    setOf(links_[id].other(v)).erase(id);
    markRow(links_[id].other(v));
    links_[id].alive = false;
    freeLinks_.push_back(id);
    --nLinks_;
  }
  setOf(v).clear();
  markRow(v);
  if (nodeOverloads_.erase(names_[v])) markNode(v);
}

std::vector<uint32_t> LinkState::orderedLinks(uint32_t v) const {
  std::vector<uint32_t> ids(nodeLinks_[v]->begin(), nodeLinks_[v]->end());
  std::sort(ids.begin(), ids.end(),
            [&](uint32_t a, uint32_t b) { return links_[a].less(links_[b]); });
  return ids;
}

bool LinkState::updateNodeOverloaded(const std::string& n, bool o, Metric up, Metric down) {
  auto it = nodeOverloads_.find(n);
  if (it != nodeOverloads_.end()) {
    const bool before = it->second.value();
    const bool changed = it->second.update(o, up, down);
    if (it->second.value() != before) markNode(*nodeId(n));
    return changed;
  }
  nodeOverloads_.emplace(n, Holdable<bool>(o));
  if (o) markNode(ensureNode(n));
  return false;  // a new node's overload bit is not a topology change
}

void LinkState::invalidate(bool topologyChanged) {
  if (!topologyChanged) return;
  for (LinkState* w : store_->views) w->dropMemo();
}

void LinkState::dropMemo() const {
  spfResults_.clear();
  spfMaps_.clear();
  kthPaths_.clear();
  kthLinkPaths_.clear();
  countedOnDevice_.clear();
}

// ---- mutators -------------------------------------------------------------
LinkStateChange LinkState::updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric up,
                                                   Metric down) {
  // LinkState.cpp:564-719
  mutating();
  LinkStateChange change;
  newStamps();
  const std::string& node = db.thisNodeName;
  const uint32_t v = ensureNode(node);
  AdjacencyDatabase prior = std::move(adjacencyDatabases_[node]);
  adjacencyDatabases_[node] = db;

  const std::vector<uint32_t> oldLinks = orderedLinks(v);
  std::vector<Link> newLinks;
  for (const auto& adj : db.adjacencies) {
    if (auto l = maybeMakeLink(node, adj)) newLinks.push_back(std::move(*l));
  }
  std::sort(newLinks.begin(), newLinks.end(),
            [](const Link& a, const Link& b) { return a.less(b); });

  change.topologyChanged |= updateNodeOverloaded(node, db.isOverloaded, up, down);
  change.nodeLabelChanged = prior.nodeLabel != db.nodeLabel;

  size_t ni = 0, oi = 0;
  while (ni < newLinks.size() || oi < oldLinks.size()) {
    if (ni < newLinks.size() && (oi == oldLinks.size() || newLinks[ni].less(links_[oldLinks[oi]]))) {
      Link& l = newLinks[ni++];
      l.holdUpTtl = up;
      change.topologyChanged |= l.isUp();
      addLink(std::move(l));
      continue;
    }
    if (oi < oldLinks.size() && (ni == newLinks.size() || links_[oldLinks[oi]].less(newLinks[ni]))) {
      change.topologyChanged |= links_[oldLinks[oi]].isUp();
      removeLink(oldLinks[oi++]);
      continue;
    }
    const Link& nl = newLinks[ni++];
    const uint32_t id = oldLinks[oi++];
    Link& ol = links_[id];
    const bool side1 = ol.is1(v);
    const bool nside1 = nl.is1(v);
    auto& om = side1 ? ol.metric1 : ol.metric2;
    const Metric nm = nside1 ? nl.metric1.value() : nl.metric2.value();
    if (nm != om.value()) {
      change.topologyChanged |= om.update(nm, up, down);
      markLink(id);
    }
    auto& oo = side1 ? ol.overload1 : ol.overload2;
    const bool no = nside1 ? nl.overload1.value() : nl.overload2.value();
    if (no != oo.value()) {
      const bool wasUp = ol.isUp();
      oo.update(no, up, down);
      change.topologyChanged |= wasUp != ol.isUp();
      markLink(id);
    }
    const int32_t nlab = nside1 ? nl.adjLabel1 : nl.adjLabel2;
    if (nlab != ol.adjLabelFrom(v)) {
      change.linkAttributesChanged = true;
      (side1 ? ol.adjLabel1 : ol.adjLabel2) = nlab;
    }
    const BinaryAddress& n4 = nside1 ? nl.nhV41 : nl.nhV42;
    if (n4 != ol.nhV4From(v)) {
      change.linkAttributesChanged = true;
      (side1 ? ol.nhV41 : ol.nhV42) = n4;
    }
    const BinaryAddress& n6 = nside1 ? nl.nhV61 : nl.nhV62;
    if (n6 != ol.nhV6From(v)) {
      change.linkAttributesChanged = true;
      (side1 ? ol.nhV61 : ol.nhV62) = n6;
    }
  }
  invalidate(change.topologyChanged);
  return change;
}

LinkStateChange LinkState::deleteAdjacencyDatabase(const std::string& node) {
  mutating();
  LinkStateChange c;  // LinkState.cpp:721-738
  newStamps();
  auto it = adjacencyDatabases_.find(node);
  if (it == adjacencyDatabases_.end()) return c;
  removeNode(*nodeId(node));
  adjacencyDatabases_.erase(it);
  c.topologyChanged = true;
  invalidate(true);
  return c;
}

LinkStateChange LinkState::decrementHolds() {  // LinkState.cpp:500-514
  mutating();
  LinkStateChange c;
  newStamps();
  for (uint32_t id = 0; id < links_.size(); ++id) {
    Link& l = links_[id];
    if (!l.alive) continue;
    bool expired = false;
    if (l.holdUpTtl != 0) expired |= (--l.holdUpTtl == 0);
    expired |= l.metric1.decrementTtl();
    expired |= l.metric2.decrementTtl();
    expired |= l.overload1.decrementTtl();
    expired |= l.overload2.decrementTtl();
    if (expired) markLink(id);
    c.topologyChanged |= expired;
  }
  for (auto& [name, hv] : nodeOverloads_) {
    if (hv.decrementTtl()) {
      c.topologyChanged = true;
      markNode(*nodeId(name));
    }
  }
  invalidate(c.topologyChanged);
  return c;
}

bool LinkState::hasHolds() const {
  for (const auto& l : links_) {
    if (l.alive && (l.holdUpTtl != 0 || l.metric1.hasHold() || l.metric2.hasHold() ||
                    l.overload1.hasHold() || l.overload2.hasHold()))
      return true;
  }
  for (const auto& kv : nodeOverloads_)
    if (kv.second.hasHold()) return true;
  return false;
}

// ---- device mirror -----------------------------------------------------------
void LinkState::flushMirror() const {
  const uint32_t N = static_cast<uint32_t>(names_.size());
  if (!structDirty_ && !rowsDirty_.empty()) {
    // links added / removed, node set unchanged: rewrite only the changed
    // rows (in LinkSet order) inside their load-time capacity
    std::vector<uint32_t> rows(rowsDirty_.begin(), rowsDirty_.end()), ptr(1, 0), col, wout, win, meta;
    std::sort(rows.begin(), rows.end());
    bool fits = true;
    for (uint32_t v : rows) {
      if (nodeLinks_[v]->size() > rowPtr_[v + 1] - rowPtr_[v]) {
        fits = false;
        break;
      }
      for (uint32_t id : *nodeLinks_[v]) {
        const Link& l = links_[id];
        const uint32_t u = l.other(v);
        const bool up = l.isUp();
        col.push_back(u);
        wout.push_back(up ? toDeviceMetric(l.metricFrom(v)) : 1u);
        win.push_back(up ? toDeviceMetric(l.metricFrom(u)) : 1u);
        meta.push_back(id | (up ? 0u : ORH_META_DOWN));
      }
      ptr.push_back(static_cast<uint32_t>(col.size()));
    }
    const int rc = fits ? orh_graph_apply_delta(graph_, static_cast<uint32_t>(rows.size()), rows.data(),
                                                ptr.data(), col.data(), wout.data(), win.data(),
                                                meta.data(), static_cast<uint32_t>(links_.size()))
                        : ORH_E_UNSUPPORTED;
    if (rc == ORH_OK) {
      ++mirrorDeltas_;
      entriesOfLink_.resize(links_.size(), {0u, 0u});
      for (uint32_t v : rows) {
        uint32_t e = rowPtr_[v];
        for (uint32_t id : *nodeLinks_[v]) {
          const Link& l = links_[id];
          col_[e] = l.other(v);
          linkOfEntry_[e] = id;
          (l.is1(v) ? entriesOfLink_[id].first : entriesOfLink_[id].second) = e;
          ++e;
        }
        for (; e < rowPtr_[v + 1]; ++e) {
          col_[e] = v;
          linkOfEntry_[e] = ~0u;
        }
      }
      rowsDirty_.clear();
    } else if (rc == ORH_E_UNSUPPORTED) {
      structDirty_ = true;  // a row outgrew its capacity: reload
    } else {
      check(ctx_, rc, "orh_graph_apply_delta");
    }
  }
  if (structDirty_) {
    KspProf prof;
    // rows sized from the link sets, then filled per node on the pool (C4's
    // 50k-node WAN: ~38 ms on one thread, mostly cache misses into links_)
    rowPtr_.assign(N + 1, 0);
    for (uint32_t v = 0; v < N; ++v)
      rowPtr_[v + 1] = rowPtr_[v] + static_cast<uint32_t>(nodeLinks_[v]->size());
    const uint32_t E = rowPtr_[N];
    col_.assign(E, 0u);
    linkOfEntry_.assign(E, 0u);
    std::vector<uint32_t> wout(E), win(E), meta(E);
    std::vector<uint8_t> ovl(N, 0);
    entriesOfLink_.assign(links_.size(), {0u, 0u});
    auto fillCsr = [&](size_t, size_t lo, size_t hi) {
      for (size_t v = lo; v < hi; ++v) {
        uint32_t e = rowPtr_[v];
        for (uint32_t id : *nodeLinks_[v]) {  // LinkSet iteration order
          const Link& l = links_[id];
          const uint32_t x = static_cast<uint32_t>(v), u = l.other(x);
          col_[e] = u;
          linkOfEntry_[e] = id;
          const bool up = l.isUp();
          wout[e] = up ? toDeviceMetric(l.metricFrom(x)) : 1u;
          win[e] = up ? toDeviceMetric(l.metricFrom(u)) : 1u;
          meta[e] = id | (up ? 0u : ORH_META_DOWN);
          auto& eo = entriesOfLink_[id];  // the two ends are distinct fields
          (l.is1(x) ? eo.first : eo.second) = e;
          ++e;
        }
        ovl[v] = isNodeOverloaded(names_[v]) ? 1 : 0;
      }
    };
    auto& pool = WorkerPool::instance();
    const bool par = N >= 4096 && pool.size() > 1;
    if (par) pool.parallelFor(N, fillCsr);
    else fillCsr(0, 0, N);
    // DijkstraQ ties break on the node name (LinkState.h:488-498): names are
    // unique, so chunks sorted on the pool and merged give std::sort's order
    std::vector<std::pair<std::string_view, uint32_t>> byName(N);
    for (uint32_t v = 0; v < N; ++v) byName[v] = {names_[v], v};
    auto less = [](const std::pair<std::string_view, uint32_t>& a,
                   const std::pair<std::string_view, uint32_t>& b) { return a.first < b.first; };
    if (par) {
      const size_t P = pool.size();
      auto at = [&](size_t c) { return byName.begin() + static_cast<std::ptrdiff_t>(N * std::min(c, P) / P); };
      pool.parallelFor(P, [&](size_t, size_t b, size_t e) {
        for (size_t c = b; c < e; ++c) std::sort(at(c), at(c + 1), less);
      });
      for (size_t w = 1; w < P; w *= 2) {
        const size_t groups = (P + 2 * w - 1) / (2 * w);
        pool.parallelFor(groups, [&](size_t, size_t b, size_t e) {
          for (size_t k = b; k < e; ++k)
            std::inplace_merge(at(2 * w * k), at(2 * w * k + w), at(2 * w * k + 2 * w), less);
        });
      }
    } else {
      std::sort(byName.begin(), byName.end(), less);
    }
    std::vector<uint32_t> nameRank(N);
    for (uint32_t r = 0; r < N; ++r) nameRank[byName[r].second] = r;
    prof.mark("mirror: host CSR");
    orh_csr c{};
    c.n_nodes = N;
    c.name_rank = nameRank.data();
    c.n_edges = static_cast<uint32_t>(col_.size());
    c.n_links = static_cast<uint32_t>(links_.size());
    c.row_ptr = rowPtr_.data();
    c.col = col_.data();
    c.w_out = wout.data();
    c.w_in = win.data();
    c.meta = meta.data();
    c.node_overloaded = ovl.data();
    check(ctx_, orh_graph_load(graph_, &c), "orh_graph_load");
    prof.mark("mirror: orh_graph_load");
    ++mirrorLoads_;
    structDirty_ = false;
    rowsDirty_.clear();
    patchLinks_.clear();
    patchNodes_.clear();
    return;
  }
  if (!patchLinks_.empty()) {
    std::vector<uint32_t> idx, wout, win, meta;
    for (uint32_t id : patchLinks_) {
      const Link& l = links_[id];
      if (!l.alive) continue;
      const bool up = l.isUp();
      for (int s = 0; s < 2; ++s) {
        const uint32_t v = s == 0 ? l.n1 : l.n2;
        const uint32_t e = s == 0 ? entriesOfLink_[id].first : entriesOfLink_[id].second;
        idx.push_back(e);
        wout.push_back(up ? toDeviceMetric(l.metricFrom(v)) : 1u);
        win.push_back(up ? toDeviceMetric(l.metricFrom(l.other(v))) : 1u);
        meta.push_back(id | (up ? 0u : ORH_META_DOWN));
      }
    }
    check(ctx_, orh_graph_patch_edges(graph_, static_cast<uint32_t>(idx.size()), idx.data(),
                                      wout.data(), win.data(), meta.data()),
          "orh_graph_patch_edges");
    patchLinks_.clear();
  }
  if (!patchNodes_.empty()) {
    std::vector<uint32_t> idx;
    std::vector<uint8_t> ovl;
    for (uint32_t v : patchNodes_) {
      idx.push_back(v);
      ovl.push_back(isNodeOverloaded(names_[v]) ? 1 : 0);
    }
    check(ctx_, orh_graph_patch_nodes(graph_, static_cast<uint32_t>(idx.size()), idx.data(),
                                      ovl.data()),
          "orh_graph_patch_nodes");
    patchNodes_.clear();
  }
}

orh_graph* LinkState::deviceGraph() const {
  flushMirror();
  return graph_;
}

void LinkState::fillRows(const std::vector<uint32_t>& srcIds, bool useLinkMetric,
                         const orh_spf_request& req, std::vector<SpfRow>& rows) const {
  const uint32_t N = static_cast<uint32_t>(names_.size());
  const uint32_t n = static_cast<uint32_t>(srcIds.size());
  uint32_t words = 1, flags = 0;
  check(ctx_, orh_spf_words(graph_, srcIds.data(), n, &words), "orh_spf_words");
  check(ctx_, orh_graph_flags(graph_, &flags), "orh_graph_flags");
  const size_t nd = static_cast<size_t>(n) * N;
  std::vector<uint32_t> nh, order;
  std::vector<uint64_t> dist64;
  // zero-metric links / 64-bit path metrics: the reference's extraction order
  // decides the first hops and the pathLinks order (LinkState.cpp:808-882)
  const bool exact = useLinkMetric && flags != 0;
  if (exact) nh.resize(nd * words);
  const bool wide = useLinkMetric && (flags & ORH_GRAPH_WIDE_METRIC);
  if (exact) {
    dist64.resize(nd);
    order.resize(nd);
    check(ctx_, orh_spf_batch_exact(graph_, &req, words, dist64.data(), nh.data(), order.data()),
          "orh_spf_batch_exact");
  } else {
    // rows land in the context's pinned buffer; copied out per row below
    const uint32_t *hd = nullptr, *hn = nullptr;
    KspProf prof;
    check(ctx_, orh_spf_batch_pinned(graph_, &req, words, &hd, &hn), "orh_spf_batch_pinned");
    prof.mark("rows: device + D2H");
    auto fill = [&](size_t, size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        const size_t b = i * N;
        rows[i].dist.assign(hd + b, hd + b + N);
        rows[i].nh.assign(hn + b * words, hn + (b + N) * words);
      }
    };
    if (n > 1) WorkerPool::instance().parallelFor(n, fill);
    else fill(0, 0, n);
    prof.mark("rows: host copies");
  }
  for (uint32_t i = 0; i < n; ++i) {
    SpfRow& row = rows[i];
    const uint32_t src = srcIds[i];
    const size_t b = static_cast<size_t>(i) * N;
    row.srcName = names_[src];
    row.src = src;
    row.known = true;
    row.useLinkMetric = useLinkMetric;
    row.words = words;
    row.n = N;
    if (!exact) {
      // filled from the pinned rows above
    } else if (wide) {
      row.dist64.assign(dist64.begin() + b, dist64.begin() + b + N);
    } else {  // path metrics < 2^32 - 1: the u32 row (route selection reads it)
      row.dist.resize(N);
      for (uint32_t v = 0; v < N; ++v)
        row.dist[v] = dist64[b + v] == ~0ull ? ORH_UNREACHABLE : static_cast<uint32_t>(dist64[b + v]);
    }
    if (exact) {
      row.order.assign(order.begin() + b, order.begin() + b + N);
      row.nh.assign(nh.begin() + b * words, nh.begin() + (b + N) * words);
    }
    uint32_t nn = 0;
    check(ctx_, orh_graph_neighbors(graph_, src, nullptr, 0, &nn), "orh_graph_neighbors");
    row.nbrs.resize(nn);
    check(ctx_, orh_graph_neighbors(graph_, src, row.nbrs.data(), nn, &nn), "orh_graph_neighbors");
  }
  spfRuns_ += n;
}

SpfRow LinkState::spfOnDevice(uint32_t src, bool useLinkMetric,
                              const std::vector<uint32_t>* ignore) const {
  flushMirror();
  uint32_t ptr[2] = {0, ignore ? static_cast<uint32_t>(ignore->size()) : 0u};
  orh_spf_request req{};
  req.h_srcs = &src;
  req.n_src = 1;
  req.use_link_metric = useLinkMetric ? 1 : 0;
  if (ignore && !ignore->empty()) {
    req.h_ignore_ptr = ptr;
    req.h_ignore_links = ignore->data();
  }
  std::vector<SpfRow> rows(1);
  fillRows({src}, useLinkMetric, req, rows);
  return std::move(rows[0]);
}

std::vector<SpfRow> LinkState::runSpfBatch(
    const std::vector<uint32_t>& srcIds, bool useLinkMetric,
    const std::vector<std::vector<uint32_t>>* ignoreSets) const {
  std::vector<SpfRow> rows(srcIds.size());
  if (srcIds.empty()) return rows;
  flushMirror();
  std::vector<uint32_t> ptr, flat;
  orh_spf_request req{};
  req.h_srcs = srcIds.data();
  req.n_src = static_cast<uint32_t>(srcIds.size());
  req.use_link_metric = useLinkMetric ? 1 : 0;
  if (ignoreSets) {
    if (ignoreSets->size() != srcIds.size())
      throw std::invalid_argument("runSpfBatch: one ignore set per source");
    ptr.push_back(0);
    for (const auto& ign : *ignoreSets) {
      flat.insert(flat.end(), ign.begin(), ign.end());
      ptr.push_back(static_cast<uint32_t>(flat.size()));
    }
    req.h_ignore_ptr = ptr.data();
    req.h_ignore_links = flat.empty() ? ptr.data() : flat.data();
  }
  fillRows(srcIds, useLinkMetric, req, rows);
  return rows;
}

void LinkState::prefetchSpfResults(const std::vector<std::string>& nodes,
                                   bool useLinkMetric) const {
  std::vector<uint32_t> ids;
  std::unordered_set<uint32_t> seen;
  for (const auto& nm : nodes) {
    if (spfResults_.count({nm, useLinkMetric})) continue;
    auto id = nodeId(nm);
    if (id && seen.insert(*id).second) ids.push_back(*id);
  }
  auto rows = runSpfBatch(ids, useLinkMetric, nullptr);
  for (auto& r : rows) {
    std::string name = r.srcName;
    spfResults_.emplace(std::make_pair(std::move(name), useLinkMetric), std::move(r));
  }
}

void LinkState::prefetchKthPaths(const std::vector<std::pair<std::string, std::string>>& pairs) const {
  // the whole batch on the device (orh_ksp2_batch: k = 1 rows and traces, k = 2
  // searches and traces); only the paths come back. Graphs that need the
  // exact kernel's extraction order, unknown nodes and pairs that outgrow the
  // device trace's bounds take the host path below.
  KspProf prof;
  std::vector<const std::pair<std::string, std::string>*> dev;
  std::vector<std::pair<std::string, std::string>> host;
  std::vector<uint32_t> hs, hd;
  {
    std::unordered_set<std::pair<std::string, std::string>, StrPairHash> seen;
    seen.reserve(pairs.size());
    kthPaths_.reserve(2 * pairs.size());  // per shard: its share on top of what it holds
    for (const auto& pr : pairs) {
      if (!seen.insert(pr).second) continue;
      const bool any = !kthPaths_.empty();  // (a cold batch skips the key copies)
      const bool m1 = any && kthPaths_.count(std::make_tuple(pr.first, pr.second, size_t{1})) != 0;
      const bool m2 = any && kthPaths_.count(std::make_tuple(pr.first, pr.second, size_t{2})) != 0;
      if (m1 && m2) continue;
      auto s = nodeId(pr.first);
      auto d = nodeId(pr.second);
      if (!s || !d || m1 || m2) {  // partly memoized, or the reference's unknown-node results
        host.push_back(pr);
        continue;
      }
      dev.push_back(&pr);
      hs.push_back(*s);
      hd.push_back(*d);
    }
  }
  // ORH_KSP_HOST=1: host traces over device rows for every pair (A/B, tests)
  if (const char* e = getenv("ORH_KSP_HOST"); e && *e == '1') {
    for (const auto* pr : dev) host.push_back(*pr);
    dev.clear();
  }
  if (!dev.empty()) {
    flushMirror();
    const uint32_t* blocks = nullptr;
    uint32_t bw = 0;
    const int rc = orh_ksp2_batch(graph_, static_cast<uint32_t>(dev.size()), hs.data(), hd.data(), &blocks, &bw);
    if (rc == ORH_E_UNSUPPORTED) {
      for (const auto* pr : dev) host.push_back(*pr);
    } else {
      check(ctx_, rc, "orh_ksp2_batch");
      prof.mark("device batch");
      // spf_runs the reference's way: one per source not yet memoized
      // (getSpfResult), one per pair with k = 1 paths (runSpf ignoring them)
      std::unordered_set<std::string> srcCounted;
      // the pairs' path blocks -> vectors and memo keys on the pool, then
      // the memo's 16 shards filled on the pool (a shard by one thread)
      std::vector<std::pair<std::vector<Path>, std::vector<Path>>> parsed(dev.size());
      using MemoKey = KthMemo<std::vector<Path>>::Key;
      std::vector<std::pair<MemoKey, MemoKey>> keys(dev.size());
      // the keys' shards, computed with the keys: the fill below must not
      // hash a key another shard's thread may be moving out
      std::vector<std::pair<uint8_t, uint8_t>> keyShard(dev.size());
      auto parseRange = [&](size_t, size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
          const uint32_t* b = blocks + i * static_cast<size_t>(bw);
          if (b[0] != 0) continue;
          keys[i] = {MemoKey(dev[i]->first, dev[i]->second, 1), MemoKey(dev[i]->first, dev[i]->second, 2)};
          keyShard[i] = {static_cast<uint8_t>(KthMemo<std::vector<Path>>::shardOf(keys[i].first)),
                         static_cast<uint8_t>(KthMemo<std::vector<Path>>::shardOf(keys[i].second))};
          auto parse = [&](size_t w, std::vector<Path>& out) {
            const uint32_t n = b[w++];
            out.reserve(n);
            for (uint32_t k = 0; k < n; ++k) {
              const uint32_t len = b[w++];
              out.emplace_back(b + w, b + w + len);
              w += len;
            }
          };
          parse(2, parsed[i].first);
          parse(b[1], parsed[i].second);
        }
      };
      if (dev.size() >= 64) WorkerPool::instance().parallelFor(dev.size(), parseRange);
      else parseRange(0, 0, dev.size());
      for (size_t i = 0; i < dev.size(); ++i) {
        const uint32_t* b = blocks + i * static_cast<size_t>(bw);
        if (b[0] != 0) {
          host.push_back(*dev[i]);
          continue;
        }
        ++kspDevicePairs_;
        std::vector<Path>& k1 = parsed[i].first;
        std::vector<Path>& k2 = parsed[i].second;
        const std::string& src = dev[i]->first;
        if (!spfResults_.count({src, true}) && !countedOnDevice_.count(src) && srcCounted.insert(src).second) {
          ++spfRuns_;
          countedOnDevice_.insert(src);
        }
        if (!k1.empty()) ++spfRuns_;
        (void)k2;
      }
      auto fill = [&](size_t, size_t lo, size_t hi) {
        for (size_t sh = lo; sh < hi; ++sh) {
          auto& m = kthPaths_.shard(sh);
          for (size_t i = 0; i < dev.size(); ++i) {
            const uint32_t* b = blocks + i * static_cast<size_t>(bw);
            if (b[0] != 0) continue;
            if (keyShard[i].first == sh) m.emplace(std::move(keys[i].first), std::move(parsed[i].first));
            if (keyShard[i].second == sh) m.emplace(std::move(keys[i].second), std::move(parsed[i].second));
          }
        }
      };
      if (dev.size() >= 64) WorkerPool::instance().parallelFor(KthMemo<std::vector<Path>>::kShards, fill, KthMemo<std::vector<Path>>::kShards);
      else fill(0, 0, KthMemo<std::vector<Path>>::kShards);
      prof.mark("paths");
    }
  }
  kspHostPairs_ += host.size();
  if (!host.empty()) prefetchKthPathsHost(host);
}

void LinkState::prefetchKthPathsHost(const std::vector<std::pair<std::string, std::string>>& pairs) const {
  // k = 1: traces over the memoized SPF of each source (batched)
  KspProf prof;
  std::vector<std::string> srcs;
  for (const auto& pr : pairs) srcs.push_back(pr.first);
  prefetchSpfResults(srcs, true);
  prof.mark("k=1 rows");
  // k = 1 traces over the memoized rows, independent per pair: on the pool
  {
    std::vector<const std::pair<std::string, std::string>*> need;
    std::vector<const SpfRow*> rows1;
    std::set<std::pair<std::string, std::string>> seen;
    for (const auto& pr : pairs) {
      if (kthPaths_.count(std::make_tuple(pr.first, pr.second, size_t{1}))) continue;
      if (!seen.insert(pr).second) continue;
      need.push_back(&pr);
      rows1.push_back(&getSpfRow(pr.first, true));
    }
    std::vector<std::vector<Path>> traced(need.size());
    auto trace = [&](size_t, size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) traced[i] = traceKthPaths(need[i]->first, need[i]->second, *rows1[i], nullptr);
    };
    if (need.size() > 8) WorkerPool::instance().parallelFor(need.size(), trace);
    else trace(0, 0, need.size());
    for (size_t i = 0; i < need.size(); ++i)
      {
        auto key = std::make_tuple(need[i]->first, need[i]->second, size_t{1});
        kthPaths_.of(key).emplace(std::move(key), std::move(traced[i]));
      }
  }
  prof.mark("k=1 traces");
  // k = 2: one fresh SPF per pair with its k = 1 links ignored, all in one launch
  std::vector<uint32_t> ids;
  std::vector<std::vector<uint32_t>> ign;
  std::vector<const std::pair<std::string, std::string>*> todo;
  std::set<std::pair<std::string, std::string>> queued;
  for (const auto& pr : pairs) {
    if (kthPaths_.count(std::make_tuple(pr.first, pr.second, size_t{2}))) continue;
    if (!queued.insert(pr).second) continue;
    std::unordered_set<uint32_t> s;
    for (const auto& p : getKthPathIds(pr.first, pr.second, 1))
      for (uint32_t lid : p) s.insert(lid);
    auto id = nodeId(pr.first);
    if (s.empty() || !id) {
      getKthPathIds(pr.first, pr.second, 2);  // no re-run needed (memoized row)
      continue;
    }
    ids.push_back(*id);
    ign.emplace_back(s.begin(), s.end());
    todo.push_back(&pr);
  }
  prof.mark("k=2 ignore sets");
  auto rows = runSpfBatch(ids, true, &ign);
  prof.mark("k=2 rows");
  std::vector<std::vector<Path>> traced(todo.size());
  auto trace = [&](size_t, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const std::unordered_set<uint32_t> ignore(ign[i].begin(), ign[i].end());
      traced[i] = traceKthPaths(todo[i]->first, todo[i]->second, rows[i], &ignore);
    }
  };
  if (todo.size() > 8) WorkerPool::instance().parallelFor(todo.size(), trace);
  else trace(0, 0, todo.size());
  for (size_t i = 0; i < todo.size(); ++i)
    {
      auto key = std::make_tuple(todo[i]->first, todo[i]->second, size_t{2});
      kthPaths_.of(key).emplace(std::move(key), std::move(traced[i]));
    }
  prof.mark("k=2 traces");
}

const SpfRow& LinkState::getSpfRow(const std::string& node, bool useLinkMetric) const {
  auto key = std::make_pair(node, useLinkMetric);
  auto it = spfResults_.find(key);
  if (it != spfResults_.end()) return it->second;
  auto id = nodeId(node);
  SpfRow row;
  if (id) {
    row = spfOnDevice(*id, useLinkMetric, nullptr);
    if (useLinkMetric && countedOnDevice_.erase(node)) --spfRuns_;  // counted by a KSP2 batch
  } else {
    // unknown source: the reference result holds only the source itself
    row.srcName = node;
    row.known = false;
    row.useLinkMetric = useLinkMetric;
    ++spfRuns_;
  }
  return spfResults_.emplace(key, std::move(row)).first->second;
}

const SpfResult& LinkState::getSpfResult(const std::string& node, bool useLinkMetric) const {
  auto key = std::make_pair(node, useLinkMetric);
  auto it = spfMaps_.find(key);
  if (it != spfMaps_.end()) return it->second;
  const SpfRow& row = getSpfRow(node, useLinkMetric);
  SpfResult res;
  if (!row.known) {
    res.emplace(node, NodeSpfResult(0));  // only the source itself (LinkState.cpp:817-819)
  } else {
    res.reserve(row.n);
    for (uint32_t v = 0; v < row.n; ++v) {
      if (!row.reachable(v)) continue;
      NodeSpfResult r(row.metric(v));
      row.forEachNextHop(v, [&](uint32_t nb) { r.addNextHop(names_[nb]); });
      for (const auto& [lid, prev] : pathLinks(row, v)) r.addPath(LinkRef(this, lid), names_[prev]);
      res.emplace(names_[v], std::move(r));
    }
  }
  return spfMaps_.emplace(key, std::move(res)).first->second;
}

SpfRow LinkState::runSpf(const std::string& node, bool useLinkMetric,
                         const std::vector<uint32_t>& ignore) const {
  auto id = nodeId(node);
  if (!id) {
    SpfRow row;
    row.srcName = node;
    row.useLinkMetric = useLinkMetric;
    ++spfRuns_;
    return row;
  }
  return spfOnDevice(*id, useLinkMetric, &ignore);
}

std::optional<Metric> LinkState::getMetricFromAToB(const std::string& a, const std::string& b,
                                                   bool useLinkMetric) const {
  if (a == b) return 0;  // LinkState.cpp:740-751
  const SpfRow& row = getSpfRow(a, useLinkMetric);
  auto id = nodeId(b);
  if (!id || !row.reachable(*id)) return std::nullopt;
  return row.metric(*id);
}

Metric LinkState::getMaxHopsToNode(const std::string& node) const {
  const SpfRow& row = getSpfRow(node, false);  // LinkState.cpp:753-760
  Metric mx = 0;
  if (!row.known) return 0;
  for (uint32_t v = 0; v < row.n; ++v)
    if (row.reachable(v)) mx = std::max(mx, row.metric(v));
  return mx;
}

// ---- K-shortest edge-disjoint paths -----------------------------------------
std::vector<std::pair<uint32_t, uint32_t>> LinkState::pathLinks(
    const SpfRow& row, uint32_t v, const std::unordered_set<uint32_t>* ignore) const {
  // predecessors (link, prev) of v in the order runSpf appends them: by
  // extraction order of prev - (dist, name) for metrics >= 1, the recorded
  // order of exact rows - then prev's LinkSet iteration order
  // (LinkState.cpp:821-873). A prev extracted after v (possible only over a
  // zero-metric link) never relaxed v.
  struct Cand {
    Metric dist;
    const std::string* name;
    uint32_t pos;
    uint32_t link;
    uint32_t prev;
  };
  std::vector<Cand> cands;
  if (!row.reachable(v) || v == row.src) return {};
  for (uint32_t id : *nodeLinks_[v]) {
    const Link& l = links_[id];
    if (!l.isUp() || (ignore && ignore->count(id))) continue;
    const uint32_t u = l.other(v);
    if (!row.reachable(u)) continue;
    if (u != row.src && isNodeOverloaded(names_[u])) continue;
    const Metric w = row.useLinkMetric ? l.metricFrom(u) : 1;
    if (row.metric(u) + w != row.metric(v)) continue;
    if (!row.order.empty() && row.order[u] > row.order[v]) continue;
    uint32_t pos = 0;
    for (uint32_t x : *nodeLinks_[u]) {
      if (x == id) break;
      ++pos;
    }
    cands.push_back({row.order.empty() ? row.metric(u) : row.order[u], &names_[u], pos, id, u});
  }
  std::sort(cands.begin(), cands.end(), [](const Cand& a, const Cand& b) {
    if (a.dist != b.dist) return a.dist < b.dist;  // the order rank for exact rows
    if (*a.name != *b.name) return *a.name < *b.name;
    return a.pos < b.pos;
  });
  std::vector<std::pair<uint32_t, uint32_t>> out;
  for (const auto& c : cands) out.emplace_back(c.link, c.prev);
  return out;
}

std::optional<Path> LinkState::traceOnePath(uint32_t src, uint32_t dst, const SpfRow& row,
                                            std::unordered_set<uint32_t>& visited,
                                            const std::unordered_set<uint32_t>* ignore) const {
  // greedy DFS dst -> src; a link is consumed on first touch (LinkState.cpp:398-419)
  if (src == dst) return Path{};
  for (const auto& [lid, prev] : pathLinks(row, dst, ignore)) {
    if (visited.insert(lid).second) {
      auto p = traceOnePath(src, prev, row, visited, ignore);
      if (p) {
        p->push_back(lid);
        return p;
      }
    }
  }
  return std::nullopt;
}

const std::vector<LinkPath>& LinkState::getKthPaths(const std::string& src, const std::string& dst,
                                                    size_t k) const {
  auto key = std::make_tuple(src, dst, k);
  auto& lmemo = kthLinkPaths_.of(key);
  auto it = lmemo.find(key);
  if (it != lmemo.end()) return it->second;
  std::vector<LinkPath> out;
  for (const auto& p : getKthPathIds(src, dst, k)) {
    LinkPath lp;
    lp.reserve(p.size());
    for (uint32_t lid : p) lp.emplace_back(this, lid);
    out.push_back(std::move(lp));
  }
  return kthLinkPaths_.of(key).emplace(key, std::move(out)).first->second;
}

const std::vector<Path>& LinkState::getKthPathIds(const std::string& src, const std::string& dst,
                                                  size_t k) const {
  if (k < 1) throw std::invalid_argument("getKthPaths: k must be >= 1");
  auto key = std::make_tuple(src, dst, k);
  auto& memo = kthPaths_.of(key);
  auto it = memo.find(key);
  if (it != memo.end()) return it->second;

  std::unordered_set<uint32_t> ignore;
  for (size_t i = 1; i < k; ++i)
    for (const auto& p : getKthPathIds(src, dst, i))
      for (uint32_t lid : p) ignore.insert(lid);

  std::vector<Path> paths;
  SpfRow fresh;
  const SpfRow* row;
  if (ignore.empty()) {
    row = &getSpfRow(src, true);
  } else {
    std::vector<uint32_t> ign(ignore.begin(), ignore.end());
    fresh = runSpf(src, true, ign);
    row = &fresh;
  }
  paths = traceKthPaths(src, dst, *row, ignore.empty() ? nullptr : &ignore);
  return kthPaths_.of(key).emplace(key, std::move(paths)).first->second;
}

std::vector<Path> LinkState::traceKthPaths(const std::string& src, const std::string& dst,
                                           const SpfRow& row,
                                           const std::unordered_set<uint32_t>* ignore) const {
  // successive greedy traces sharing one visited-link set (LinkState.cpp:778-791)
  std::vector<Path> paths;
  auto s = nodeId(src);
  auto d = nodeId(dst);
  const bool hasDst = (src == dst) || (s && d && row.reachable(*d));
  if (hasDst && s && d) {
    std::unordered_set<uint32_t> visited;
    auto p = traceOnePath(*s, *d, row, visited, ignore);
    while (p && !p->empty()) {
      paths.push_back(std::move(*p));
      p = traceOnePath(*s, *d, row, visited, ignore);
    }
  }
  return paths;
}

bool LinkState::pathAInPathB(const LinkPath& a, const LinkPath& b) {  // LinkState.h:395-410
  if (a.size() > b.size()) return false;
  for (size_t i = 0; i + a.size() <= b.size(); ++i) {
    size_t k = 0;
    while (k < a.size() && a[k] == b[i + k]) ++k;
    if (k == a.size()) return true;
  }
  return false;
}

// ---- LinkRef (LinkState.cpp:163-260, :347-360) -------------------------------
const Link& LinkRef::raw() const { return ls_->link(id_); }
bool LinkRef::end1(const std::string& nodeName) const {
  const Link& l = raw();
  if (ls_->nodeName(l.n1) == nodeName) return true;
  if (ls_->nodeName(l.n2) == nodeName) return false;
  throw std::invalid_argument(nodeName);
}
const std::string& LinkRef::getArea() const { return raw().area; }
const std::string& LinkRef::getOtherNodeName(const std::string& nodeName) const {
  return ls_->nodeName(end1(nodeName) ? raw().n2 : raw().n1);
}
const std::string& LinkRef::firstNodeName() const { return raw().on1; }
const std::string& LinkRef::secondNodeName() const { return raw().on2; }
const std::string& LinkRef::getIfaceFromNode(const std::string& nodeName) const {
  return end1(nodeName) ? raw().if1 : raw().if2;
}
Metric LinkRef::getMetricFromNode(const std::string& nodeName) const {
  return end1(nodeName) ? raw().metric1.value() : raw().metric2.value();
}
int32_t LinkRef::getAdjLabelFromNode(const std::string& nodeName) const {
  return end1(nodeName) ? raw().adjLabel1 : raw().adjLabel2;
}
bool LinkRef::getOverloadFromNode(const std::string& nodeName) const {
  return end1(nodeName) ? raw().overload1.value() : raw().overload2.value();
}
const BinaryAddress& LinkRef::getNhV4FromNode(const std::string& nodeName) const {
  return end1(nodeName) ? raw().nhV41 : raw().nhV42;
}
const BinaryAddress& LinkRef::getNhV6FromNode(const std::string& nodeName) const {
  return end1(nodeName) ? raw().nhV61 : raw().nhV62;
}
bool LinkRef::isUp() const { return raw().isUp(); }
bool LinkRef::hasHolds() const {
  const Link& l = raw();
  return l.holdUpTtl != 0 || l.metric1.hasHold() || l.metric2.hasHold() || l.overload1.hasHold() ||
         l.overload2.hasHold();
}
std::string LinkRef::toString() const {  // LinkState.cpp:363-366
  const Link& l = raw();
  return l.area + " - " + ls_->nodeName(l.n1) + "%" + l.if1 + " <---> " + ls_->nodeName(l.n2) + "%" + l.if2;
}
std::string LinkRef::directionalToString(const std::string& fromNode) const {  // :368-377
  return getArea() + " - " + fromNode + "%" + getIfaceFromNode(fromNode) + " ---> " +
         getOtherNodeName(fromNode) + "%" + getIfaceFromNode(getOtherNodeName(fromNode));
}
bool LinkRef::operator<(const LinkRef& o) const { return raw().less(o.raw()); }

bool LinkState::pathAInPathB(const Path& a, const Path& b) {  // LinkState.h:395-410
  if (a.size() > b.size()) return false;
  for (size_t i = 0; i + a.size() <= b.size(); ++i) {
    size_t k = 0;
    while (k < a.size() && a[k] == b[i + k]) ++k;
    if (k == a.size()) return true;
  }
  return false;
}

}  // namespace openr_amd
