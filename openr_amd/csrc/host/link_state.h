// Drop-in LinkState for the OpenR Decision module, backed by libopenr_hip.
//
// Public behaviour follows openr/decision/LinkState.h:177-469:
//   updateAdjacencyDatabase / deleteAdjacencyDatabase / decrementHolds with
//   the same LinkStateChange flags, bidirectional-link rule, ordered-FIB
//   holds and memo invalidation; getSpfResult / getKthPaths /
//   getMetricFromAToB / getMaxHopsToNode with the same results.
//
// What differs is where the SPF runs: the host keeps the graph store with
// dense node / link ids and mirrors it into a device CSR (orh_graph); every
// SPF (memoized per source, or fresh with links ignored for KSP2) is an
// orh_spf_* call on the GPU. The host never runs Dijkstra. Attribute-only
// changes (metric, overload, holds) are applied to the mirror as in-place
// patches; structural changes (links added or removed) re-upload it.
//
// Per-node link sets are std::unordered_set<link id> hashed with the
// reference Link::hash, so their iteration order -- which the reference's
// KSP2 trace depends on (LinkState.cpp:844, :398-419) -- is reproduced.
#pragma once

#include <map>
#include <memory>
#include <optional>
#include <string>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../../include/openr_hip.h"
#include "hash.h"
#include "host_types.h"

namespace openr_amd {

// process-wide libopenr_hip context of the device this process drives
// (ORH_DEVICE env or device 0); throws if no GPU is available
orh_ctx* defaultContext();

// context of stream lane `lane` on the same device: lane 0 is defaultContext(),
// lanes 1..kMaxLanes-1 are extra contexts (own HIP stream, own scratch) created
// on first use, so independent searches (what-if topologies) overlap on the GPU
constexpr unsigned kMaxLanes = 32;
orh_ctx* laneContext(unsigned lane);

template <class T>
class Holdable {  // HoldableValue, LinkState.h:36-58
 public:
  explicit Holdable(T v) : val_(v) {}
  void reset(T v) {
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
  bool update(T v, Metric upTtl, Metric downTtl);

 private:
  T val_;
  std::optional<T> held_;
  Metric ttl_{0};
};

struct Link {
  std::string area;
  uint32_t n1{0}, n2{0};  // node ids of the constructor's (nodeName1, nodeName2)
  std::string if1, if2;
  Holdable<Metric> metric1{1}, metric2{1};
  Holdable<bool> overload1{false}, overload2{false};
  int32_t adjLabel1{0}, adjLabel2{0};
  BinaryAddress nhV41, nhV42, nhV61, nhV62;
  Metric holdUpTtl{0};
  // orderedNames_ = minmax((name1, if1), (name2, if2))
  std::string on1, oif1, on2, oif2;
  size_t hash{0};
  bool alive{false};

  bool isUp() const { return holdUpTtl == 0 && !overload1.value() && !overload2.value(); }
  bool is1(uint32_t node) const { return node == n1; }
  uint32_t other(uint32_t node) const { return node == n1 ? n2 : n1; }
  const std::string& ifFrom(uint32_t node) const { return is1(node) ? if1 : if2; }
  Metric metricFrom(uint32_t node) const {
    return is1(node) ? metric1.value() : metric2.value();
  }
  int32_t adjLabelFrom(uint32_t node) const { return is1(node) ? adjLabel1 : adjLabel2; }
  bool overloadFrom(uint32_t node) const {
    return is1(node) ? overload1.value() : overload2.value();
  }
  const BinaryAddress& nhV4From(uint32_t node) const { return is1(node) ? nhV41 : nhV42; }
  const BinaryAddress& nhV6From(uint32_t node) const { return is1(node) ? nhV61 : nhV62; }
  bool less(const Link& o) const;  // Link::operator< (LinkState.cpp:347-353)
  bool same(const Link& o) const {
    return hash == o.hash && on1 == o.on1 && oif1 == o.oif1 && on2 == o.on2 && oif2 == o.oif2;
  }
};

using Path = std::vector<uint32_t>;  // link ids, src -> dst

class LinkState;

// A link of a LinkState in the shape the reference's callers use its
// std::shared_ptr<Link> (LinkState.h:82-175, getters LinkState.cpp:163-260):
// `link->getMetricFromNode(name)`, `link->getOtherNodeName(name)`, ... so
// code such as selectBestPathsKsp2's label / nexthop loop
// (Decision.cpp:1035-1076) compiles unchanged over getKthPaths' paths and
// NodeSpfResult::pathLinks. A node that is not an end of the link throws
// std::invalid_argument (LinkState.cpp:171). Valid while the LinkState
// lives; the id is the LinkState's link id (LinkState::link).
class LinkRef {
 public:
  LinkRef() = default;
  LinkRef(const LinkState* ls, uint32_t id) : ls_(ls), id_(id) {}
  const LinkRef* operator->() const { return this; }
  uint32_t id() const { return id_; }
  const Link& raw() const;

  const std::string& getArea() const;
  const std::string& getOtherNodeName(const std::string& nodeName) const;
  const std::string& firstNodeName() const;
  const std::string& secondNodeName() const;
  const std::string& getIfaceFromNode(const std::string& nodeName) const;
  Metric getMetricFromNode(const std::string& nodeName) const;
  int32_t getAdjLabelFromNode(const std::string& nodeName) const;
  bool getOverloadFromNode(const std::string& nodeName) const;
  const BinaryAddress& getNhV4FromNode(const std::string& nodeName) const;
  const BinaryAddress& getNhV6FromNode(const std::string& nodeName) const;
  bool isUp() const;
  bool hasHolds() const;
  std::string toString() const;
  std::string directionalToString(const std::string& fromNode) const;
  bool operator==(const LinkRef& o) const { return ls_ == o.ls_ && id_ == o.id_; }
  bool operator!=(const LinkRef& o) const { return !(*this == o); }
  bool operator<(const LinkRef& o) const;  // Link::operator< (hash, ordered names)

 private:
  bool end1(const std::string& nodeName) const;  // true: end 1, false: end 2, else throws
  const LinkState* ls_{nullptr};
  uint32_t id_{0};
};
using LinkPath = std::vector<LinkRef>;  // the reference's LinkState::Path (links src -> dst)

// One source's SPF result as produced by the device: dist row + first-hop
// bitmask row over the source's distinct neighbours (orh_graph_neighbors).
// Rows of the exact kernel (zero-metric links, or path metrics that can reach
// 2^32) also carry the extraction order; their distances are 64-bit when the
// graph's path metrics can exceed 32 bits.
struct SpfRow {
  std::string srcName;
  uint32_t src{0};
  bool known{false};  // src has a node id in this area
  bool useLinkMetric{true};
  uint32_t words{1};
  uint32_t n{0};                 // nodes in the row
  std::vector<uint32_t> dist;    // ORH_UNREACHABLE when absent (empty when dist64 is used)
  std::vector<uint64_t> dist64;  // ~0 when absent (wide-metric graphs only)
  std::vector<uint32_t> order;   // extraction order (exact rows only, ~0 when absent)
  std::vector<uint32_t> nh;      // [N * words]
  std::vector<uint32_t> nbrs;    // bit k <-> node id nbrs[k]

  bool reachable(uint32_t v) const {
    if (!known || v >= n) return false;
    return dist64.empty() ? dist[v] != ORH_UNREACHABLE : dist64[v] != ~0ull;
  }
  Metric metric(uint32_t v) const { return dist64.empty() ? Metric{dist[v]} : dist64[v]; }
  template <class F>
  void forEachNextHop(uint32_t v, F&& f) const {
    for (uint32_t k = 0; k < words; ++k) {
      uint32_t m = nh[static_cast<size_t>(v) * words + k];
      while (m) {
        const int b = __builtin_ctz(m);
        m &= m - 1;
        f(nbrs[k * 32 + b]);
      }
    }
  }
};

// LinkState::NodeSpfResult (LinkState.h:203-256): metric, the first-hop
// neighbour names and the (link, previous node) predecessors in the
// reference's pathLinks order; links are named by their LinkState id
// (LinkState::link(id)) instead of a shared_ptr<Link>
class NodeSpfResult {
 public:
  struct PathLink {  // LinkState.h:205-210
    LinkRef link;
    std::string prevNode;
  };
  explicit NodeSpfResult(Metric m) : metric_(m) {}
  Metric metric() const { return metric_; }
  const std::vector<PathLink>& pathLinks() const { return pathLinks_; }
  const std::unordered_set<std::string>& nextHops() const { return nextHops_; }
  void addPath(LinkRef link, const std::string& prevNode) { pathLinks_.push_back({link, prevNode}); }
  void addNextHop(const std::string& nh) { nextHops_.insert(nh); }

 private:
  Metric metric_;
  std::vector<PathLink> pathLinks_;
  std::unordered_set<std::string> nextHops_;
};
using SpfResult = std::unordered_map<std::string /* otherNodeName */, NodeSpfResult>;

// The host graph store of one area (node ids, links, per-node link sets,
// overloads, adjacency databases): owned by one LinkState and shared by its
// device replicas (LinkState's replica constructor), so a topology held on N
// devices is stored and updated on the host once (LinkState.cpp:564-719 run
// once), and every device mirror is patched from the same delta.
struct LinkIdHash {
  const std::vector<Link>* links;
  size_t operator()(uint32_t id) const { return (*links)[id].hash; }
};
using LinkSet = std::unordered_set<uint32_t, LinkIdHash>;

struct LinkStateStore {
  std::unordered_map<std::string, uint32_t> ids;
  std::vector<std::string> names;
  std::vector<Link> links;
  std::vector<uint32_t> freeLinks;
  size_t nLinks{0};
  std::vector<std::unique_ptr<LinkSet>> nodeLinks;
  std::unordered_map<std::string, Holdable<bool>> nodeOverloads;
  std::unordered_map<std::string, AdjacencyDatabase> adjacencyDatabases;
  std::vector<LinkState*> views;  // the owner first, then its device replicas
};

class LinkState {
 public:
  explicit LinkState(const std::string& area, orh_ctx* ctx = nullptr);
  // a device replica of `primary`: the same host store (nothing copied, no
  // update applied twice), its own device mirror on `ctx`, its own memo. The
  // store is mutated through the primary only; every mutation marks the
  // replicas' mirrors dirty and clears their memos as it does the primary's.
  // The primary outlives its replicas.
  LinkState(LinkState& primary, orh_ctx* ctx);
  ~LinkState();
  LinkState(LinkState&&) = delete;
  LinkState(const LinkState&) = delete;
  bool isReplica() const { return replica_; }

  const std::string& getArea() const { return area_; }

  LinkStateChange updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl = 0,
                                          Metric holdDownTtl = 0);
  LinkStateChange deleteAdjacencyDatabase(const std::string& node);
  LinkStateChange decrementHolds();
  bool hasHolds() const;

  // memoized SPF from `node` (LinkState.cpp:793-803) in the reference's
  // shape: reachable node name -> {metric, nextHops, pathLinks}
  // (LinkState.h:203-260, :271-272); built from the row on first use
  const SpfResult& getSpfResult(const std::string& node, bool useLinkMetric = true) const;
  // the same memoized SPF as the device row (dist + first-hop bitmask per
  // node): what route building reads, without materialising names
  const SpfRow& getSpfRow(const std::string& node, bool useLinkMetric = true) const;
  // fresh SPF with links ignored (runSpf(src, true, linksToIgnore))
  SpfRow runSpf(const std::string& node, bool useLinkMetric,
                const std::vector<uint32_t>& ignoreLinks) const;
  // getKthPaths (LinkState.cpp:762-791) as link ids (what the route build
  // reads) and in the reference's type, links as LinkRef handles
  // (LinkState.h:293-294); both memoized per (src, dst, k)
  const std::vector<Path>& getKthPathIds(const std::string& src, const std::string& dst,
                                         size_t k) const;
  const std::vector<LinkPath>& getKthPaths(const std::string& src, const std::string& dst,
                                           size_t k) const;

  // batched forms: one device launch for many SPFs (the reference runs them
  // one by one). runSpfBatch: sources by node id, optional per-source ignore
  // sets (what-if SPFs). prefetch*: fill the memos for many queries at once
  // (getSpfResult for every node; getKthPaths for every (src, dst) pair with
  // all k = 2 re-runs in one launch); later getSpfResult / getKthPaths calls
  // are memo hits with identical results.
  std::vector<SpfRow> runSpfBatch(const std::vector<uint32_t>& srcIds, bool useLinkMetric,
                                  const std::vector<std::vector<uint32_t>>* ignoreSets) const;
  void prefetchSpfResults(const std::vector<std::string>& nodes, bool useLinkMetric = true) const;
  void prefetchKthPaths(const std::vector<std::pair<std::string, std::string>>& pairs) const;
  // drop every memoized SPF row and k-th path set (what a topology change
  // does): benchmarks repeat a cold prefetch with it
  void dropMemo() const;
  // the same over host traces of device rows (exact-order graphs, pairs the
  // device trace flags)
  void prefetchKthPathsHost(const std::vector<std::pair<std::string, std::string>>& pairs) const;
  std::optional<Metric> getMetricFromAToB(const std::string& a, const std::string& b,
                                          bool useLinkMetric = true) const;
  Metric getMaxHopsToNode(const std::string& node) const;

  // pathLinks of `v` in `row` in the reference's insertion order
  std::vector<std::pair<uint32_t, uint32_t>> pathLinks(
      const SpfRow& row, uint32_t v, const std::unordered_set<uint32_t>* ignore = nullptr) const;
  static bool pathAInPathB(const Path& a, const Path& b);
  static bool pathAInPathB(const LinkPath& a, const LinkPath& b);

  bool hasNode(const std::string& n) const { return adjacencyDatabases_.count(n) != 0; }
  // unique across LinkState instances and renewed by every mutator: equal
  // stamps mean the same object in the same state
  uint64_t stateStamp() const { return stamp_; }
  bool isNodeOverloaded(const std::string& n) const;
  std::optional<uint32_t> nodeId(const std::string& n) const;
  const std::string& nodeName(uint32_t id) const { return names_[id]; }
  uint32_t numNodeIds() const { return static_cast<uint32_t>(names_.size()); }
  std::vector<uint32_t> linksFromNode(const std::string& n) const;  // LinkSet order
  const Link& link(uint32_t id) const { return links_[id]; }
  uint32_t numLinkSlots() const { return static_cast<uint32_t>(links_.size()); }
  bool linkAlive(uint32_t id) const;
  size_t numLinks() const { return nLinks_; }
  size_t numNodes() const;
  const std::unordered_map<std::string, AdjacencyDatabase>& getAdjacencyDatabases() const {
    return adjacencyDatabases_;
  }
  uint64_t spfRuns() const { return spfRuns_; }

  // device mirror access (bench / batch callers)
  orh_graph* deviceGraph() const;  // flushes pending deltas first
  // device mirror uploads so far: full orh_graph_load calls, row deltas
  std::pair<uint64_t, uint64_t> mirrorStats() const { return {mirrorLoads_, mirrorDeltas_}; }
  orh_ctx* context() const { return ctx_; }

 private:
  uint32_t ensureNode(const std::string& n);
  std::optional<Link> maybeMakeLink(const std::string& node, const Adjacency& adj);
  uint32_t addLink(Link&& l);
  void removeLink(uint32_t id);
  void removeNode(uint32_t v);
  bool updateNodeOverloaded(const std::string& n, bool o, Metric up, Metric down);
  std::vector<uint32_t> orderedLinks(uint32_t v) const;
  LinkSet& setOf(uint32_t v);
  void invalidate(bool topologyChanged);
  void flushMirror() const;
  SpfRow spfOnDevice(uint32_t src, bool useLinkMetric,
                     const std::vector<uint32_t>* ignore) const;
  // rows from the device for sources `srcIds` (the exact kernel when the
  // graph needs it); rows[i].src etc. filled in
  void fillRows(const std::vector<uint32_t>& srcIds, bool useLinkMetric, const orh_spf_request& req,
                std::vector<SpfRow>& rows) const;
  std::vector<Path> traceKthPaths(const std::string& src, const std::string& dst,
                                  const SpfRow& row,
                                  const std::unordered_set<uint32_t>* ignore) const;
  std::optional<Path> traceOnePath(uint32_t src, uint32_t dst, const SpfRow& row,
                                   std::unordered_set<uint32_t>& visited,
                                   const std::unordered_set<uint32_t>* ignore) const;

  // device-mirror bookkeeping of every view of the store (this one and its
  // replicas): what a mutation must re-upload, and the memos it invalidates
  void markStruct();
  void markRow(uint32_t v);
  void markLink(uint32_t id);
  void markNode(uint32_t v);
  void newStamps();
  void mutating() const;  // throws on a replica

  std::string area_;
  uint64_t stamp_;
  static uint64_t nextStamp();
  orh_ctx* ctx_;
  mutable orh_graph* graph_{nullptr};
  bool replica_{false};

  // the host graph store (shared with the replicas) under its old names
  std::shared_ptr<LinkStateStore> store_;
  std::unordered_map<std::string, uint32_t>& ids_;
  std::vector<std::string>& names_;
  std::vector<Link>& links_;
  std::vector<uint32_t>& freeLinks_;
  size_t& nLinks_;
  std::vector<std::unique_ptr<LinkSet>>& nodeLinks_;
  std::unordered_map<std::string, Holdable<bool>>& nodeOverloads_;
  std::unordered_map<std::string, AdjacencyDatabase>& adjacencyDatabases_;

  // device mirror bookkeeping
  mutable bool structDirty_{true};                 // node set changed: full orh_graph_load
  mutable std::unordered_set<uint32_t> rowsDirty_;  // link sets changed: orh_graph_apply_delta
  mutable uint64_t mirrorLoads_{0}, mirrorDeltas_{0};
  mutable std::unordered_set<uint32_t> patchLinks_;
  mutable std::unordered_set<uint32_t> patchNodes_;
  mutable std::vector<uint32_t> rowPtr_;  // host copy of the uploaded CSR
  mutable std::vector<uint32_t> col_, linkOfEntry_;
  mutable std::vector<std::pair<uint32_t, uint32_t>> entriesOfLink_;

  // memo (LinkState.h:279-301)
  mutable std::map<std::pair<std::string, bool>, SpfRow> spfResults_;
  mutable std::map<std::pair<std::string, bool>, SpfResult> spfMaps_;  // getSpfResult views
  // (src, dst, k) memos: looked up, never iterated (LinkState.h:298-301)
  mutable KthMemo<std::vector<Path>> kthPaths_;
  mutable KthMemo<std::vector<LinkPath>> kthLinkPaths_;
  mutable uint64_t spfRuns_{0};
  // sources whose SPF a device KSP2 batch ran and counted (the reference's
  // memoized getSpfResult, LinkState.cpp:775-776) without keeping the row on
  // the host: a later getSpfRow of one computes the row but does not count it
  mutable std::unordered_set<std::string> countedOnDevice_;

 public:
  // prefetchKthPaths pairs traced on the device / on the host (tests, A/B)
  mutable uint64_t kspDevicePairs_{0}, kspHostPairs_{0};
};

}  // namespace openr_amd
