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

#include <atomic>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>

#include "link_state.h"
#include "rib_policy.h"

namespace openr_amd {

using PrefixEntries = std::unordered_map<NodeAndArea, PrefixEntryRef, StrPairHash>;

// one advertisement as the device mirror numbers it (order within a prefix)
struct AdvRef {
  const NodeAndArea* key;
  const PrefixEntryRef* entry;  // shared with the routes built from it
};

// PrefixState (openr/decision/PrefixState.h:22-70) plus a device mirror of
// it for SpfSolver's device route selection: every prefix gets a dense id,
// advertiser names and areas get ids, and updatePrefix / deletePrefix record
// the prefix as dirty; the next route build uploads only the dirty prefixes'
// advertisement lists (orh_prefix_apply_delta), the first one everything
// (orh_prefix_load).
class PrefixState {
 public:
  PrefixState() = default;
  PrefixState(const PrefixState&) = delete;
  PrefixState& operator=(const PrefixState&) = delete;
  ~PrefixState();

  std::vector<Cidr> updatePrefix(const std::string& node, const std::string& area,
                                 const PrefixEntry& e);
  // the same, taking the entry (no copy of it)
  std::vector<Cidr> updatePrefix(const std::string& node, const std::string& area, PrefixEntry&& e);
  // updatePrefix without the changed-prefix list: whether the prefix changed
  bool upsertPrefix(const std::string& node, const std::string& area, PrefixEntry&& e);
  // capacity for n more prefixes (a bulk load: no rehash of the maps)
  void reserve(size_t n);
  std::vector<Cidr> deletePrefix(const std::string& node, const std::string& area,
                                 const Cidr& prefix);
  const std::unordered_map<Cidr, PrefixEntries, CidrHash>& prefixes() const { return prefixes_; }
  // advertisements with forwardingAlgorithm KSP2_ED_ECMP (lets buildRouteDb
  // skip its KSP2 planning pass when there are none)
  size_t ksp2Entries() const { return ksp2Entries_; }

  // ---- device mirror (used by SpfSolver) ----
  // brings the mirror on `ctx` up to date (one mirror per context: a route
  // build sharded over devices keeps one per device); returns it
  // The PrefixState must not be mutated while a build reads it (the Python
  // bindings release the GIL during builds: the caller serialises updates).
  orh_prefix_set* syncDevice(orh_ctx* ctx) const;
  // frees the mirror on `ctx` (e.g. once a sharded build's extra device
  // contexts are gone); false when there is none. A later build there
  // uploads a fresh one
  bool dropDeviceMirror(orh_ctx* ctx);
  size_t deviceMirrors() const { return mirrors_.size(); }
  uint32_t numPrefixIds() const { return static_cast<uint32_t>(cidrOf_.size()); }
  const Cidr& prefixOf(uint32_t pid) const { return cidrOf_[pid]; }
  bool prefixLive(uint32_t pid) const { return live_[pid] != 0; }
  // the advertisements of pid in the order the device numbers them
  const AdvRef* advs(uint32_t pid, uint32_t* n) const {
    *n = run_[pid].second;
    return advPool_.data() + run_[pid].first;
  }
  std::optional<uint32_t> pidOf(const Cidr& prefix) const {
    auto it = pid_.find(prefix);
    if (it == pid_.end()) return std::nullopt;
    return it->second;
  }
  // change stamps (an incremental rebuild's "what changed since"): every
  // updatePrefix / deletePrefix that changes a prefix advances stamp(); a
  // prefix id carries the stamp of its last change, and withdrawn prefixes
  // are logged with theirs (ids are reused)
  uint64_t stamp() const { return stamp_; }
  uint64_t pidStamp(uint32_t pid) const { return pidStamp_[pid]; }
  // process-unique instance id (stamps are process-unique too)
  uint64_t id() const { return id_; }
  // calls f(prefix) for each prefix withdrawn after `since`; false when the
  // log no longer reaches back that far
  template <class F>
  bool forEachDeletedSince(uint64_t since, F&& f) const {
    if (since < deletedFloor_) return false;
    for (auto it = deleted_.rbegin(); it != deleted_.rend() && it->first > since; ++it) f(it->second);
    return true;
  }
  std::optional<uint32_t> nameId(const std::string& n) const;
  uint32_t numNames() const { return static_cast<uint32_t>(names_.size()); }
  const std::string& name(uint32_t id) const { return names_[id]; }
  std::optional<uint32_t> areaId(const std::string& a) const;
  uint32_t numAreas() const { return static_cast<uint32_t>(areas_.size()); }
  const std::string& area(uint32_t id) const { return areas_[id]; }
  // tag sets of the advertisements (ids 1 .. numTagSets(); 0 = no tags;
  // ids saturate at ORH_ADV_TAGSET_OVF)
  uint32_t tagSetId(const std::set<std::string>& tags) const;
  uint32_t numTagSets() const { return static_cast<uint32_t>(tagSets_.size()); }
  const std::set<std::string>& tagSet(uint32_t id) const { return *tagSets_[id - 1]; }
  // tag sets from the limit-th on share ORH_ADV_TAGSET_OVF (their routes take
  // RibPolicy on the host: ORH_POL_HOST); tests lower the limit to reach that
  // path, before the first tagged advertisement
  uint32_t tagSetIdLimit() const { return tagIdLimit_; }
  void setTagSetIdLimit(uint32_t limit);

 private:
  void touch(const Cidr& prefix, bool erased);
  uint32_t internName(const std::string& n);
  uint32_t internArea(const std::string& a);
  uint32_t internTagSet(const std::set<std::string>& tags);
  orh_adv advRecord(const NodeAndArea& na, const PrefixEntry& e) const;

  std::unordered_map<Cidr, PrefixEntries, CidrHash> prefixes_;
  size_t ksp2Entries_{0};

  std::unordered_map<Cidr, uint32_t, CidrHash> pid_;
  std::vector<Cidr> cidrOf_;
  std::vector<uint8_t> live_;
  std::vector<uint32_t> freePids_;
  std::vector<uint32_t> dirty_;
  uint64_t id_{nextGeneration()};
  uint64_t stamp_{nextGeneration()};
  std::vector<uint64_t> pidStamp_;
  static constexpr size_t kDeletedLog = 1u << 20;
  std::deque<std::pair<uint64_t, Cidr>> deleted_;
  uint64_t deletedFloor_{0};
  std::vector<uint8_t> isDirty_;
  std::unordered_map<std::string, uint32_t> nameIds_, areaIds_;
  std::vector<std::string> names_, areas_;
  std::map<std::set<std::string>, uint32_t> tagSetIds_;
  std::vector<const std::set<std::string>*> tagSets_;  // id - 1 -> set (map nodes are stable)
  uint32_t tagIdLimit_{ORH_ADV_TAGSET_OVF};

  mutable std::vector<AdvRef> advPool_;
  mutable std::vector<std::pair<uint32_t, uint32_t>> run_;  // pid -> (offset, count)
  mutable size_t advLive_{0};
  mutable bool hostFull_{true};  // every run rebuilt at the next sync (pool renumbered)
  // one device mirror per context (a route build sharded over devices keeps
  // one per device); each tracks the prefixes changed since its own last sync
  struct Mirror {
    orh_ctx* ctx{nullptr};
    orh_prefix_set* dev{nullptr};
    bool full{true};
    uint32_t namesOrdered{0}, areasOrdered{0};
    std::vector<uint32_t> dirty;
    std::vector<uint8_t> isDirty;
  };
  mutable std::vector<std::unique_ptr<Mirror>> mirrors_;
  mutable std::mutex syncMu_;
  // device records of pids `ids` (all pids when ids is null) from the host runs
  void buildRecords(const std::vector<uint32_t>* ids, std::vector<uint32_t>& ptr, std::vector<orh_adv>& recs,
                    std::vector<uint8_t>& fl) const;
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

// Collects the phase times (name, ms) of the route builds this thread runs
// while it is alive (the phases ORH_ROUTE_PROF prints; " select: ..." entries
// subdivide "select (device)"). For measurement: bench.py reports them.
class RoutePhaseCapture {
 public:
  RoutePhaseCapture();
  ~RoutePhaseCapture();
  RoutePhaseCapture(const RoutePhaseCapture&) = delete;
  RoutePhaseCapture& operator=(const RoutePhaseCapture&) = delete;
  std::vector<std::pair<const char*, double>> phases;

 private:
  std::vector<std::pair<const char*, double>>* prev_;
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
  // buildRouteDb, then policy->applyPolicy(db.unicastRoutes): the full
  // rebuild of Decision::rebuildRoutes (Decision.cpp:1888-1900). The same
  // database, with the policy decided per route on the device for the routes
  // the device selected (orh_route_policy) and its weights set while they are
  // materialised; host-path and static routes take RibPolicy::applyAction.
  // Without an active policy this is buildRouteDb.
  struct PolicyStats {
    uint64_t updated{0};      // routes the policy transformed (PolicyChange.updatedRoutes)
    uint64_t invalidated{0};  // statements that would have dropped every nexthop
    uint64_t onDevice{0};     // routes whose statement the device decided
    double deviceMs{0};       // policy tables + kernel + copy-out (host wall time)
  };
  std::optional<DecisionRouteDb> buildRouteDbWithPolicy(const std::string& me, const AreaLinkStates& als,
                                                        const PrefixState& ps, RibPolicy* policy,
                                                        PolicyStats* stats = nullptr);
  std::optional<RibUnicastEntry> createRouteForPrefixOrGetStaticRoute(
      const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
      const Cidr& prefix);

  // createRouteForPrefixOrGetStaticRoute for many prefixes at once (the
  // incremental branch of Decision::rebuildRoutes, Decision.cpp:1902-1911):
  // one device selection pass over the prefix mirror, then the listed
  // prefixes materialised on the host pool; the same results as one call per
  // prefix
  std::vector<std::optional<RibUnicastEntry>> createRoutesForPrefixes(
      const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
      const std::vector<Cidr>& prefixes);

  // Decision::rebuildRoutes' full rebuild (Decision.cpp:1888-1900:
  // buildRouteDb, RibPolicy, calculateUpdate) as a delta against `current`,
  // the route DB built from this solver's selection snapshot `selGen` with
  // the prefix state at `psStamp` and the same policy: the device selection
  // runs for every prefix and is compared on the device with the snapshot
  // (orh_route_diff); only prefixes whose selection record changed, prefixes
  // changed since psStamp, and host-path prefixes get a route built, the
  // policy applied and compared with current's entry. MPLS routes are rebuilt
  // and compared in full. nullopt when a delta cannot stand for the full
  // rebuild (no snapshot, KSP2, prefix shards, my nexthop templates changed,
  // ...): the caller rebuilds in full. The update equals calculateUpdate's.
  std::optional<DecisionRouteUpdate> buildRouteDelta(const std::string& me, const AreaLinkStates& als,
                                                     const PrefixState& ps, const DecisionRouteDb& current,
                                                     uint64_t selGen, uint64_t psStamp, RibPolicy* policy);
  // the selection snapshot of the last device selection (0: none), and the
  // static routes' version
  uint64_t selGen() const { return havePrev_ ? selGen_ : 0; }
  uint64_t staticEpoch() const { return staticEpoch_; }
  uint64_t routeBuildRuns() const { return routeBuildRuns_; }
  // prefixes of the last buildRouteDb whose selection ran on the device /
  // took the host path (BGP, SR_MPLS, KSP2, minNexthop, self-advertised)
  uint64_t deviceSelected() const { return deviceSelected_; }
  // prefix sharding over `world` route builders: this
  // solver builds the unicast routes of the prefix ids in its contiguous
  // block (and the static routes of prefixes it owns); node-label, adj-label
  // and static MPLS routes are built by shard 0. The union of the shards'
  // databases is the unsharded database.
  void setPrefixShard(uint32_t rank, uint32_t world);
  uint64_t hostSelected() const { return hostSelected_; }
  // device time of the last build's selection kernel and its algorithmic
  // bytes (B_sel: headers 8 B + records 20 B per advertisement + per
  // advertisement and area a 4 B distance gather + outputs 9 + 4 W bytes)
  double lastSelectMs() const { return lastSelectMs_; }
  uint64_t lastSelectBytes() const { return lastSelectBytes_; }
  ~SpfSolver();

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

  // device route selection over the PrefixState mirror; false when the
  // inputs need the host path for every prefix
  // diff = true: compare with the previous snapshot on the device and copy
  // back only the changed records (changedPids_; lastDiffed_ says whether
  // the compare could run)
  bool selectOnDevice(const std::string& me, const AreaLinkStates& als, const PrefixState& ps,
                      bool diff = false);
  std::optional<DecisionRouteDb> buildRouteDbImpl(const std::string& me, const AreaLinkStates& als,
                                                  const PrefixState& ps, bool mplsOnly,
                                                  RibPolicy* policy = nullptr);
  // the route of a device-selected prefix; with the device policy on, its
  // statement's weights applied (or RibPolicy::applyAction for ORH_POL_HOST)
  RibUnicastEntry materialize(uint32_t pid, const PrefixState& ps) const;
  // RibPolicy decided on the device for the last selection (devPol_); false
  // when the policy does not fit the device form (> 32 statements, no
  // selection on the device)
  bool policyOnDevice(const PrefixState& ps, RibPolicy& policy);
  struct DevicePolicy {
    bool on{false};
    RibPolicy* policy{nullptr};
    std::vector<uint8_t> stmt;  // per prefix id: statement, ORH_POL_NONE / _HOST
    // weight[s][area][first-hop bit] of statement s
    std::vector<std::vector<std::vector<int32_t>>> weight;
    uint64_t deviceInvalidated{0};
    mutable std::atomic<uint64_t> hostInvalidated{0}, hostUpdated{0};
    uint64_t onDevice{0};
    double ms{0};
    void reset() {
      on = false;
      policy = nullptr;
      stmt.clear();
      weight.clear();
      deviceInvalidated = onDevice = 0;
      hostInvalidated = 0;
      hostUpdated = 0;
      ms = 0;
    }
  } devPol_;
  uint8_t* dPolOut_{nullptr};
  size_t dPolOutCap_{0};
  PolicyStats* policyStats_{nullptr};  // set while buildRouteDbWithPolicy runs

  // device selection workspace (per solver)
  struct AreaWork {
    const LinkState* ls{nullptr};
    uint32_t lsNodes{0}, psNames{0};      // name_node built for these sizes
    std::vector<uint32_t> nameNode;       // ps name id -> node id in ls
    uint32_t* dNameNode{nullptr};
    size_t dNameNodeCap{0};
    uint32_t* dRow{nullptr};              // me's dist row | first-hop rows
    size_t dRowCap{0};
    uint32_t words{0}, wordOff{0};
    // per first-hop bit: tight up links of me to that neighbour as nexthop
    // templates (metric set per route), v6 and v4 addresses
    std::vector<std::vector<NextHopThrift>> tmpl6, tmpl4;
    // the templates in my LinkSet iteration order as (bit, index in
    // tmpl[bit]): getNextHopsThrift's insertion order (Decision.cpp:1245-1246)
    std::vector<std::pair<uint32_t, uint32_t>> linkOrder;
  };
  std::vector<AreaWork> areaWork_;
  // areaWork_ indices in AreaLinkStates iteration order (the reference's
  // outer loop over areaLinkStates, Decision.cpp:1245)
  std::vector<uint32_t> areaIter_;
  // inserts the nexthops of first-hop mask m (indexed by each area's
  // wordOff) in the reference's order with the given metric and weight 0,
  // the MPLS action act(template); with wt, each inserted element's weight
  // under wt[area][bit] is recorded in *wts (by element address)
  template <class Act>
  void insertTemplates(const uint32_t* m, bool v4, int32_t metric,
                       const std::vector<std::vector<int32_t>>* wt,
                       std::vector<std::pair<const NextHopThrift*, int32_t>>* wts, NextHopSet& out,
                       Act&& act) const;
  orh_ctx* selCtx_{nullptr};
  uint8_t* dSel_{nullptr};  // status | metric | best | mask
  size_t dSelCap_{0};
  // the previous selection (snapshot selGen_, prevN_ prefixes, layout digest
  // of the nexthop templates it was made with) and the diff output
  uint8_t* dSelPrev_{nullptr};
  size_t dSelPrevCap_{0};
  uint32_t* dDiff_{nullptr};
  size_t dDiffCap_{0};
  bool havePrev_{false}, lastDiffed_{false};
  uint64_t selGen_{0}, prevLayout_{0}, staticEpoch_{0};
  // the route build's flat slot array (two-pass fill, buildRouteDbImpl):
  // uninitialised storage kept across builds (no page faults per build; C5:
  // 1M slots of ~100 B) and per-(worker, output shard) lists of the slots
  // holding a constructed route (empty between builds)
  struct RouteSlots {
    struct Free {
      void operator()(void* p) const { ::operator delete(p); }
    };
    std::unique_ptr<void, Free> mem;
    size_t cap{0};
    std::vector<std::vector<uint32_t>> lists;
    void reserve(size_t n) {
      if (n <= cap) return;
      mem.reset(::operator new(n * sizeof(RibUnicastEntry)));
      cap = n;
    }
    RibUnicastEntry* at(size_t i) { return static_cast<RibUnicastEntry*>(mem.get()) + i; }
  };
  RouteSlots routeSlots_;
  // inputs of the last MPLS route build (every area's LinkState stamp, me,
  // static routes): a delta rebuild with the same inputs keeps the routes
  std::vector<std::pair<const LinkState*, uint64_t>> mplsInputs(const AreaLinkStates& als) const;
  std::vector<std::pair<const LinkState*, uint64_t>> mplsKey_;
  std::string mplsMe_;
  uint64_t mplsStatic_{0};
  bool mplsKeyOk_{false};
  uint32_t prevN_{0}, prevWords_{0};
  std::vector<uint32_t> changedPids_;
  std::vector<uint8_t> selStatus_;
  std::vector<uint32_t> selMetric_, selBest_, selMask_;
  uint32_t selWords_{0};
  uint64_t deviceSelected_{0}, hostSelected_{0};
  uint32_t shardRank_{0}, shardWorld_{1};
  double lastSelectMs_{0};
  uint64_t lastSelectBytes_{0};
  // this solver's contiguous block of the prefix ids [0, n)
  std::pair<uint32_t, uint32_t> shardRange(uint32_t n) const {
    if (shardWorld_ <= 1) return {0u, n};
    const uint64_t base = n / shardWorld_, rem = n % shardWorld_;
    const uint64_t lo = shardRank_ * base + std::min<uint64_t>(shardRank_, rem);
    const uint64_t hi = lo + base + (shardRank_ < rem ? 1 : 0);
    return {static_cast<uint32_t>(lo), static_cast<uint32_t>(hi)};
  }
  bool ownsPid(uint32_t pid, uint32_t n) const {
    const auto [lo, hi] = shardRange(n);
    return pid >= lo && pid < hi;
  }

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
