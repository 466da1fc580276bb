// Multi-GPU forms of the SPF path inside the drop-in library,
// without torch or a launcher: one topology mirrored on several devices, the
// all-sources SPF split over them in contiguous source blocks of equal work,
// each block swept on its own device stream. Every source is independent
// given the read-only topology, so there is no collective on the data path;
// rows stay on the device that computed them until a consumer fetches or
// gathers them (a central RIB).
#pragma once

#include <memory>
#include <utility>
#include <vector>

#include "link_state.h"
#include "spf_solver.h"
#include "whatif_batch.h"

namespace openr_amd {

// The libopenr_hip context of (device, slot): one orh_ctx - own HIP stream and
// scratch - per pair, created on first use. Slot 0 of the process's default
// device is defaultContext(); further slots on one device are extra streams
// (or, on a one-GPU box, a rehearsal of several devices).
orh_ctx* deviceContext(int device, unsigned slot = 0);

// One area's LinkState on several devices: replica 0 (the primary) owns the
// host graph store, replicas 1.. are device views of it (LinkState's replica
// constructor): a mutation is applied to the store once and marks every
// replica's device mirror with the same delta, and the replicas answer alike.
// devices may repeat a device id (a second context on that device).
class ReplicatedLinkState {
 public:
  ReplicatedLinkState(const std::string& area, const std::vector<int>& devices);
  ~ReplicatedLinkState();
  LinkStateChange updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl = 0,
                                          Metric holdDownTtl = 0);
  LinkStateChange deleteAdjacencyDatabase(const std::string& node);
  LinkStateChange decrementHolds();
  size_t replicas() const { return reps_.size(); }
  const LinkState& replica(size_t i) const { return *reps_.at(i); }
  const LinkState& primary() const { return *reps_[0]; }

 private:
  std::vector<std::unique_ptr<LinkState>> reps_;
};

// All-sources SPF (LinkState::runSpf from every listed source, dist + first-hop
// rows) sharded over a ReplicatedLinkState's devices. Sources keep their
// order; replica r sweeps the contiguous block r, cut so the blocks carry equal
// work (1 + links / 16 per source: a source's first hops read one row per
// neighbour, so Clos spines weigh more), the same cut as openr_amd.sharding.
// degree_weighted_sources. Every block uses the whole list's mask width, so
// rows of all blocks have one shape.
class MultiDeviceSweep {
 public:
  MultiDeviceSweep(const ReplicatedLinkState& rls, const std::vector<std::string>& srcs,
                   bool useLinkMetric = true);
  ~MultiDeviceSweep();
  MultiDeviceSweep(const MultiDeviceSweep&) = delete;
  MultiDeviceSweep& operator=(const MultiDeviceSweep&) = delete;

  // every block, asynchronously on its device's stream. Each run sweeps the
  // replicas' graphs as they are now (pending deltas flushed); a topology
  // whose node count or mask width outgrew the sweep's buffers throws
  // std::runtime_error (make a new sweep)
  void run();
  void runBlock(size_t r);  // block r alone (per-device timing, rehearsals on one GPU)
  void sync();  // waits for every device
  size_t sources() const { return total_; }
  uint32_t nodes() const { return n_; }
  uint32_t words() const { return words_; }
  size_t blocks() const { return blocks_.size(); }
  std::pair<size_t, size_t> block(size_t r) const { return {blocks_.at(r).lo, blocks_.at(r).hi}; }
  // device time of block r's last sweep (HIP events on its stream; waits for it)
  double lastMs(size_t r) const;
  // source i's rows into host memory: dist[N], nh[N * words()]
  void fetch(size_t i, uint32_t* dist, uint32_t* nh) const;
  // every row in source order into host arrays dist[S][N], nh[S][N * words()]
  void gather(uint32_t* dist, uint32_t* nh) const;

 private:
  struct Block {
    const LinkState* ls{nullptr};
    orh_graph* g{nullptr};
    orh_ctx* ctx{nullptr};
    size_t lo{0}, hi{0};
    std::vector<uint32_t> srcs;  // node ids on this replica
    uint32_t* dDist{nullptr};
    uint32_t* dNh{nullptr};
  };
  const Block& blockOf(size_t i) const;
  std::vector<Block> blocks_;
  bool useLinkMetric_;
  uint32_t n_{0}, words_{1};
  size_t total_{0};
};

// Contiguous blocks of `items` weighted by w(i), one per device: cut points
// of the prefix sums at k/world of the total (block r = [cuts[r], cuts[r+1]))
std::vector<size_t> equalWorkCuts(const std::vector<double>& w, size_t world);

// A what-if job (WhatIfBatch: requests (source, ignored links)) split over a
// ReplicatedLinkState's devices by source: the sources are cut into
// contiguous blocks of equal request counts, and device r's job holds the
// base rows of block r's sources and runs exactly their requests (SURVEY.md
// §8e: "what-if batches shard naturally"). Every request is independent given
// the topology, so there is no collective; per-request results (tier /
// affected count, row digests) come back in the caller's request order.
class MultiDeviceWhatIf {
 public:
  // blocks per job from which each block searches its largest repairs in full
  static constexpr size_t kSearchLargeBlocks = 4;
  MultiDeviceWhatIf(const ReplicatedLinkState& rls, const std::vector<std::string>& srcs,
                    const std::vector<uint32_t>& srcIdx, const std::vector<std::vector<uint32_t>>& ignore,
                    uint32_t chunk, bool useLinkMetric = true, bool shareBase = false);
  MultiDeviceWhatIf(const MultiDeviceWhatIf&) = delete;
  MultiDeviceWhatIf& operator=(const MultiDeviceWhatIf&) = delete;
  // every block at once: one host thread per device drives its job
  void run();
  void runBlock(size_t r);
  void sync();
  // free block r's row buffers and job (rehearsals on one GPU: a block's
  // buffers only while it runs); its next run allocates them again
  void release(size_t r);
  void setDigests(bool on);
  size_t blocks() const { return blocks_.size(); }
  std::pair<size_t, size_t> sourceBlock(size_t r) const { return {blocks_.at(r).lo, blocks_.at(r).hi}; }
  size_t blockRequests(size_t r) const { return blocks_.at(r).reqs.size(); }
  size_t requests() const { return total_; }
  // device ms of block r's last run; 0 for a block with no requests (no job)
  // or one released since
  double lastMs(size_t r) const {
    const Block& b = blocks_.at(r);
    return b.job ? b.job->lastMs() : 0.0;
  }
  void info(uint32_t* out) const;     // [requests()] in the caller's order
  void digests(uint64_t* out) const;  // [requests()] (setDigests(true) before the run)

 private:
  struct Block {
    size_t lo{0}, hi{0};        // sources [lo, hi)
    std::vector<size_t> reqs;   // the caller's request indices, in order
    std::unique_ptr<WhatIfBatch> job;
  };
  std::vector<Block> blocks_;
  size_t total_{0};
};

// getKthPaths (LinkState.cpp:762-791) for a batch of (src, dst) pairs split
// over a ReplicatedLinkState's devices by source: pairs of one source stay on
// one device (its k = 1 row is searched once), sources are cut into
// contiguous blocks of equal pair counts (first-appearance order). Each
// block is one orh_ksp2_batch on its device; pairs the device trace flags,
// and graphs that need the exact kernel, take the replica's getKthPaths.
// Paths are LinkState link ids (the same on every replica: each applied the
// same updates in the same order).
class MultiDeviceKthPaths {
 public:
  MultiDeviceKthPaths(const ReplicatedLinkState& rls,
                      const std::vector<std::pair<std::string, std::string>>& pairs);
  MultiDeviceKthPaths(const MultiDeviceKthPaths&) = delete;
  MultiDeviceKthPaths& operator=(const MultiDeviceKthPaths&) = delete;
  void run();  // every block at once, one host thread per device
  void runBlock(size_t r);
  double lastMs(size_t r) const { return blocks_.at(r).ms; }  // wall time of block r's last run
  size_t blocks() const { return blocks_.size(); }
  size_t blockPairs(size_t r) const { return blocks_.at(r).pairs.size(); }
  size_t pairs() const { return pairs_.size(); }
  // the k-th paths (k = 1, 2) of pair i from the last run
  const std::vector<Path>& paths(size_t i, size_t k) const;
  // pairs of the last run traced on the device / by the host fallback
  size_t devicePairs() const;

 private:
  struct Block {
    const LinkState* ls{nullptr};
    std::vector<size_t> pairs;  // the caller's pair indices
    double ms{0};
    size_t onDevice{0};
  };
  std::vector<std::pair<std::string, std::string>> pairs_;
  std::vector<Block> blocks_;
  std::vector<std::vector<Path>> k1_, k2_;
};

// Every area's LinkState mirrored on several devices: one AreaLinkStates per
// device (each area's LinkState on that device's context), every mutation
// applied to all of them; replica 0 answers like the reference's
// AreaLinkStates.
class ReplicatedAreaLinkStates {
 public:
  explicit ReplicatedAreaLinkStates(const std::vector<int>& devices);
  ~ReplicatedAreaLinkStates();
  void addArea(const std::string& area);
  // the area is db.area (added on first use)
  LinkStateChange updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl = 0,
                                          Metric holdDownTtl = 0);
  LinkStateChange deleteAdjacencyDatabase(const std::string& area, const std::string& node);
  size_t replicas() const { return reps_.size(); }
  const AreaLinkStates& replica(size_t r) const { return *reps_.at(r); }
  orh_ctx* context(size_t r) const { return ctxs_.at(r); }

 private:
  std::vector<orh_ctx*> ctxs_;
  std::vector<std::unique_ptr<AreaLinkStates>> reps_;
};

// SpfSolver::buildRouteDb (Decision.cpp:615-792) with the prefixes sharded
// over devices ("100k-prefix route selection sharded over
// 8 GPUs"): shard r is a SpfSolver owning the prefix-id block r
// (setPrefixShard) on replica r's areas; its SPF, route selection and policy
// run on device r, and its routes are materialised by its own host thread;
// shard 0 also builds the MPLS routes. The shards' unicast maps are spliced
// into one DecisionRouteDb, which equals the unsharded build.
class ShardedRouteBuilder {
 public:
  ShardedRouteBuilder(const ReplicatedAreaLinkStates& areas, const std::string& myNodeName, bool enableV4,
                      bool enableOrderedFib = false, bool bgpDryRun = false,
                      bool enableBestRouteSelection = false);
  ShardedRouteBuilder(const ShardedRouteBuilder&) = delete;
  ShardedRouteBuilder& operator=(const ShardedRouteBuilder&) = delete;
  std::optional<DecisionRouteDb> buildRouteDb(const std::string& me, const PrefixState& ps);
  // shard r alone (its own DecisionRouteDb part; per-device timing)
  std::optional<DecisionRouteDb> buildShard(size_t r, const std::string& me, const PrefixState& ps);
  void updateStaticUnicastRoutes(const std::vector<std::pair<Cidr, std::vector<NextHopThrift>>>& upd,
                                 const std::vector<Cidr>& del);
  void updateStaticMplsRoutes(const std::vector<std::pair<int32_t, std::vector<NextHopThrift>>>& upd,
                              const std::vector<int32_t>& del);
  size_t shards() const { return solvers_.size(); }
  SpfSolver& shard(size_t r) { return *solvers_.at(r); }
  // wall times of the last buildRouteDb: each shard's build (its thread), the merge
  double lastShardMs(size_t r) const { return shardMs_.at(r); }
  double lastMergeMs() const { return mergeMs_; }
  // drops ps's device mirrors on the shards' contexts (all but the default
  // context's); returns how many were freed
  size_t releasePrefixMirrors(PrefixState& ps) const;

 private:
  const ReplicatedAreaLinkStates& areas_;
  std::vector<std::unique_ptr<SpfSolver>> solvers_;
  std::vector<double> shardMs_;
  double mergeMs_{0};
};

}  // namespace openr_amd
