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

namespace openr_amd {

// The libopenr_hip context of (device, slot): one orh_ctx - own HIP stream and
// scratch - per pair, created on first use. Slot 0 of the process's default
// device is defaultContext(); further slots on one device are extra streams
// (or, on a one-GPU box, a rehearsal of several devices).
orh_ctx* deviceContext(int device, unsigned slot = 0);

// One area's LinkState on several devices: every mutation goes to every
// replica (each mirrors the same graph into its device), and the replicas
// answer alike; replica 0 is the primary. devices may repeat a device id
// (a second context on that device).
class ReplicatedLinkState {
 public:
  ReplicatedLinkState(const std::string& area, const std::vector<int>& devices);
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

  void run();   // every block, asynchronously on its device's stream
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

}  // namespace openr_amd
