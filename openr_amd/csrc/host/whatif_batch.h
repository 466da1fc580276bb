// Batched link-failure what-if SPFs ("4,096 links x 64
// sources" of runSpf(src, true, {link}), LinkState.cpp:808-882) through one
// what-if job of libopenr_hip (orh_whatif_*): the sources' plain rows are
// searched once, then the requests run in chunks into device row buffers; a
// request's row is its source's row except below a tight ignored link, where
// the job re-derives it (bit-identical to a fresh runSpf).
//
// This is the library form a caller outside Python drives (the bench, the
// multi-device split in multi_device.h); the Python binding wraps it.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "link_state.h"

namespace openr_amd {

class WhatIfBatch {
 public:
  // request i = (srcs[srcIdx[i]], ignore[i]) with ignore sets of LinkState link
  // ids; chunk = requests per orh_whatif_run. shareBase: ORH_WHATIF_SHARE_BASE
  // (a request whose source row stands references the job's base row);
  // searchLarge: ORH_WHATIF_SEARCH_LARGE (the largest repairs searched in
  // full: for a device's block of a split job)
  WhatIfBatch(const LinkState& ls, const std::vector<std::string>& srcs, const std::vector<uint32_t>& srcIdx,
              const std::vector<std::vector<uint32_t>>& ignore, uint32_t chunk, bool useLinkMetric = true,
              bool shareBase = false, bool searchLarge = false);
  ~WhatIfBatch();
  WhatIfBatch(const WhatIfBatch&) = delete;
  WhatIfBatch& operator=(const WhatIfBatch&) = delete;

  // the sources' plain searches (the first run; later runs refresh them on
  // the graph as it is now), then every chunk; asynchronous on the context
  // stream
  void run();
  void sync() const;
  // device time of the last run (base searches to the last chunk, HIP events)
  double lastMs() const;
  // per request (caller's order): ORH_WHATIF_TIER | ORH_WHATIF_AFFECTED << 3
  void info(uint32_t* out) const;
  // verification mode: every chunk's rows are digested (orh_row_digest) before
  // their buffer is reused, and a shared-base request gets its source row's
  // digest; each chunk is flushed first, so runs in this mode are slower
  void setDigests(bool on);
  void digests(uint64_t* out) const;
  // rows of request i; only the last chunk's rows are still in the buffers
  // (std::out_of_range otherwise)
  void fetch(size_t i, uint32_t* dist, uint32_t* nh) const;
  // free the row buffers and the job (the next run allocates them again)
  void release();

  size_t requests() const { return srcIdx_.size(); }
  size_t sources() const { return srcs_.size(); }
  uint32_t chunk() const { return chunk_; }
  uint32_t nodes() const { return n_; }
  uint32_t edges() const { return edges_; }
  orh_ctx* context() const { return ctx_; }

 private:
  struct Chunk {
    size_t lo, hi;
    std::vector<uint32_t> ptr, links;
  };
  void allocate();
  const LinkState& ls_;
  bool useLinkMetric_;
  bool shareBase_;
  bool searchLarge_;
  bool digests_{false};
  std::vector<uint32_t> srcs_, srcIdx_;
  std::vector<Chunk> chunks_;
  uint32_t chunk_{1};
  orh_graph* graph_{nullptr};
  orh_ctx* ctx_{nullptr};
  orh_whatif* job_{nullptr};
  uint64_t stamp_{0};  // LinkState::stateStamp the job was created at
  uint32_t n_{0}, edges_{0};
  // up to three row buffers, cycled between chunks, so a chunk's repairs
  // (which write into its rows) overlap the next two chunks' copies
  static constexpr size_t kBufs = 3;
  int nBuf_{0};
  uint32_t* dDist_[kBufs] = {};
  uint32_t* dNh_[kBufs] = {};
  uint32_t* dInfo_{nullptr};
  uint64_t* dDigest_{nullptr};      // [requests] (verification mode)
  uint64_t* dBaseDigest_{nullptr};  // [sources]
};

}  // namespace openr_amd
