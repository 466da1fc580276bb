// WhatIfBatch: see whatif_batch.h.
#include "whatif_batch.h"

#include <algorithm>
#include <stdexcept>

namespace openr_amd {

namespace {

void check(orh_ctx* ctx, int rc, const char* what) {
  if (rc != ORH_OK)
    throw std::runtime_error(std::string("WhatIfBatch: ") + what + " failed (" + std::to_string(rc) +
                             "): " + (ctx ? orh_last_error(ctx) : ""));
}

}  // namespace

WhatIfBatch::WhatIfBatch(const LinkState& ls, const std::vector<std::string>& srcs,
                         const std::vector<uint32_t>& srcIdx, const std::vector<std::vector<uint32_t>>& ignore,
                         uint32_t chunk, bool useLinkMetric, bool shareBase, bool searchLarge)
    : ls_(ls), useLinkMetric_(useLinkMetric), shareBase_(shareBase), searchLarge_(searchLarge) {
  if (srcIdx.size() != ignore.size()) throw std::invalid_argument("WhatIfBatch: one ignore set per request");
  if (chunk == 0) throw std::invalid_argument("WhatIfBatch: chunk must be positive");
  for (const auto& s : srcs) {
    auto id = ls.nodeId(s);
    if (!id) throw std::invalid_argument("WhatIfBatch: unknown source " + s);
    srcs_.push_back(*id);
  }
  for (uint32_t i : srcIdx)
    if (i >= srcs_.size()) throw std::invalid_argument("WhatIfBatch: source index out of range");
  srcIdx_ = srcIdx;
  // per chunk: the ignore CSR rebased to the chunk
  const size_t n = srcIdx.size();
  chunk_ = static_cast<uint32_t>(std::min<size_t>(chunk, std::max<size_t>(n, 1)));
  for (size_t c0 = 0; c0 < n; c0 += chunk_) {
    const size_t c1 = std::min(n, c0 + chunk_);
    std::vector<uint32_t> ptr{0}, links;
    for (size_t i = c0; i < c1; ++i) {
      links.insert(links.end(), ignore[i].begin(), ignore[i].end());
      ptr.push_back(static_cast<uint32_t>(links.size()));
    }
    if (links.empty()) links.push_back(0);  // non-null pointer
    chunks_.push_back({c0, c1, std::move(ptr), std::move(links)});
  }
  graph_ = ls.deviceGraph();
  ctx_ = ls.context();
  check(ctx_, orh_graph_info(graph_, &n_, &edges_), "orh_graph_info");
  check(ctx_, orh_device_alloc(ctx_, std::max<size_t>(n, 1) * 4, reinterpret_cast<void**>(&dInfo_)),
        "orh_device_alloc");
  allocate();
}

void WhatIfBatch::allocate() {
  if (nBuf_) return;
  const size_t rows = static_cast<size_t>(chunk_) * n_;
  const int want = static_cast<int>(std::max<size_t>(1, std::min<size_t>(chunks_.size(), kBufs)));
  for (int b = 0; b < want; ++b) {
    if (orh_device_alloc(ctx_, rows * 4, reinterpret_cast<void**>(&dDist_[b])) != ORH_OK ||
        orh_device_alloc(ctx_, rows * 4, reinterpret_cast<void**>(&dNh_[b])) != ORH_OK) {
      nBuf_ = b + 1;
      release();
      throw std::runtime_error("WhatIfBatch: device allocation failed (" + std::to_string(rows * 8) +
                               " bytes of rows per buffer)");
    }
    nBuf_ = b + 1;
  }
}

void WhatIfBatch::release() {
  if (job_) {
    orh_whatif_destroy(job_);
    job_ = nullptr;
  }
  for (int b = 0; b < nBuf_; ++b) {
    if (dDist_[b]) orh_device_free(ctx_, dDist_[b]);
    if (dNh_[b]) orh_device_free(ctx_, dNh_[b]);
    dDist_[b] = dNh_[b] = nullptr;
  }
  nBuf_ = 0;
}

WhatIfBatch::~WhatIfBatch() {
  release();
  if (dInfo_) orh_device_free(ctx_, dInfo_);
  if (dDigest_) orh_device_free(ctx_, dDigest_);
  if (dBaseDigest_) orh_device_free(ctx_, dBaseDigest_);
}

void WhatIfBatch::setDigests(bool on) {
  digests_ = on;
  if (!on || dDigest_) return;
  check(ctx_, orh_device_alloc(ctx_, std::max<size_t>(srcIdx_.size(), 1) * 8, reinterpret_cast<void**>(&dDigest_)),
        "orh_device_alloc");
  check(ctx_, orh_device_alloc(ctx_, std::max<size_t>(srcs_.size(), 1) * 8, reinterpret_cast<void**>(&dBaseDigest_)),
        "orh_device_alloc");
}

void WhatIfBatch::run() {
  // the graph as it is now: a what-if job is bound to its graph's structure
  // (orh_whatif_run fails with ORH_E_STATE after a delta or reload)
  {
    uint32_t n = 0, e = 0;
    check(ctx_, orh_graph_info(ls_.deviceGraph(), &n, &e), "orh_graph_info");  // flushes pending deltas
    if (n != n_)
      throw std::runtime_error("WhatIfBatch: the topology's node count changed (" + std::to_string(n_) + " -> " +
                               std::to_string(n) + "): rows are sized for the old one, make a new batch");
    edges_ = e;
  }
  allocate();
  if (job_ && ls_.stateStamp() != stamp_) {  // the LinkState changed: a job on the graph as it is now
    orh_whatif_destroy(job_);
    job_ = nullptr;
  }
  if (!job_) {
    stamp_ = ls_.stateStamp();
    check(ctx_, orh_whatif_create(graph_, srcs_.data(), static_cast<uint32_t>(srcs_.size()), useLinkMetric_ ? 1 : 0,
                                  &job_),
          "orh_whatif_create");
    const uint32_t fl = (shareBase_ ? ORH_WHATIF_SHARE_BASE : 0u) | (searchLarge_ ? ORH_WHATIF_SEARCH_LARGE : 0u);
    if (fl) check(ctx_, orh_whatif_set_flags(job_, fl), "orh_whatif_set_flags");
  } else {
    check(ctx_, orh_whatif_refresh(job_), "orh_whatif_refresh");
  }
  if (digests_) {
    const uint32_t *bd = nullptr, *bn = nullptr;
    check(ctx_, orh_whatif_base_rows(job_, &bd, &bn), "orh_whatif_base_rows");
    check(ctx_, orh_row_digest(ctx_, bd, bn, 1, n_, static_cast<uint32_t>(srcs_.size()), dBaseDigest_),
          "orh_row_digest");
  }
  for (size_t c = 0; c < chunks_.size(); ++c) {
    const Chunk& ch = chunks_[c];
    const uint32_t nr = static_cast<uint32_t>(ch.hi - ch.lo);
    const int b = static_cast<int>(c % nBuf_);  // cycle the row buffers
    check(ctx_,
          orh_whatif_run(job_, nr, srcIdx_.data() + ch.lo, ch.ptr.data(), ch.links.data(), dDist_[b], dNh_[b],
                         dInfo_ + ch.lo),
          "orh_whatif_run");
    if (digests_) {  // the chunk's rows complete in stream order, then digested
      check(ctx_, orh_whatif_flush(job_), "orh_whatif_flush");
      check(ctx_, orh_row_digest(ctx_, dDist_[b], dNh_[b], 1, n_, nr, dDigest_ + ch.lo), "orh_row_digest");
    }
  }
  check(ctx_, orh_whatif_flush(job_), "orh_whatif_flush");
}

double WhatIfBatch::lastMs() const {
  double ms = 0;
  if (!job_) throw std::logic_error("WhatIfBatch: no run");
  check(ctx_, orh_whatif_elapsed_ms(job_, &ms), "orh_whatif_elapsed_ms");
  return ms;
}

void WhatIfBatch::sync() const { check(ctx_, orh_sync(ctx_), "orh_sync"); }

void WhatIfBatch::info(uint32_t* out) const {
  check(ctx_, orh_memcpy_d2h(ctx_, out, dInfo_, srcIdx_.size() * 4), "orh_memcpy_d2h");
}

void WhatIfBatch::digests(uint64_t* out) const {
  if (!digests_) throw std::logic_error("WhatIfBatch: digests were not enabled for the last run");
  check(ctx_, orh_memcpy_d2h(ctx_, out, dDigest_, srcIdx_.size() * 8), "orh_memcpy_d2h");
  if (!shareBase_) return;
  // a request whose source row stands was not copied: its row is the base row
  std::vector<uint32_t> inf(srcIdx_.size());
  std::vector<uint64_t> base(srcs_.size());
  info(inf.data());
  check(ctx_, orh_memcpy_d2h(ctx_, base.data(), dBaseDigest_, base.size() * 8), "orh_memcpy_d2h");
  for (size_t i = 0; i < inf.size(); ++i)
    if (ORH_WHATIF_TIER(inf[i]) == 0) out[i] = base[srcIdx_[i]];
}

void WhatIfBatch::fetch(size_t i, uint32_t* dist, uint32_t* nh) const {
  const Chunk& last = chunks_.back();
  if (i < last.lo || i >= last.hi) throw std::out_of_range("WhatIfBatch.fetch: not in the last chunk");
  if (!job_ || !nBuf_) throw std::logic_error("WhatIfBatch.fetch: no rows (not run, or released)");
  const size_t r = i - last.lo;
  const int b = static_cast<int>((chunks_.size() - 1) % nBuf_);
  const uint32_t* d = dDist_[b] + r * n_;
  const uint32_t* m = dNh_[b] + r * n_;
  if (shareBase_) {  // a request whose source row stands reads the job's base row
    uint32_t inf = 0;
    check(ctx_, orh_memcpy_d2h(ctx_, &inf, dInfo_ + i, 4), "orh_memcpy_d2h");
    if (ORH_WHATIF_TIER(inf) == 0) {
      const uint32_t *bd = nullptr, *bn = nullptr;
      check(ctx_, orh_whatif_base_rows(job_, &bd, &bn), "orh_whatif_base_rows");
      d = bd + static_cast<size_t>(srcIdx_[i]) * n_;
      m = bn + static_cast<size_t>(srcIdx_[i]) * n_;
    }
  }
  check(ctx_, orh_memcpy_d2h(ctx_, dist, d, n_ * 4ull), "orh_memcpy_d2h");
  check(ctx_, orh_memcpy_d2h(ctx_, nh, m, n_ * 4ull), "orh_memcpy_d2h");
}

}  // namespace openr_amd
