// Multi-GPU forms of the SPF path (see multi_device.h).
#include "multi_device.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

namespace openr_amd {

namespace {

void check(orh_ctx* ctx, int rc, const char* what) {
  if (rc != ORH_OK)
    throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " +
                             (ctx ? orh_last_error(ctx) : ""));
}

}  // namespace

orh_ctx* deviceContext(int device, unsigned slot) {
  int def = 0;
  if (const char* e = std::getenv("ORH_DEVICE")) def = std::atoi(e);
  if (device == def && slot == 0) return defaultContext();
  static std::mutex mu;
  static std::map<std::pair<int, unsigned>, orh_ctx*> ctxs;  // process lifetime, as the lanes
  std::lock_guard<std::mutex> lock(mu);
  orh_ctx*& c = ctxs[{device, slot}];
  if (!c) {
    const int rc = orh_create(device, 0, &c);
    if (rc != ORH_OK) {
      c = nullptr;
      throw std::runtime_error("libopenr_hip: orh_create(device " + std::to_string(device) + ", slot " +
                               std::to_string(slot) + ") failed (rc=" + std::to_string(rc) + ")");
    }
  }
  return c;
}

// ---- ReplicatedLinkState -----------------------------------------------------
ReplicatedLinkState::ReplicatedLinkState(const std::string& area, const std::vector<int>& devices) {
  if (devices.empty()) throw std::invalid_argument("ReplicatedLinkState: no devices");
  std::map<int, unsigned> seen;
  for (int d : devices) reps_.push_back(std::make_unique<LinkState>(area, deviceContext(d, seen[d]++)));
}

LinkStateChange ReplicatedLinkState::updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl,
                                                             Metric holdDownTtl) {
  LinkStateChange c = reps_[0]->updateAdjacencyDatabase(db, holdUpTtl, holdDownTtl);
  for (size_t r = 1; r < reps_.size(); ++r) reps_[r]->updateAdjacencyDatabase(db, holdUpTtl, holdDownTtl);
  return c;
}

LinkStateChange ReplicatedLinkState::deleteAdjacencyDatabase(const std::string& node) {
  LinkStateChange c = reps_[0]->deleteAdjacencyDatabase(node);
  for (size_t r = 1; r < reps_.size(); ++r) reps_[r]->deleteAdjacencyDatabase(node);
  return c;
}

LinkStateChange ReplicatedLinkState::decrementHolds() {
  LinkStateChange c = reps_[0]->decrementHolds();
  for (size_t r = 1; r < reps_.size(); ++r) reps_[r]->decrementHolds();
  return c;
}

// ---- MultiDeviceSweep --------------------------------------------------------
MultiDeviceSweep::MultiDeviceSweep(const ReplicatedLinkState& rls, const std::vector<std::string>& srcs,
                                   bool useLinkMetric)
    : useLinkMetric_(useLinkMetric), total_(srcs.size()) {
  const LinkState& ls0 = rls.primary();
  const size_t world = rls.replicas();
  // equal-work contiguous blocks (prefix-sum cut points)
  std::vector<double> w(srcs.size());
  double sum = 0;
  for (size_t i = 0; i < srcs.size(); ++i) {
    if (!ls0.nodeId(srcs[i])) throw std::invalid_argument("MultiDeviceSweep: unknown source " + srcs[i]);
    w[i] = 1.0 + static_cast<double>(ls0.linksFromNode(srcs[i]).size()) / 16.0;
    sum += w[i];
  }
  std::vector<size_t> cuts{0};
  double acc = 0;
  for (size_t i = 0, k = 1; i < srcs.size(); ++i) {
    acc += w[i];
    while (k < world && acc >= sum * static_cast<double>(k) / static_cast<double>(world) && cuts.size() <= k) {
      cuts.push_back(i + 1);
      ++k;
    }
  }
  while (cuts.size() < world) cuts.push_back(srcs.size());
  cuts.push_back(srcs.size());
  // one mask width for every block: the whole list's
  {
    std::vector<uint32_t> ids;
    ids.reserve(srcs.size());
    for (const auto& s : srcs) ids.push_back(*ls0.nodeId(s));
    orh_graph* g0 = ls0.deviceGraph();
    uint32_t ne = 0;
    check(ls0.context(), orh_graph_info(g0, &n_, &ne), "orh_graph_info");
    if (!ids.empty())
      check(ls0.context(), orh_spf_words(g0, ids.data(), static_cast<uint32_t>(ids.size()), &words_),
            "orh_spf_words");
    words_ = std::max(words_, 1u);
  }
  for (size_t r = 0; r < world; ++r) {
    Block b;
    const LinkState& ls = rls.replica(r);
    b.lo = cuts[r];
    b.hi = cuts[r + 1];
    b.ctx = ls.context();
    b.g = ls.deviceGraph();
    for (size_t i = b.lo; i < b.hi; ++i) b.srcs.push_back(*ls.nodeId(srcs[i]));
    const size_t rows = b.hi - b.lo;
    if (rows) {
      if (orh_device_alloc(b.ctx, rows * n_ * 4ull, reinterpret_cast<void**>(&b.dDist)) != ORH_OK ||
          orh_device_alloc(b.ctx, rows * n_ * 4ull * words_, reinterpret_cast<void**>(&b.dNh)) != ORH_OK) {
        if (b.dDist) orh_device_free(b.ctx, b.dDist);
        for (auto& x : blocks_) {
          orh_device_free(x.ctx, x.dDist);
          orh_device_free(x.ctx, x.dNh);
        }
        throw std::runtime_error("MultiDeviceSweep: device allocation failed");
      }
    }
    blocks_.push_back(std::move(b));
  }
}

MultiDeviceSweep::~MultiDeviceSweep() {
  for (auto& b : blocks_) {
    if (b.dDist) orh_device_free(b.ctx, b.dDist);
    if (b.dNh) orh_device_free(b.ctx, b.dNh);
  }
}

void MultiDeviceSweep::runBlock(size_t r) {
  Block& b = blocks_.at(r);
  if (b.srcs.empty()) return;
  orh_spf_request req{};
  req.h_srcs = b.srcs.data();
  req.n_src = static_cast<uint32_t>(b.srcs.size());
  req.use_link_metric = useLinkMetric_ ? 1 : 0;
  check(b.ctx, orh_spf_run(b.g, &req, words_, b.dDist, b.dNh), "orh_spf_run");
}

void MultiDeviceSweep::run() {
  for (size_t r = 0; r < blocks_.size(); ++r) runBlock(r);
}

void MultiDeviceSweep::sync() {
  for (auto& b : blocks_) check(b.ctx, orh_sync(b.ctx), "orh_sync");
}

double MultiDeviceSweep::lastMs(size_t r) const {
  const Block& b = blocks_.at(r);
  if (b.srcs.empty()) return 0.0;
  double ms = 0;
  check(b.ctx, orh_last_spf_ms(b.ctx, &ms), "orh_last_spf_ms");
  return ms;
}

const MultiDeviceSweep::Block& MultiDeviceSweep::blockOf(size_t i) const {
  if (i >= total_) throw std::out_of_range("MultiDeviceSweep: source index out of range");
  for (const auto& b : blocks_)
    if (i >= b.lo && i < b.hi) return b;
  throw std::logic_error("MultiDeviceSweep: blocks do not cover the sources");
}

void MultiDeviceSweep::fetch(size_t i, uint32_t* dist, uint32_t* nh) const {
  const Block& b = blockOf(i);
  const size_t r = i - b.lo;
  check(b.ctx, orh_memcpy_d2h(b.ctx, dist, b.dDist + r * n_, n_ * 4ull), "orh_memcpy_d2h");
  check(b.ctx, orh_memcpy_d2h(b.ctx, nh, b.dNh + r * n_ * static_cast<size_t>(words_), n_ * 4ull * words_),
        "orh_memcpy_d2h");
}

void MultiDeviceSweep::gather(uint32_t* dist, uint32_t* nh) const {
  for (const auto& b : blocks_) {
    const size_t rows = b.hi - b.lo;
    if (!rows) continue;
    check(b.ctx, orh_memcpy_d2h(b.ctx, dist + b.lo * n_, b.dDist, rows * n_ * 4ull), "orh_memcpy_d2h");
    check(b.ctx, orh_memcpy_d2h(b.ctx, nh + b.lo * n_ * static_cast<size_t>(words_), b.dNh,
                                rows * n_ * 4ull * words_),
          "orh_memcpy_d2h");
  }
}

}  // namespace openr_amd
