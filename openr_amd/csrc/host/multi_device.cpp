// Multi-GPU forms of the SPF path (see multi_device.h).
#include "multi_device.h"

#include "parallel.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>

namespace openr_amd {

namespace {

void check(orh_ctx* ctx, int rc, const char* what) {
  if (rc != ORH_OK)
    throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) + "): " +
                             (ctx ? orh_last_error(ctx) : ""));
}

// fn(r) for every r < n, one host thread each (every device's context is
// driven by its own thread, as the ABI's single-thread-affine contexts allow);
// the first exception is rethrown
template <class F>
void onEachDevice(size_t n, F&& fn) {
  if (n <= 1) {
    if (n) fn(0);
    return;
  }
  std::vector<std::exception_ptr> err(n);
  std::vector<std::thread> th;
  th.reserve(n);
  for (size_t r = 0; r < n; ++r)
    th.emplace_back([&, r] {
      try {
        fn(r);
      } catch (...) {
        err[r] = std::current_exception();
      }
    });
  for (auto& t : th) t.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

}  // namespace

std::vector<size_t> equalWorkCuts(const std::vector<double>& w, size_t world) {
  double sum = 0;
  for (double x : w) sum += x;
  std::vector<size_t> cuts{0};
  double acc = 0;
  for (size_t i = 0, k = 1; i < w.size(); ++i) {
    acc += w[i];
    while (k < world && acc >= sum * static_cast<double>(k) / static_cast<double>(world) && cuts.size() <= k) {
      cuts.push_back(i + 1);
      ++k;
    }
  }
  while (cuts.size() < world) cuts.push_back(w.size());
  cuts.push_back(w.size());
  return cuts;
}

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
// replica 0 owns the host graph store; replicas 1.. are device views of it
// (LinkState's replica constructor): one host update per mutation, every
// device mirror marked with the same delta (LinkState.cpp:564-719 once)
ReplicatedLinkState::ReplicatedLinkState(const std::string& area, const std::vector<int>& devices) {
  if (devices.empty()) throw std::invalid_argument("ReplicatedLinkState: no devices");
  std::map<int, unsigned> seen;
  for (int d : devices) {
    orh_ctx* ctx = deviceContext(d, seen[d]++);
    if (reps_.empty()) reps_.push_back(std::make_unique<LinkState>(area, ctx));
    else reps_.push_back(std::make_unique<LinkState>(*reps_[0], ctx));
  }
}

ReplicatedLinkState::~ReplicatedLinkState() {
  while (reps_.size() > 1) reps_.pop_back();  // the replicas before the store's owner
}

LinkStateChange ReplicatedLinkState::updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl,
                                                             Metric holdDownTtl) {
  return reps_[0]->updateAdjacencyDatabase(db, holdUpTtl, holdDownTtl);
}

LinkStateChange ReplicatedLinkState::deleteAdjacencyDatabase(const std::string& node) {
  return reps_[0]->deleteAdjacencyDatabase(node);
}

LinkStateChange ReplicatedLinkState::decrementHolds() { return reps_[0]->decrementHolds(); }

// ---- MultiDeviceSweep --------------------------------------------------------
MultiDeviceSweep::MultiDeviceSweep(const ReplicatedLinkState& rls, const std::vector<std::string>& srcs,
                                   bool useLinkMetric)
    : useLinkMetric_(useLinkMetric), total_(srcs.size()) {
  const LinkState& ls0 = rls.primary();
  const size_t world = rls.replicas();
  // equal-work contiguous blocks (prefix-sum cut points)
  std::vector<double> w(srcs.size());
  for (size_t i = 0; i < srcs.size(); ++i) {
    if (!ls0.nodeId(srcs[i])) throw std::invalid_argument("MultiDeviceSweep: unknown source " + srcs[i]);
    w[i] = 1.0 + static_cast<double>(ls0.linksFromNode(srcs[i]).size()) / 16.0;
  }
  const std::vector<size_t> cuts = equalWorkCuts(w, world);
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
    b.ls = &ls;
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
  // the replica's graph as it is now (pending deltas flushed); the rows were
  // sized at construction, so a grown topology or mask width needs a new sweep
  b.g = b.ls->deviceGraph();
  uint32_t n = 0, ne = 0, words = 1;
  check(b.ctx, orh_graph_info(b.g, &n, &ne), "orh_graph_info");
  check(b.ctx, orh_spf_words(b.g, b.srcs.data(), static_cast<uint32_t>(b.srcs.size()), &words), "orh_spf_words");
  if (n != n_ || words > words_)
    throw std::runtime_error("MultiDeviceSweep: the topology changed shape since the sweep was made (nodes " +
                             std::to_string(n_) + " -> " + std::to_string(n) + ", mask words " +
                             std::to_string(words_) + " -> " + std::to_string(words) + "): make a new sweep");
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

// ---- MultiDeviceWhatIf -------------------------------------------------------
MultiDeviceWhatIf::MultiDeviceWhatIf(const ReplicatedLinkState& rls, const std::vector<std::string>& srcs,
                                     const std::vector<uint32_t>& srcIdx,
                                     const std::vector<std::vector<uint32_t>>& ignore, uint32_t chunk,
                                     bool useLinkMetric, bool shareBase)
    : total_(srcIdx.size()) {
  if (srcIdx.size() != ignore.size()) throw std::invalid_argument("MultiDeviceWhatIf: one ignore set per request");
  const size_t world = rls.replicas();
  // link ids name the same link on every replica (the same updates applied
  // in the same order); check the cheap invariant
  for (size_t r = 1; r < world; ++r)
    if (rls.replica(r).numLinkSlots() != rls.primary().numLinkSlots() ||
        rls.replica(r).numNodeIds() != rls.primary().numNodeIds())
      throw std::logic_error("MultiDeviceWhatIf: replicas disagree");
  std::vector<double> w(srcs.size(), 0.0);  // work of a source = its request count
  for (uint32_t i : srcIdx) {
    if (i >= srcs.size()) throw std::invalid_argument("MultiDeviceWhatIf: source index out of range");
    w[i] += 1.0;
  }
  const std::vector<size_t> cuts = equalWorkCuts(w, world);
  blocks_.resize(world);
  for (size_t r = 0; r < world; ++r) {
    blocks_[r].lo = cuts[r];
    blocks_[r].hi = cuts[r + 1];
  }
  std::vector<uint32_t> owner(srcs.size());
  for (size_t r = 0; r < world; ++r)
    for (size_t i = cuts[r]; i < cuts[r + 1]; ++i) owner[i] = static_cast<uint32_t>(r);
  for (size_t i = 0; i < srcIdx.size(); ++i) blocks_[owner[srcIdx[i]]].reqs.push_back(i);
  for (size_t r = 0; r < world; ++r) {
    Block& b = blocks_[r];
    if (b.reqs.empty()) continue;
    std::vector<std::string> bs(srcs.begin() + static_cast<ptrdiff_t>(b.lo), srcs.begin() + static_cast<ptrdiff_t>(b.hi));
    std::vector<uint32_t> bi;
    std::vector<std::vector<uint32_t>> bg;
    bi.reserve(b.reqs.size());
    bg.reserve(b.reqs.size());
    for (size_t i : b.reqs) {
      bi.push_back(static_cast<uint32_t>(srcIdx[i] - b.lo));
      bg.push_back(ignore[i]);
    }
    // blocks of a 4-way or wider split are short jobs: their largest repairs
    // are searched in full (ORH_WHATIF_SEARCH_LARGE; rehearsal at 8 blocks:
    // the slowest block 7.1 -> 5.2 ms, profiles/r06/r_whatif_full_ab.txt)
    // ORH_MD_CHUNKS=n (A/B): a block's requests in at least n chunks, so its
    // repairs overlap its later copies as the whole job's do
    static const uint32_t minChunks = [] {
      const char* e = std::getenv("ORH_MD_CHUNKS");
      return e && std::atoi(e) > 0 ? static_cast<uint32_t>(std::atoi(e)) : 1u;
    }();
    const uint32_t n = static_cast<uint32_t>(b.reqs.size());
    const uint32_t bchunk = std::max<uint32_t>(1, std::min(chunk, (n + minChunks - 1) / minChunks));
    b.job = std::make_unique<WhatIfBatch>(rls.replica(r), bs, bi, bg, bchunk, useLinkMetric, shareBase,
                                          world >= kSearchLargeBlocks);
  }
}

void MultiDeviceWhatIf::run() {
  onEachDevice(blocks_.size(), [&](size_t r) { runBlock(r); });
}

void MultiDeviceWhatIf::runBlock(size_t r) {
  Block& b = blocks_.at(r);
  if (b.job) b.job->run();
}

void MultiDeviceWhatIf::sync() {
  for (auto& b : blocks_)
    if (b.job) b.job->sync();
}

void MultiDeviceWhatIf::release(size_t r) {
  Block& b = blocks_.at(r);
  if (b.job) b.job->release();
}

void MultiDeviceWhatIf::setDigests(bool on) {
  for (auto& b : blocks_)
    if (b.job) b.job->setDigests(on);
}

void MultiDeviceWhatIf::info(uint32_t* out) const {
  std::vector<uint32_t> tmp;
  for (const auto& b : blocks_) {
    if (!b.job) continue;
    tmp.resize(b.reqs.size());
    b.job->info(tmp.data());
    for (size_t k = 0; k < b.reqs.size(); ++k) out[b.reqs[k]] = tmp[k];
  }
}

void MultiDeviceWhatIf::digests(uint64_t* out) const {
  std::vector<uint64_t> tmp;
  for (const auto& b : blocks_) {
    if (!b.job) continue;
    tmp.resize(b.reqs.size());
    b.job->digests(tmp.data());
    for (size_t k = 0; k < b.reqs.size(); ++k) out[b.reqs[k]] = tmp[k];
  }
}

// ---- MultiDeviceKthPaths -----------------------------------------------------
MultiDeviceKthPaths::MultiDeviceKthPaths(const ReplicatedLinkState& rls,
                                         const std::vector<std::pair<std::string, std::string>>& pairs)
    : pairs_(pairs), k1_(pairs.size()), k2_(pairs.size()) {
  const size_t world = rls.replicas();
  // distinct sources in first-appearance order, weighted by their pair counts
  std::unordered_map<std::string, size_t> srcPos;
  std::vector<std::vector<size_t>> bySrc;
  for (size_t i = 0; i < pairs.size(); ++i) {
    auto [it, fresh] = srcPos.emplace(pairs[i].first, bySrc.size());
    if (fresh) bySrc.emplace_back();
    bySrc[it->second].push_back(i);
  }
  std::vector<double> w;
  w.reserve(bySrc.size());
  for (const auto& v : bySrc) w.push_back(static_cast<double>(v.size()));
  const std::vector<size_t> cuts = equalWorkCuts(w, world);
  blocks_.resize(world);
  for (size_t r = 0; r < world; ++r) {
    blocks_[r].ls = &rls.replica(r);
    for (size_t s = cuts[r]; s < cuts[r + 1]; ++s)
      blocks_[r].pairs.insert(blocks_[r].pairs.end(), bySrc[s].begin(), bySrc[s].end());
  }
}

void MultiDeviceKthPaths::run() {
  onEachDevice(blocks_.size(), [&](size_t r) { runBlock(r); });
}

void MultiDeviceKthPaths::runBlock(size_t r) {
  Block& b = blocks_.at(r);
  const auto t0 = std::chrono::steady_clock::now();
  b.onDevice = 0;
  std::vector<size_t> host;
  std::vector<size_t> dev;
  std::vector<uint32_t> hs, hd;
  for (size_t i : b.pairs) {
    auto s = b.ls->nodeId(pairs_[i].first);
    auto d = b.ls->nodeId(pairs_[i].second);
    if (!s || !d) {
      host.push_back(i);
      continue;
    }
    dev.push_back(i);
    hs.push_back(*s);
    hd.push_back(*d);
  }
  if (!dev.empty()) {
    orh_graph* g = b.ls->deviceGraph();
    const uint32_t* blk = nullptr;
    uint32_t bw = 0;
    const int rc = orh_ksp2_batch(g, static_cast<uint32_t>(dev.size()), hs.data(), hd.data(), &blk, &bw);
    if (rc == ORH_E_UNSUPPORTED) {
      host.insert(host.end(), dev.begin(), dev.end());
    } else {
      check(b.ls->context(), rc, "orh_ksp2_batch");
      for (size_t j = 0; j < dev.size(); ++j) {
        const uint32_t* p = blk + j * static_cast<size_t>(bw);
        const size_t i = dev[j];
        if (p[0] != 0) {  // outgrew the device trace's bounds
          host.push_back(i);
          continue;
        }
        auto parse = [&](size_t at, std::vector<Path>& out) {
          out.clear();
          const uint32_t n = p[at++];
          for (uint32_t k = 0; k < n; ++k) {
            const uint32_t len = p[at++];
            out.emplace_back(p + at, p + at + len);
            at += len;
          }
        };
        parse(2, k1_[i]);
        parse(p[1], k2_[i]);
        ++b.onDevice;
      }
    }
  }
  for (size_t i : host) {  // the replica's own getKthPaths (host traces over device rows)
    k1_[i] = b.ls->getKthPathIds(pairs_[i].first, pairs_[i].second, 1);
    k2_[i] = b.ls->getKthPathIds(pairs_[i].first, pairs_[i].second, 2);
  }
  b.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

const std::vector<Path>& MultiDeviceKthPaths::paths(size_t i, size_t k) const {
  if (i >= pairs_.size() || (k != 1 && k != 2)) throw std::out_of_range("MultiDeviceKthPaths.paths");
  return k == 1 ? k1_[i] : k2_[i];
}

size_t MultiDeviceKthPaths::devicePairs() const {
  size_t n = 0;
  for (const auto& b : blocks_) n += b.onDevice;
  return n;
}

// ---- ReplicatedAreaLinkStates --------------------------------------------------
ReplicatedAreaLinkStates::ReplicatedAreaLinkStates(const std::vector<int>& devices) {
  if (devices.empty()) throw std::invalid_argument("ReplicatedAreaLinkStates: no devices");
  std::map<int, unsigned> seen;
  for (int d : devices) {
    ctxs_.push_back(deviceContext(d, seen[d]++));
    reps_.push_back(std::make_unique<AreaLinkStates>());
  }
}

ReplicatedAreaLinkStates::~ReplicatedAreaLinkStates() {
  while (reps_.size() > 1) reps_.pop_back();  // the replicas before the stores' owners
}

void ReplicatedAreaLinkStates::addArea(const std::string& area) {
  if (!reps_[0]->count(area))
    reps_[0]->emplace(std::piecewise_construct, std::forward_as_tuple(area), std::forward_as_tuple(area, ctxs_[0]));
  LinkState& primary = reps_[0]->at(area);
  for (size_t r = 1; r < reps_.size(); ++r)
    if (!reps_[r]->count(area))
      reps_[r]->emplace(std::piecewise_construct, std::forward_as_tuple(area),
                        std::forward_as_tuple(primary, ctxs_[r]));
}

LinkStateChange ReplicatedAreaLinkStates::updateAdjacencyDatabase(const AdjacencyDatabase& db, Metric holdUpTtl,
                                                                  Metric holdDownTtl) {
  addArea(db.area);  // one host update: the replicas share replica 0's store
  return reps_[0]->at(db.area).updateAdjacencyDatabase(db, holdUpTtl, holdDownTtl);
}

LinkStateChange ReplicatedAreaLinkStates::deleteAdjacencyDatabase(const std::string& area, const std::string& node) {
  addArea(area);
  return reps_[0]->at(area).deleteAdjacencyDatabase(node);
}

// ---- ShardedRouteBuilder -----------------------------------------------------
ShardedRouteBuilder::ShardedRouteBuilder(const ReplicatedAreaLinkStates& areas, const std::string& myNodeName,
                                         bool enableV4, bool enableOrderedFib, bool bgpDryRun,
                                         bool enableBestRouteSelection)
    : areas_(areas), shardMs_(areas.replicas(), 0.0) {
  const size_t world = areas.replicas();
  for (size_t r = 0; r < world; ++r) {
    solvers_.push_back(std::make_unique<SpfSolver>(myNodeName, enableV4, enableOrderedFib, bgpDryRun,
                                                   enableBestRouteSelection));
    solvers_.back()->setPrefixShard(static_cast<uint32_t>(r), static_cast<uint32_t>(world));
  }
}

size_t ShardedRouteBuilder::releasePrefixMirrors(PrefixState& ps) const {
  size_t n = 0;
  orh_ctx* keep = defaultContext();
  for (size_t r = 0; r < areas_.replicas(); ++r)
    if (areas_.context(r) != keep && ps.dropDeviceMirror(areas_.context(r))) ++n;
  return n;
}

void ShardedRouteBuilder::updateStaticUnicastRoutes(
    const std::vector<std::pair<Cidr, std::vector<NextHopThrift>>>& upd, const std::vector<Cidr>& del) {
  for (auto& s : solvers_) s->updateStaticUnicastRoutes(upd, del);
}

void ShardedRouteBuilder::updateStaticMplsRoutes(
    const std::vector<std::pair<int32_t, std::vector<NextHopThrift>>>& upd, const std::vector<int32_t>& del) {
  for (auto& s : solvers_) s->updateStaticMplsRoutes(upd, del);
}

std::optional<DecisionRouteDb> ShardedRouteBuilder::buildShard(size_t r, const std::string& me,
                                                               const PrefixState& ps) {
  const auto t0 = std::chrono::steady_clock::now();
  auto db = solvers_.at(r)->buildRouteDb(me, areas_.replica(r), ps);
  shardMs_[r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return db;
}

std::optional<DecisionRouteDb> ShardedRouteBuilder::buildRouteDb(const std::string& me, const PrefixState& ps) {
  const size_t world = solvers_.size();
  // every device's prefix mirror brought up to date first (the host runs are
  // rebuilt once, on this thread)
  for (size_t r = 0; r < world; ++r) ps.syncDevice(areas_.context(r));
  std::vector<std::optional<DecisionRouteDb>> parts(world);
  onEachDevice(world, [&](size_t r) { parts[r] = buildShard(r, me, ps); });
  const auto t0 = std::chrono::steady_clock::now();
  if (!parts[0]) return std::nullopt;  // me in no area: every shard says so
  DecisionRouteDb db = std::move(*parts[0]);
  std::vector<UnicastRouteMap> rest;
  rest.reserve(world - 1);
  for (size_t r = 1; r < world; ++r)
    if (parts[r]) rest.push_back(std::move(parts[r]->unicastRoutes));
  if (!rest.empty()) mergeParts(db.unicastRoutes, rest, WorkerPool::instance());
  mergeMs_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return db;
}

}  // namespace openr_amd
