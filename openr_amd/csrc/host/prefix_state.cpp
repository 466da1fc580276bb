// PrefixState (openr/decision/PrefixState.cpp:17-56) and its device mirror
// (orh_prefix_set): see spf_solver.h.
#include <algorithm>
#include <type_traits>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <stdexcept>

#include "parallel.h"
#include "spf_solver.h"

namespace openr_amd {

namespace {

void check(orh_ctx* ctx, int rc, const char* what) {
  if (rc != ORH_OK)
    throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) +
                             "): " + (ctx ? orh_last_error(ctx) : ""));
}

}  // namespace

PrefixState::~PrefixState() {
  for (auto& m : mirrors_)
    if (m->dev) orh_prefix_destroy(m->dev);
}

std::vector<Cidr> PrefixState::updatePrefix(const std::string& node, const std::string& area,
                                            const PrefixEntry& e) {
  return updatePrefix(node, area, PrefixEntry(e));
}

std::vector<Cidr> PrefixState::updatePrefix(const std::string& node, const std::string& area,
                                            PrefixEntry&& e) {
  Cidr key{e.addr, e.len};
  if (!upsertPrefix(node, area, std::move(e))) return {};
  return {key};
}

bool PrefixState::upsertPrefix(const std::string& node, const std::string& area, PrefixEntry&& e) {
  Cidr key{e.addr, e.len};
  auto& entries = prefixes_[key];
  auto it = entries.find(NodeAndArea{node, area});
  if (it != entries.end() && it->second == e) return false;
  const bool ksp2 = e.forwardingAlgorithm == kAlgoKsp2EdEcmp;
  internName(node);
  internArea(area);
  internTagSet(e.tags);
  if (it == entries.end()) {
    entries.emplace(NodeAndArea{node, area}, PrefixEntryRef(std::move(e)));
  } else {
    ksp2Entries_ -= it->second->forwardingAlgorithm == kAlgoKsp2EdEcmp;
    it->second = PrefixEntryRef(std::move(e));
  }
  ksp2Entries_ += ksp2;
  touch(key, false);
  return true;
}

void PrefixState::reserve(size_t n) {
  // grown geometrically: a load fed in chunks rehashes O(log n) times
  auto grow = [](auto& c, size_t want) {
    if constexpr (std::is_same_v<std::decay_t<decltype(c)>, std::vector<typename std::decay_t<decltype(c)>::value_type>>) {
      if (c.capacity() < want) c.reserve(std::max(want, 2 * c.size()));
    } else {
      if (want > c.bucket_count() * c.max_load_factor()) c.reserve(std::max(want, 2 * c.size()));
    }
  };
  const size_t want = cidrOf_.size() + n;
  grow(prefixes_, want);
  grow(pid_, want);
  grow(cidrOf_, want);
  grow(live_, want);
  grow(isDirty_, want);
  grow(pidStamp_, want);
  grow(run_, want);
  grow(dirty_, dirty_.size() + n);
}

// distinct PrefixEntry.tags sets get ids (0: no tags) that the device mirror
// carries per advertisement, so a RibPolicy tag matcher becomes a table
// lookup per route (orh_route_policy); interned here, on the calling thread,
// so the device records read the table concurrently
uint32_t PrefixState::internTagSet(const std::set<std::string>& tags) {
  if (tags.empty()) return 0;
  if (auto it = tagSetIds_.find(tags); it != tagSetIds_.end()) return it->second;
  auto [it, inserted] = tagSetIds_.emplace(tags, 0u);
  if (inserted) {
    tagSets_.push_back(&it->first);
    it->second = tagSets_.size() < tagIdLimit_ ? static_cast<uint32_t>(tagSets_.size()) : ORH_ADV_TAGSET_OVF;
  }
  return it->second;
}

void PrefixState::setTagSetIdLimit(uint32_t limit) {
  if (!tagSets_.empty()) throw std::logic_error("setTagSetIdLimit: tag sets already interned");
  tagIdLimit_ = std::clamp<uint32_t>(limit, 1u, ORH_ADV_TAGSET_OVF);
}

uint32_t PrefixState::tagSetId(const std::set<std::string>& tags) const {
  if (tags.empty()) return 0;
  auto it = tagSetIds_.find(tags);
  return it == tagSetIds_.end() ? ORH_ADV_TAGSET_OVF : it->second;
}

std::vector<Cidr> PrefixState::deletePrefix(const std::string& node, const std::string& area,
                                            const Cidr& prefix) {
  auto it = prefixes_.find(prefix);
  if (it == prefixes_.end()) return {};
  auto e = it->second.find(NodeAndArea{node, area});
  if (e == it->second.end()) return {};
  ksp2Entries_ -= e->second->forwardingAlgorithm == kAlgoKsp2EdEcmp;
  it->second.erase(e);
  const bool gone = it->second.empty();
  if (gone) prefixes_.erase(it);
  touch(prefix, gone);
  return {prefix};
}

// (looked up first: emplace would build - and free - a node per call)
uint32_t PrefixState::internName(const std::string& n) {
  if (auto it = nameIds_.find(n); it != nameIds_.end()) return it->second;
  nameIds_.emplace(n, static_cast<uint32_t>(names_.size()));
  names_.push_back(n);
  return static_cast<uint32_t>(names_.size() - 1);
}

uint32_t PrefixState::internArea(const std::string& a) {
  if (auto it = areaIds_.find(a); it != areaIds_.end()) return it->second;
  areaIds_.emplace(a, static_cast<uint32_t>(areas_.size()));
  areas_.push_back(a);
  return static_cast<uint32_t>(areas_.size() - 1);
}

std::optional<uint32_t> PrefixState::nameId(const std::string& n) const {
  auto it = nameIds_.find(n);
  if (it == nameIds_.end()) return std::nullopt;
  return it->second;
}

std::optional<uint32_t> PrefixState::areaId(const std::string& a) const {
  auto it = areaIds_.find(a);
  if (it == areaIds_.end()) return std::nullopt;
  return it->second;
}

// a prefix whose advertisement list changed: give it a dense id (or free the
// id when its last advertisement is withdrawn) and queue it for upload
void PrefixState::touch(const Cidr& prefix, bool erased) {
  uint32_t pid;
  stamp_ = nextGeneration();
  // one lookup: a new prefix's slot is made here and numbered below
  auto [it, fresh] = erased ? std::make_pair(pid_.find(prefix), false) : pid_.try_emplace(prefix, 0u);
  if (erased && it == pid_.end()) return;
  if (!fresh) {
    pid = it->second;
    if (erased) {
      pid_.erase(it);
      live_[pid] = 0;
      freePids_.push_back(pid);
      // the prefix's id may go to another prefix: its key is logged
      deleted_.emplace_back(stamp_, prefix);
      if (deleted_.size() > kDeletedLog) {
        deletedFloor_ = deleted_.front().first;
        deleted_.pop_front();
      }
    }
  } else {
    if (!freePids_.empty()) {
      pid = freePids_.back();
      freePids_.pop_back();
      cidrOf_[pid] = prefix;
    } else {
      pid = static_cast<uint32_t>(cidrOf_.size());
      cidrOf_.push_back(prefix);
      live_.push_back(0);
      isDirty_.push_back(0);
      pidStamp_.push_back(0);
      run_.emplace_back(0u, 0u);
    }
    it->second = pid;
    live_[pid] = 1;
  }
  pidStamp_[pid] = stamp_;
  if (!isDirty_[pid]) {
    isDirty_[pid] = 1;
    dirty_.push_back(pid);
  }
  for (auto& m : mirrors_) {  // every device mirror re-uploads it at its next sync
    if (m->full) continue;
    // a mirror that has not synced for a long time (its context no longer
    // builds) stops collecting: past half the prefix ids it reloads whole at
    // its next sync instead, so its dirty list stays bounded
    if (m->dirty.size() > cidrOf_.size() / 2 + 1024) {
      m->full = true;
      std::vector<uint32_t>().swap(m->dirty);
      std::vector<uint8_t>().swap(m->isDirty);
      continue;
    }
    if (m->isDirty.size() <= pid) m->isDirty.resize(cidrOf_.size(), 0);
    if (!m->isDirty[pid]) {
      m->isDirty[pid] = 1;
      m->dirty.push_back(pid);
    }
  }
}

// the device record of one advertisement
orh_adv PrefixState::advRecord(const NodeAndArea& na, const PrefixEntry& e) const {
  uint32_t meta = areaIds_.at(na.second) & ORH_ADV_AREA_MASK;
  if (e.forwardingType == kFwdSrMpls) meta |= ORH_ADV_SR_MPLS;
  if (e.forwardingAlgorithm == kAlgoKsp2EdEcmp) meta |= ORH_ADV_KSP2;
  if (e.type == kPrefixTypeBgp) meta |= ORH_ADV_BGP;
  if (e.minNexthop) meta |= ORH_ADV_MIN_NEXTHOP;
  if (e.prependLabel) meta |= ORH_ADV_PREPEND;
  meta |= tagSetId(e.tags) << ORH_ADV_TAGSET_SHIFT;
  return orh_adv{nameIds_.at(na.first), meta, e.pathPreference, e.sourcePreference, e.distance};
}

void PrefixState::buildRecords(const std::vector<uint32_t>* ids, std::vector<uint32_t>& ptr,
                               std::vector<orh_adv>& recs, std::vector<uint8_t>& fl) const {
  const size_t n = ids ? ids->size() : cidrOf_.size();
  ptr.assign(n + 1, 0);
  fl.assign(n, 0);
  auto& pool = WorkerPool::instance();
  auto each = [&](auto&& fn) {
    if (n >= 16384 && pool.size() > 1) {
      pool.parallelFor(n, [&](size_t, size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) fn(i);
      });
    } else {
      for (size_t i = 0; i < n; ++i) fn(i);
    }
  };
  each([&](size_t i) {
    const uint32_t pid = ids ? (*ids)[i] : static_cast<uint32_t>(i);
    if (!live_[pid]) return;
    ptr[i + 1] = run_[pid].second;
    fl[i] = cidrOf_[pid].first.size() == 4 ? ORH_PFX_V4 : 0;
  });
  for (size_t i = 0; i < n; ++i) ptr[i + 1] += ptr[i];
  recs.resize(ptr[n]);
  each([&](size_t i) {
    const uint32_t pid = ids ? (*ids)[i] : static_cast<uint32_t>(i);
    if (!live_[pid]) return;
    const AdvRef* a = advPool_.data() + run_[pid].first;
    for (uint32_t k = 0; k < ptr[i + 1] - ptr[i]; ++k) recs[ptr[i] + k] = advRecord(*a[k].key, **a[k].entry);
  });
}

bool PrefixState::dropDeviceMirror(orh_ctx* ctx) {
  std::lock_guard<std::mutex> lock(syncMu_);
  for (auto it = mirrors_.begin(); it != mirrors_.end(); ++it) {
    if ((*it)->ctx != ctx) continue;
    if ((*it)->dev) orh_prefix_destroy((*it)->dev);
    mirrors_.erase(it);
    return true;
  }
  return false;
}

orh_prefix_set* PrefixState::syncDevice(orh_ctx* ctx) const {
  if (areas_.size() > ORH_ADV_AREA_MASK + 1)
    throw std::runtime_error("PrefixState: more than 256 areas for the device mirror");
  std::lock_guard<std::mutex> lock(syncMu_);
  Mirror* m = nullptr;
  for (auto& x : mirrors_)
    if (x->ctx == ctx) m = x.get();
  if (!m) {
    auto fresh = std::make_unique<Mirror>();
    fresh->ctx = ctx;
    check(ctx, orh_prefix_create(ctx, &fresh->dev), "orh_prefix_create");
    m = fresh.get();
    mirrors_.push_back(std::move(fresh));
  }
  auto& self = const_cast<PrefixState&>(*this);  // dirty lists: bookkeeping only
  // 1. the host runs (advertisements per prefix id in device numbering order).
  // Host pool mostly garbage: renumber every prefix (and reload every device
  // mirror, whose pools hold the same garbage)
  if (advPool_.size() > 4096 && advPool_.size() > 2 * advLive_) hostFull_ = true;
  // the records the host pass built, reused by the mirrors that need exactly
  // those prefixes (every mirror, when one device builds)
  bool builtAll = false;
  std::vector<uint32_t> bPtr;
  std::vector<orh_adv> bRecs;
  std::vector<uint8_t> bFl;
  std::vector<uint32_t> bIds;
  if (hostFull_) {
    // every prefix's run, in pid order: counts, offsets, then the records,
    // each pass on the worker pool for large states (C5: 1M prefixes)
    const uint32_t n = static_cast<uint32_t>(cidrOf_.size());
    std::vector<const PrefixEntries*> ents(n, nullptr);
    std::vector<uint32_t> ptr(n + 1, 0);
    std::vector<uint8_t> fl(n, 0);
    auto& pool = WorkerPool::instance();
    auto each = [&](auto&& fn) {
      if (n >= 16384 && pool.size() > 1) {
        pool.parallelFor(n, [&](size_t, size_t b, size_t e) {
          for (size_t pid = b; pid < e; ++pid) fn(static_cast<uint32_t>(pid));
        });
      } else {
        for (uint32_t pid = 0; pid < n; ++pid) fn(pid);
      }
    };
    each([&](uint32_t pid) {
      if (!live_[pid]) return;
      auto it = prefixes_.find(cidrOf_[pid]);
      if (it == prefixes_.end()) return;
      ents[pid] = &it->second;
      ptr[pid + 1] = static_cast<uint32_t>(it->second.size());
      fl[pid] = it->first.first.size() == 4 ? ORH_PFX_V4 : 0;
    });
    for (uint32_t pid = 0; pid < n; ++pid) ptr[pid + 1] += ptr[pid];
    std::vector<orh_adv> recs(ptr[n]);
    advPool_.reserve(ptr[n] + ptr[n] / 4 + 1024);  // later deltas append without regrowth
    advPool_.assign(ptr[n], AdvRef{});
    advLive_ = ptr[n];
    each([&](uint32_t pid) {
      run_[pid] = {ptr[pid], ptr[pid + 1] - ptr[pid]};
      if (!ents[pid]) return;
      uint32_t k = ptr[pid];
      for (const auto& [na, e] : *ents[pid]) {
        advPool_[k] = AdvRef{&na, &e};
        recs[k] = advRecord(na, *e);
        ++k;
      }
    });
    hostFull_ = false;
    builtAll = true;
    bPtr = std::move(ptr);
    bRecs = std::move(recs);
    bFl = std::move(fl);
    for (auto& x : mirrors_) {
      x->full = true;
      x->dirty.clear();
      x->isDirty.clear();
    }
  } else if (!dirty_.empty()) {
    // the dirty prefixes' runs appended to the host pool in dirty order (the
    // numbering the device delta uses): counts, offsets, then the records,
    // on the worker pool for large deltas
    const size_t nd = dirty_.size();
    std::vector<const PrefixEntries*> ents(nd, nullptr);
    std::vector<uint32_t> ptr(nd + 1, 0);
    std::vector<uint8_t> fl(nd, 0);
    auto& pool = WorkerPool::instance();
    auto each = [&](auto&& fn) {
      if (nd >= 4096 && pool.size() > 1) {
        pool.parallelFor(nd, [&](size_t, size_t b, size_t e) {
          for (size_t i = b; i < e; ++i) fn(i);
        });
      } else {
        for (size_t i = 0; i < nd; ++i) fn(i);
      }
    };
    each([&](size_t i) {
      const uint32_t pid = dirty_[i];
      if (!live_[pid]) return;
      auto it = prefixes_.find(cidrOf_[pid]);
      if (it == prefixes_.end()) return;
      ents[i] = &it->second;
      ptr[i + 1] = static_cast<uint32_t>(it->second.size());
      fl[i] = it->first.first.size() == 4 ? ORH_PFX_V4 : 0;
    });
    for (size_t i = 0; i < nd; ++i) {
      advLive_ -= run_[dirty_[i]].second;
      ptr[i + 1] += ptr[i];
    }
    advLive_ += ptr[nd];
    const uint32_t base = static_cast<uint32_t>(advPool_.size());
    advPool_.resize(base + ptr[nd]);
    std::vector<orh_adv> recs(ptr[nd]);
    each([&](size_t i) {
      const uint32_t pid = dirty_[i];
      run_[pid] = {base + ptr[i], ptr[i + 1] - ptr[i]};
      if (!ents[i]) return;
      uint32_t k = ptr[i];
      for (const auto& [na, e] : *ents[i]) {
        advPool_[base + k] = AdvRef{&na, &e};
        recs[k] = advRecord(na, *e);
        ++k;
      }
    });
    bIds = dirty_;
    bPtr = std::move(ptr);
    bRecs = std::move(recs);
    bFl = std::move(fl);
  }
  for (uint32_t pid : dirty_) self.isDirty_[pid] = 0;
  self.dirty_.clear();
  // 2. this context's device mirror
  if (m->full) {
    if (!builtAll) buildRecords(nullptr, bPtr, bRecs, bFl);
    check(ctx, orh_prefix_load(m->dev, static_cast<uint32_t>(cidrOf_.size()), bPtr.data(), bRecs.data(),
                               bFl.data()),
          "orh_prefix_load");
    m->full = false;
  } else if (!m->dirty.empty()) {
    const auto t1 = std::chrono::steady_clock::now();
    if (m->dirty != bIds) buildRecords(&m->dirty, bPtr, bRecs, bFl);
    check(ctx, orh_prefix_apply_delta(m->dev, static_cast<uint32_t>(m->dirty.size()), m->dirty.data(),
                                      bPtr.data(), bRecs.data(), bFl.data()),
          "orh_prefix_apply_delta");
    if (std::getenv("ORH_ROUTE_PROF")) {  // phase times (see spf_solver.cpp)
      const auto t2 = std::chrono::steady_clock::now();
      std::fprintf(stderr, "route-prof   sync: %zu dirty prefixes, device delta %.3f ms\n", m->dirty.size(),
                   std::chrono::duration<double, std::milli>(t2 - t1).count());
    }
  }
  for (uint32_t pid : m->dirty) m->isDirty[pid] = 0;
  m->dirty.clear();
  if (m->namesOrdered != names_.size() || m->areasOrdered != areas_.size()) {
    // std::set<NodeAndArea> order = byte order of the names, then areas
    auto ranks = [](const std::vector<std::string>& v) {
      std::vector<uint32_t> idx(v.size()), rank(v.size());
      std::iota(idx.begin(), idx.end(), 0u);
      std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return v[a] < v[b]; });
      for (uint32_t r = 0; r < idx.size(); ++r) rank[idx[r]] = r;
      return rank;
    };
    const auto nr = ranks(names_), ar = ranks(areas_);
    check(ctx, orh_prefix_set_order(m->dev, static_cast<uint32_t>(names_.size()), nr.data(),
                                    static_cast<uint32_t>(areas_.size()), ar.data()),
          "orh_prefix_set_order");
    m->namesOrdered = static_cast<uint32_t>(names_.size());
    m->areasOrdered = static_cast<uint32_t>(areas_.size());
  }
  return m->dev;
}

}  // namespace openr_amd
