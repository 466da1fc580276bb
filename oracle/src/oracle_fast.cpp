// TEST INFRASTRUCTURE ONLY — see oracle_fast.h.
#include "oracle_fast.h"

#include <algorithm>
#include <numeric>
#include <queue>
#include <stdexcept>

namespace oracle {

namespace {

std::string key(const std::string& n1, const std::string& if1, const std::string& n2) {
  std::string k;
  k.reserve(n1.size() + if1.size() + n2.size() + 2);
  k += n1;
  k += '\x01';
  k += if1;
  k += '\x01';
  k += n2;
  return k;
}

uint64_t fmix64(uint64_t z) {  // orh_row_digest's mixer
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

FastChecker::FastChecker(const LinkState& ls, const std::vector<std::string>& order) : names_(order) {
  const size_t n = names_.size();
  std::unordered_map<std::string, uint32_t> idx;
  idx.reserve(n * 2);
  for (size_t i = 0; i < n; ++i)
    if (!idx.emplace(names_[i], static_cast<uint32_t>(i)).second)
      throw std::invalid_argument("FastChecker: duplicate node " + names_[i]);
  std::vector<uint32_t> byName(n);
  std::iota(byName.begin(), byName.end(), 0u);
  std::sort(byName.begin(), byName.end(), [&](uint32_t a, uint32_t b) { return names_[a] < names_[b]; });
  nameRank_.resize(n);
  for (uint32_t r = 0; r < n; ++r) nameRank_[byName[r]] = r;
  overloaded_.resize(n);
  std::unordered_map<const Link*, uint32_t> linkOf;
  ptr_.assign(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    overloaded_[i] = ls.isNodeOverloaded(names_[i]) ? 1 : 0;
    for (const auto& l : ls.linksFromNode(names_[i])) {  // LinkSet iteration order
      auto [it, fresh] = linkOf.emplace(l.get(), static_cast<uint32_t>(up_.size()));
      if (fresh) {
        up_.push_back(l->isUp() ? 1 : 0);
        const std::string& a = l->firstNodeName();
        const std::string& b = l->secondNodeName();
        desc_.emplace_back(a, l->getIfaceFromNode(a), b, l->getIfaceFromNode(b));
        byDesc_.emplace(key(a, l->getIfaceFromNode(a), b), it->second);
        byDesc_.emplace(key(b, l->getIfaceFromNode(b), a), it->second);
      }
      auto o = idx.find(l->getOtherNodeName(names_[i]));
      if (o == idx.end()) throw std::invalid_argument("FastChecker: node " + l->getOtherNodeName(names_[i]) +
                                                      " not in order");
      adj_.push_back(Adj{o->second, it->second, l->getMetricFromNode(names_[i])});
    }
    ptr_[i + 1] = static_cast<uint32_t>(adj_.size());
  }
  links_.resize(up_.size());
}

int64_t FastChecker::linkIndex(const std::string& n1, const std::string& if1, const std::string& n2) const {
  auto it = byDesc_.find(key(n1, if1, n2));
  return it == byDesc_.end() ? -1 : static_cast<int64_t>(it->second);
}

std::vector<uint32_t> FastChecker::neighbours(uint32_t src) const {
  std::vector<uint32_t> v;
  for (uint32_t e = ptr_[src]; e < ptr_[src + 1]; ++e) v.push_back(adj_[e].other);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  return v;
}

void FastChecker::spf(uint32_t src, const std::vector<uint32_t>& ignore, Row& out) const {
  std::vector<uint8_t> ignored(up_.size(), 0);
  for (uint32_t l : ignore) {
    if (l >= up_.size()) throw std::out_of_range("FastChecker: link index");
    ignored[l] = 1;
  }
  spfMasked(src, ignored, out);
}

void FastChecker::spfMasked(uint32_t src, const std::vector<uint8_t>& ignored, Row& out) const {
  const size_t n = names_.size();
  if (src >= n) throw std::out_of_range("FastChecker: source index");
  constexpr uint64_t kInf = ~0ull;
  out.dist.assign(n, kInf);
  // distances: binary-heap Dijkstra (lazy deletion); transit only through the
  // source and nodes that are not overloaded (LinkState.cpp:831-838)
  using Q = std::tuple<uint64_t, uint32_t>;
  std::priority_queue<Q, std::vector<Q>, std::greater<Q>> q;
  std::vector<uint8_t> done(n, 0);
  out.dist[src] = 0;
  q.emplace(0, src);
  while (!q.empty()) {
    const auto [d, v] = q.top();
    q.pop();
    if (done[v] || d != out.dist[v]) continue;
    done[v] = 1;
    if (v != src && overloaded_[v]) continue;
    for (uint32_t e = ptr_[v]; e < ptr_[v + 1]; ++e) {
      const Adj& a = adj_[e];
      if (!up_[a.link] || ignored[a.link]) continue;
      if (a.metric == 0) throw std::invalid_argument("FastChecker: zero-metric link (closed form needs >= 1)");
      const uint64_t nd = d + a.metric;
      if (nd < out.dist[a.other]) {
        out.dist[a.other] = nd;
        q.emplace(nd, a.other);
      }
    }
  }
  // first hops, closed form, nodes in ascending distance
  const std::vector<uint32_t> nb = neighbours(src);
  out.words = std::max<uint32_t>(1, static_cast<uint32_t>((nb.size() + 31) / 32));
  const uint32_t W = out.words;
  out.nh.assign(n * W, 0u);
  std::vector<uint32_t> reach;
  for (uint32_t v = 0; v < n; ++v)
    if (out.dist[v] != kInf && v != src) reach.push_back(v);
  std::sort(reach.begin(), reach.end(), [&](uint32_t a, uint32_t b) { return out.dist[a] < out.dist[b]; });
  for (uint32_t u : reach) {
    uint32_t* mu = out.nh.data() + static_cast<size_t>(u) * W;
    for (uint32_t e = ptr_[u]; e < ptr_[u + 1]; ++e) {
      const Adj& a = adj_[e];
      const uint32_t v = a.other;  // the link from v to u
      if (!up_[a.link] || ignored[a.link] || out.dist[v] == kInf) continue;
      if (v != src && overloaded_[v]) continue;
      // metric from v's side of this link
      uint64_t wv = 0;
      for (uint32_t f = ptr_[v]; f < ptr_[v + 1]; ++f)
        if (adj_[f].link == a.link) {
          wv = adj_[f].metric;
          break;
        }
      if (out.dist[v] + wv != out.dist[u]) continue;
      if (v == src) {
        const uint32_t b = static_cast<uint32_t>(std::lower_bound(nb.begin(), nb.end(), u) - nb.begin());
        mu[b / 32] |= 1u << (b % 32);
      } else {
        const uint32_t* mv = out.nh.data() + static_cast<size_t>(v) * W;
        for (uint32_t k = 0; k < W; ++k) mu[k] |= mv[k];
      }
    }
  }
}

void FastChecker::pathLinks(uint32_t u, const Row& r, const std::vector<uint8_t>& ignored,
                            std::vector<std::pair<uint32_t, uint32_t>>& out) const {
  // tight predecessors (l, v), ordered by v's extraction (dist, name) and then
  // the position of l in v's LinkSet iteration
  struct P {
    uint64_t d;
    uint32_t rank, pos, link, v;
  };
  std::vector<P> ps;
  for (uint32_t e = ptr_[u]; e < ptr_[u + 1]; ++e) {
    const Adj& a = adj_[e];
    const uint32_t v = a.other;
    if (!up_[a.link] || ignored[a.link] || r.dist[v] == ~0ull) continue;
    if (r.dist[v] != 0 && overloaded_[v]) continue;  // no transit through a drained node (src: dist 0)
    for (uint32_t f = ptr_[v]; f < ptr_[v + 1]; ++f) {
      if (adj_[f].link != a.link) continue;
      if (r.dist[v] + adj_[f].metric == r.dist[u]) ps.push_back(P{r.dist[v], nameRank_[v], f - ptr_[v], a.link, v});
      break;
    }
  }
  std::sort(ps.begin(), ps.end(), [](const P& a, const P& b) {
    return std::tie(a.d, a.rank, a.pos) < std::tie(b.d, b.rank, b.pos);
  });
  out.clear();
  for (const P& p : ps) out.emplace_back(p.link, p.v);
}

bool FastChecker::trace(uint32_t src, uint32_t dst, const Row& r, const std::vector<uint8_t>& ignored,
                        std::vector<uint8_t>& visited, std::vector<uint32_t>& path) const {
  if (src == dst) return true;  // Path{}
  std::vector<std::pair<uint32_t, uint32_t>> pl;
  pathLinks(dst, r, ignored, pl);
  for (const auto& [l, prev] : pl) {
    if (visited[l]) continue;
    visited[l] = 1;  // consumed on first touch, even if the branch fails
    if (trace(src, prev, r, ignored, visited, path)) {
      path.push_back(l);
      return true;
    }
  }
  return false;
}

void FastChecker::kthPaths(uint32_t src, uint32_t dst, std::vector<std::vector<uint32_t>>& k1,
                           std::vector<std::vector<uint32_t>>& k2) const {
  k1.clear();
  k2.clear();
  auto traceAll = [&](const Row& r, const std::vector<uint8_t>& ignored, std::vector<std::vector<uint32_t>>& out) {
    if (r.dist[dst] == ~0ull) return;
    std::vector<uint8_t> visited(up_.size(), 0);
    std::vector<uint32_t> p;
    while (trace(src, dst, r, ignored, visited, p) && !p.empty()) {
      out.push_back(p);
      p.clear();
    }
  };
  std::vector<uint8_t> none(up_.size(), 0);
  Row r1;
  spfMasked(src, none, r1);
  traceAll(r1, none, k1);
  std::vector<uint8_t> ign(up_.size(), 0);
  bool any = false;
  for (const auto& p : k1)
    for (uint32_t l : p) any = ign[l] = 1;
  if (!any) {  // getSpfResult's memoized row again (LinkState.cpp:778)
    traceAll(r1, none, k2);
    return;
  }
  Row r2;
  spfMasked(src, ign, r2);
  traceAll(r2, ign, k2);
}

uint64_t FastChecker::digest(const Row& r) {
  uint64_t acc = 0;
  const size_t n = r.dist.size();
  for (size_t v = 0; v < n; ++v) {
    const uint32_t d = r.dist[v] == ~0ull ? 0xFFFFFFFFu : static_cast<uint32_t>(r.dist[v]);
    uint64_t h = fmix64(static_cast<uint64_t>(v) * 0x9E3779B97F4A7C15ull + d);
    for (uint32_t k = 0; k < r.words; ++k)
      h = fmix64(h ^ (static_cast<uint64_t>(r.nh[v * r.words + k]) + static_cast<uint64_t>(k) * 0xC2B2AE3D27D4EB4Full));
    acc += h;
  }
  return acc;
}

}  // namespace oracle
