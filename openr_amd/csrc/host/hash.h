// Hash functions whose values decide iteration order in the reference's
// unordered containers, so that order-dependent results (KSP2 tie-breaks
// among parallel links, LinkState.cpp:398-419 over :844) match exactly.
//
// folly's std::hash<std::pair<A, B>> (folly rev 1ab6a01f, not present in
// the reference tree) is hash_combine(a, b) = hash_128_to_64(H(a), H(b))
// with H = std::hash; strings use libstdc++'s std::hash<std::string>.
#pragma once

#include <array>
#include <unordered_map>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <tuple>
#include <utility>

namespace openr_amd {

inline uint64_t hash128to64(uint64_t upper, uint64_t lower) {
  constexpr uint64_t kMul = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lower ^ upper) * kMul;
  a ^= (a >> 47);
  uint64_t b = (upper ^ a) * kMul;
  b ^= (b >> 47);
  return b * kMul;
}

inline size_t strHash(const std::string& s) { return std::hash<std::string>{}(s); }

inline size_t pairHash(const std::string& a, const std::string& b) {
  return hash128to64(strHash(a), strHash(b));
}

struct StrPairHash {
  size_t operator()(const std::pair<std::string, std::string>& p) const {
    return pairHash(p.first, p.second);
  }
};

// memo keys (src, dst, k) of getKthPaths; lookup only, never iteration order
struct KthKeyHash {
  size_t operator()(const std::tuple<std::string, std::string, size_t>& k) const {
    return hash128to64(pairHash(std::get<0>(k), std::get<1>(k)), std::get<2>(k));
  }
};

// the (src, dst, k) memo as 16 hash shards (by the key hash's top bits), so
// a batch's entries go in shard by shard on the host pool
template <class V>
class KthMemo {
 public:
  using Key = std::tuple<std::string, std::string, size_t>;
  using Map = std::unordered_map<Key, V, KthKeyHash>;
  static constexpr size_t kShards = 16;
  static size_t shardOf(const Key& k) { return KthKeyHash{}(k) >> 60; }
  Map& of(const Key& k) { return s_[shardOf(k)]; }
  const Map& of(const Key& k) const { return s_[shardOf(k)]; }
  Map& shard(size_t i) { return s_[i]; }
  size_t count(const Key& k) const { return of(k).count(k); }
  bool empty() const {
    for (const auto& m : s_)
      if (!m.empty()) return false;
    return true;
  }
  void clear() {
    for (auto& m : s_) m.clear();
  }
  void reserve(size_t n) {
    for (auto& m : s_) m.reserve(m.size() + n / kShards + 1);
  }

 private:
  std::array<Map, kShards> s_;
};

// Link::hash (LinkState.cpp:138-142): pair of (node, ifName) pairs in
// std::minmax order
inline size_t linkHash(const std::string& n1, const std::string& if1, const std::string& n2,
                       const std::string& if2) {
  return hash128to64(pairHash(n1, if1), pairHash(n2, if2));
}

}  // namespace openr_amd
