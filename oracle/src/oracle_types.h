// TEST INFRASTRUCTURE ONLY — part of the CPU oracle under oracle/.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load this code, and only as the checker / the timed CPU baseline. It is
// never linked into libopenr_hip or the openr_amd host library.
//
// Thrift-shaped value types for the oracle, restating the fields the
// Decision path reads:
//   Adjacency / AdjacencyDatabase   openr/if/Types.thrift:74-175
//   PrefixMetrics / PrefixEntry     openr/if/Types.thrift:297-430
//   BinaryAddress / MplsAction /
//   NextHopThrift                   openr/if/Network.thrift:48-100
#pragma once

#include <cstdint>
#include <functional>
#include <optional>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

namespace oracle {

// folly::hash::hash_128_to_64 (folly rev 1ab6a01f, folly/hash/Hash.h), the
// mixer behind folly's std::hash<std::pair<A,B>> specialisation
// = hash_combine(first, second) = hash_128_to_64(H(first), H(second)).
inline uint64_t hash128to64(uint64_t upper, uint64_t lower) {
  const uint64_t k = 0x9ddfea08eb382d69ULL;
  uint64_t a = (lower ^ upper) * k;
  a ^= (a >> 47);
  uint64_t b = (upper ^ a) * k;
  b ^= (b >> 47);
  b *= k;
  return b;
}

inline size_t hashStr(const std::string& s) { return std::hash<std::string>()(s); }

// folly std::hash<std::pair<std::string, std::string>>
struct PairStrHash {
  size_t operator()(const std::pair<std::string, std::string>& p) const {
    return hash128to64(hashStr(p.first), hashStr(p.second));
  }
};

using NodeAndArea = std::pair<std::string, std::string>;  // Types.h:32

struct BinaryAddress {
  std::string addr;  // raw bytes (4 or 16)
  std::optional<std::string> ifName;
  bool operator==(const BinaryAddress& o) const {
    return addr == o.addr && ifName == o.ifName;
  }
  bool operator!=(const BinaryAddress& o) const { return !(*this == o); }
};

struct Adjacency {
  std::string otherNodeName;
  std::string ifName;
  BinaryAddress nextHopV6;
  BinaryAddress nextHopV4;
  int32_t metric{0};
  int32_t adjLabel{0};
  bool isOverloaded{false};
  int32_t rtt{0};
  int64_t timestamp{0};
  int64_t weight{1};
  std::string otherIfName;
};

struct AdjacencyDatabase {
  std::string thisNodeName;
  bool isOverloaded{false};
  std::vector<Adjacency> adjacencies;
  int32_t nodeLabel{0};
  std::string area;
};

struct PrefixMetrics {
  int32_t path_preference{0};
  int32_t source_preference{0};
  int32_t distance{0};
  bool operator==(const PrefixMetrics& o) const {
    return path_preference == o.path_preference &&
        source_preference == o.source_preference && distance == o.distance;
  }
};

enum PrefixTypeV : int32_t { LOOPBACK = 1, BGP = 3 };
enum FwdType : int32_t { FT_IP = 0, FT_SR_MPLS = 1 };
enum FwdAlgo : int32_t { FA_SP_ECMP = 0, FA_KSP2_ED_ECMP = 1 };
enum MplsCode : int32_t { PUSH = 0, SWAP = 1, PHP = 2, POP_AND_LOOKUP = 3 };

// legacy BGP metric vector (Types.thrift:237-290)
struct MetricEntity {
  int64_t type{0}, priority{0};
  int32_t op{0};
  bool isBestPathTieBreaker{false};
  std::vector<int64_t> metric;
  bool operator==(const MetricEntity& o) const {
    return type == o.type && priority == o.priority && op == o.op &&
        isBestPathTieBreaker == o.isBestPathTieBreaker && metric == o.metric;
  }
};
struct MetricVector {
  int64_t version{0};
  std::vector<MetricEntity> metrics;
  bool operator==(const MetricVector& o) const {
    return version == o.version && metrics == o.metrics;
  }
};

struct PrefixEntry {
  std::string prefixAddr;  // masked network bytes
  int32_t prefixLen{0};
  int32_t type{LOOPBACK};
  int32_t forwardingType{FT_IP};
  int32_t forwardingAlgorithm{FA_SP_ECMP};
  std::optional<int64_t> minNexthop;
  std::optional<int32_t> prependLabel;
  PrefixMetrics metrics;
  std::optional<MetricVector> mv;
  std::optional<std::string> data;
  std::set<std::string> tags;  // Types.thrift PrefixEntry field 11 (set<string>)
  bool operator==(const PrefixEntry& o) const {
    return prefixAddr == o.prefixAddr && prefixLen == o.prefixLen &&
        type == o.type && forwardingType == o.forwardingType &&
        forwardingAlgorithm == o.forwardingAlgorithm &&
        minNexthop == o.minNexthop && prependLabel == o.prependLabel &&
        metrics == o.metrics && mv == o.mv && data == o.data && tags == o.tags;
  }
};

struct MplsAction {
  int32_t action{0};
  std::optional<int32_t> swapLabel;
  std::optional<std::vector<int32_t>> pushLabels;
  bool operator==(const MplsAction& o) const {
    return action == o.action && swapLabel == o.swapLabel &&
        pushLabels == o.pushLabels;
  }
};

struct NextHopThrift {
  BinaryAddress address;
  int32_t weight{0};
  std::optional<MplsAction> mplsAction;
  int32_t metric{0};
  std::optional<std::string> area;
  std::optional<std::string> neighborNodeName;
  bool operator==(const NextHopThrift& o) const {
    return address == o.address && weight == o.weight &&
        mplsAction == o.mplsAction && metric == o.metric && area == o.area &&
        neighborNodeName == o.neighborNodeName;
  }
};

// std::hash<NextHopThrift> (openr/common/NetworkUtil.cpp:57-66): additive
// combination of member hashes; only affects unordered_set iteration order.
struct NextHopHash {
  size_t operator()(const NextHopThrift& nh) const {
    size_t h = hashStr(nh.address.addr);
    if (nh.address.ifName) h += hashStr(*nh.address.ifName);
    h += std::hash<int32_t>()(nh.weight) + std::hash<int32_t>()(nh.metric);
    if (nh.mplsAction) {
      h += std::hash<int32_t>()(nh.mplsAction->action);
      if (nh.mplsAction->swapLabel) h += std::hash<int32_t>()(*nh.mplsAction->swapLabel);
      if (nh.mplsAction->pushLabels)
        for (auto l : *nh.mplsAction->pushLabels) h += std::hash<int32_t>()(l);
    }
    return h;
  }
};

// folly::CIDRNetwork key: (masked address bytes, prefix length)
using Cidr = std::pair<std::string, int32_t>;
struct CidrHash {
  size_t operator()(const Cidr& c) const {
    return hash128to64(hashStr(c.first), std::hash<int32_t>()(c.second));
  }
};

inline bool isV4(const Cidr& c) { return c.first.size() == 4; }

// isMplsLabelValid (openr/common/Util.h:202-205)
inline bool isMplsLabelValid(int32_t label) {
  return (static_cast<uint32_t>(label) & 0xfff00000u) == 0;
}

}  // namespace oracle
