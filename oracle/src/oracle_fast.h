// TEST INFRASTRUCTURE ONLY — an independent fast checker for parity at scale.
//
// The faithful oracle (oracle_link_state.cpp) runs the reference's runSpf with
// its own containers (string-keyed maps, a heap re-made on every decrease):
// ~1 SPF/s on C4's 50k-node WAN, too slow to pin more than a sample of a
// 262,144-request what-if job or 1,024 KSP2 pairs. FastChecker takes a flat
// snapshot of one oracle LinkState (nodes in the caller's order, each node's
// links in its LinkSet iteration order, link up / metric / overload from the
// oracle's own getters) and restates the same semantics with flat arrays:
//
//   spf      runSpf(src, true, ignore) (LinkState.cpp:808-882) in the closed
//            form of SURVEY.md Appendix A.1: binary-heap Dijkstra over up,
//            non-ignored links, no transit through overloaded non-source
//            nodes; NH(u) = union over tight predecessors (l, v) of
//            (v = src ? {u} : NH(v)). Metrics must be >= 1.
//   pathLinks(u)  tight predecessors in extraction order of v, i.e. ascending
//            (d(v), name(v)) (DijkstraQ order, LinkState.h:488-498), then v's
//            LinkSet iteration order (Appendix A.2)
//   kthPaths getKthPaths(src, dst, 1 / 2) (LinkState.cpp:762-791) with
//            traceOnePath (:398-419): DFS over pathLinks in stored order, a
//            link consumed on first touch; k = 2 over a fresh SPF ignoring every
//            k = 1 link
//
// It shares no code with the product (openr_amd/csrc) or with the faithful
// oracle's algorithm; it is validated against the faithful oracle on random
// graphs with parallel links and drained nodes (tests/test_oracle_fast.py).
#pragma once

#include <cstdint>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "oracle_link_state.h"

namespace oracle {

class FastChecker {
 public:
  // (first node, its ifName, second node, its ifName): the oracle's link descriptor
  using Desc = std::tuple<std::string, std::string, std::string, std::string>;
  // nodes in `order` (every node of ls that has links must be listed)
  FastChecker(const LinkState& ls, const std::vector<std::string>& order);

  size_t nodes() const { return names_.size(); }
  size_t links() const { return links_.size(); }
  // the link named by (node, its ifName, other node); -1 if none
  int64_t linkIndex(const std::string& n1, const std::string& if1, const std::string& n2) const;
  Desc linkDesc(uint32_t link) const { return desc_[link]; }
  // distinct neighbour node indices of src, ascending (first-hop mask bit order)
  std::vector<uint32_t> neighbours(uint32_t src) const;

  struct Row {
    std::vector<uint64_t> dist;  // ~0 = unreachable
    std::vector<uint32_t> nh;    // [N * words] first-hop masks over neighbours(src)
    uint32_t words{1};
  };
  // runSpf(src, true, ignore) in closed form
  void spf(uint32_t src, const std::vector<uint32_t>& ignore, Row& out) const;
  // getKthPaths(src, dst, 1) and (src, dst, 2), paths as link indices src -> dst
  void kthPaths(uint32_t src, uint32_t dst, std::vector<std::vector<uint32_t>>& k1,
                std::vector<std::vector<uint32_t>>& k2) const;
  // orh_row_digest of a row with u32 distances (include/openr_hip.h)
  static uint64_t digest(const Row& r);

 private:
  struct Adj {
    uint32_t other, link;
    uint64_t metric;  // Link::getMetricFromNode(this node)
  };
  std::vector<std::string> names_;
  std::vector<uint32_t> nameRank_;  // byte order of the names (DijkstraQ tie order)
  std::vector<uint8_t> overloaded_;
  std::vector<uint32_t> ptr_;  // CSR over nodes, entries in LinkSet iteration order
  std::vector<Adj> adj_;
  std::vector<uint8_t> up_;  // per link: Link::isUp()
  std::vector<Desc> desc_;   // per link: (first node, its ifName, second node)
  std::unordered_map<std::string, uint32_t> byDesc_;
  std::vector<uint32_t> links_;  // link indices 0..L-1 (size only)

  // pathLinks of u in `r` (the reference's insertion order): (link, prev)
  void pathLinks(uint32_t u, const Row& r, const std::vector<uint8_t>& ignored,
                 std::vector<std::pair<uint32_t, uint32_t>>& out) const;
  bool trace(uint32_t src, uint32_t dst, const Row& r, const std::vector<uint8_t>& ignored,
             std::vector<uint8_t>& visited, std::vector<uint32_t>& path) const;
  void spfMasked(uint32_t src, const std::vector<uint8_t>& ignored, Row& out) const;
};

}  // namespace oracle
