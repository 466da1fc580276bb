// TEST INFRASTRUCTURE ONLY — Python bindings of the CPU oracle.
// Loaded only by tests/, __graft_entry__.smoke() and bench.py (cpu_baseline).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <thread>

#include "oracle_decision.h"
#include "oracle_fast.h"
#include "oracle_rib_policy.h"

namespace py = pybind11;
using namespace oracle;

namespace {

// fn(i) for i < n on `threads` threads (interleaved), the first exception rethrown
template <class F>
void parallelOver(size_t n, int threads, F&& fn) {
  threads = std::max(1, std::min<int>(threads, static_cast<int>(std::max<size_t>(n, 1))));
  std::vector<std::thread> ws;
  std::vector<std::exception_ptr> errs(threads);
  for (int t = 0; t < threads; ++t)
    ws.emplace_back([&, t] {
      try {
        for (size_t i = t; i < n; i += threads) fn(i);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
  for (auto& w : ws) w.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

std::string bytesOf(const py::handle& h) { return h.cast<std::string>(); }

Adjacency adjFromWire(const py::tuple& t) {
  Adjacency a;
  a.otherNodeName = t[0].cast<std::string>();
  a.ifName = t[1].cast<std::string>();
  a.nextHopV6.addr = bytesOf(t[2]);
  a.nextHopV4.addr = bytesOf(t[3]);
  a.metric = t[4].cast<int32_t>();
  a.adjLabel = t[5].cast<int32_t>();
  a.isOverloaded = t[6].cast<bool>();
  a.rtt = t[7].cast<int32_t>();
  a.timestamp = t[8].cast<int64_t>();
  a.weight = t[9].cast<int64_t>();
  a.otherIfName = t[10].cast<std::string>();
  return a;
}

AdjacencyDatabase adjDbFromWire(const py::tuple& t) {
  AdjacencyDatabase db;
  db.thisNodeName = t[0].cast<std::string>();
  db.isOverloaded = t[1].cast<bool>();
  for (auto a : t[2].cast<py::list>()) db.adjacencies.push_back(adjFromWire(a.cast<py::tuple>()));
  db.nodeLabel = t[3].cast<int32_t>();
  db.area = t[4].cast<std::string>();
  return db;
}

PrefixEntry entryFromWire(const py::tuple& t) {
  PrefixEntry e;
  e.prefixAddr = bytesOf(t[0]);
  e.prefixLen = t[1].cast<int32_t>();
  e.type = t[2].cast<int32_t>();
  e.forwardingType = t[3].cast<int32_t>();
  e.forwardingAlgorithm = t[4].cast<int32_t>();
  if (!t[5].is_none()) e.minNexthop = t[5].cast<int64_t>();
  if (!t[6].is_none()) e.prependLabel = t[6].cast<int32_t>();
  auto m = t[7].cast<py::tuple>();
  e.metrics = {m[0].cast<int32_t>(), m[1].cast<int32_t>(), m[2].cast<int32_t>()};
  if (!t[8].is_none()) {
    auto mvt = t[8].cast<py::tuple>();
    MetricVector mv;
    mv.version = mvt[0].cast<int64_t>();
    for (auto ent : mvt[1]) {
      auto et = ent.cast<py::tuple>();
      MetricEntity me;
      me.type = et[0].cast<int64_t>();
      me.priority = et[1].cast<int64_t>();
      me.op = et[2].cast<int32_t>();
      me.isBestPathTieBreaker = et[3].cast<bool>();
      me.metric = et[4].cast<std::vector<int64_t>>();
      mv.metrics.push_back(me);
    }
    e.mv = mv;
  }
  if (!t[9].is_none()) e.data = bytesOf(t[9]);
  if (t.size() > 10 && !t[10].is_none())
    for (auto tag : t[10]) e.tags.insert(tag.cast<std::string>());
  return e;
}

py::object entryToWire(const PrefixEntry& e) {
  py::object mv = py::none();
  if (e.mv) {
    py::list ents;
    for (const auto& me : e.mv->metrics)
      ents.append(py::make_tuple(me.type, me.priority, me.op, me.isBestPathTieBreaker,
                                 py::tuple(py::cast(me.metric))));
    mv = py::make_tuple(e.mv->version, ents);
  }
  return py::make_tuple(py::bytes(e.prefixAddr), e.prefixLen, e.type, e.forwardingType,
                        e.forwardingAlgorithm, py::cast(e.minNexthop),
                        py::cast(e.prependLabel),
                        py::make_tuple(e.metrics.path_preference,
                                       e.metrics.source_preference, e.metrics.distance),
                        mv, e.data ? py::object(py::bytes(*e.data)) : py::none(),
                        py::tuple(py::cast(std::vector<std::string>(e.tags.begin(), e.tags.end()))));
}

NextHopThrift nhFromWire(const py::tuple& t) {
  NextHopThrift nh;
  nh.address.addr = bytesOf(t[0]);
  if (!t[1].is_none()) nh.address.ifName = t[1].cast<std::string>();
  nh.weight = t[2].cast<int32_t>();
  if (!t[3].is_none()) {
    auto a = t[3].cast<py::tuple>();
    MplsAction act;
    act.action = a[0].cast<int32_t>();
    if (!a[1].is_none()) act.swapLabel = a[1].cast<int32_t>();
    if (!a[2].is_none()) act.pushLabels = a[2].cast<std::vector<int32_t>>();
    nh.mplsAction = act;
  }
  nh.metric = t[4].cast<int32_t>();
  if (!t[5].is_none()) nh.area = t[5].cast<std::string>();
  if (!t[6].is_none()) nh.neighborNodeName = t[6].cast<std::string>();
  return nh;
}

py::tuple nhToWire(const NextHopThrift& nh) {
  py::object act = py::none();
  if (nh.mplsAction) {
    act = py::make_tuple(nh.mplsAction->action, py::cast(nh.mplsAction->swapLabel),
                         nh.mplsAction->pushLabels
                             ? py::object(py::tuple(py::cast(*nh.mplsAction->pushLabels)))
                             : py::none());
  }
  return py::make_tuple(py::bytes(nh.address.addr), py::cast(nh.address.ifName), nh.weight,
                        act, nh.metric, py::cast(nh.area), py::cast(nh.neighborNodeName));
}

py::list nhsToWire(const NextHopSet& s) {
  py::list l;
  for (const auto& nh : s) l.append(nhToWire(nh));
  return l;
}

py::tuple unicastToWire(const RibUnicastEntry& e) {
  return py::make_tuple(py::bytes(e.prefix.first), e.prefix.second, nhsToWire(e.nexthops),
                        e.doNotInstall, e.bestArea,
                        e.bestPrefixEntry ? entryToWire(*e.bestPrefixEntry) : py::none());
}

py::tuple routeDbToWire(const DecisionRouteDb& db) {
  py::list uc, mp;
  for (const auto& [_, e] : db.unicastRoutes) uc.append(unicastToWire(e));
  for (const auto& [_, e] : db.mplsRoutes) mp.append(py::make_tuple(e.label, nhsToWire(e.nexthops)));
  return py::make_tuple(uc, mp);
}

RibUnicastEntry unicastFromWire(const py::tuple& t) {
  RibUnicastEntry e;
  e.prefix = {bytesOf(t[0]), t[1].cast<int32_t>()};
  for (auto nh : t[2]) e.nexthops.insert(nhFromWire(nh.cast<py::tuple>()));
  e.doNotInstall = t[3].cast<bool>();
  e.bestArea = t[4].cast<std::string>();
  if (!t[5].is_none()) e.bestPrefixEntry = entryFromWire(t[5].cast<py::tuple>());
  return e;
}

RibMplsEntry mplsFromWire(const py::tuple& t) {
  RibMplsEntry e;
  e.label = t[0].cast<int32_t>();
  for (auto nh : t[1]) e.nexthops.insert(nhFromWire(nh.cast<py::tuple>()));
  return e;
}

DecisionRouteDb routeDbFromWire(const py::tuple& w) {
  DecisionRouteDb db;
  for (auto u : w[0]) {
    auto e = unicastFromWire(u.cast<py::tuple>());
    db.unicastRoutes.emplace(e.prefix, e);
  }
  for (auto m : w[1]) {
    auto e = mplsFromWire(m.cast<py::tuple>());
    db.mplsRoutes.emplace(e.label, e);
  }
  return db;
}

py::tuple deltaToWire(const DecisionRouteUpdate& d) {
  py::list uu, ud, mu;
  for (const auto& kv : d.unicastRoutesToUpdate) uu.append(unicastToWire(kv.second));
  for (const auto& p : d.unicastRoutesToDelete) ud.append(py::make_tuple(py::bytes(p.first), p.second));
  for (const auto& e : d.mplsRoutesToUpdate) mu.append(py::make_tuple(e.label, nhsToWire(e.nexthops)));
  return py::make_tuple(uu, ud, mu, py::cast(d.mplsRoutesToDelete));
}

DecisionRouteUpdate deltaFromWire(const py::tuple& w) {
  DecisionRouteUpdate d;
  for (auto u : w[0]) {
    auto e = unicastFromWire(u.cast<py::tuple>());
    d.unicastRoutesToUpdate.emplace(e.prefix, e);
  }
  for (auto p : w[1]) {
    auto t = p.cast<py::tuple>();
    d.unicastRoutesToDelete.emplace_back(bytesOf(t[0]), t[1].cast<int32_t>());
  }
  for (auto m : w[2]) d.mplsRoutesToUpdate.push_back(mplsFromWire(m.cast<py::tuple>()));
  d.mplsRoutesToDelete = w[3].cast<std::vector<int32_t>>();
  return d;
}

py::tuple changeToWire(const LinkStateChange& c) {
  return py::make_tuple(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged);
}

py::tuple linkDesc(const Link& l) {
  const auto& a = l.firstNodeName();
  const auto& b = l.secondNodeName();
  return py::make_tuple(a, l.getIfaceFromNode(a), b, l.getIfaceFromNode(b));
}

py::list pathToWire(const Path& p) {
  py::list l;
  for (const auto& link : p) l.append(linkDesc(*link));
  return l;
}

// ---- canonical route-db digest (checker for full-size configs) -------------
// Each route is serialised field by field (integers little-endian, strings and
// lists length-prefixed, optionals with a presence byte; nexthops sorted by
// their serialised bytes) and hashed with FNV-1a 64; routes are ordered by
// (prefix bytes, length) and labels. The same format is implemented
// independently by the product (openr_amd/csrc/host/host_py.cpp).
struct Ser {
  std::string b;
  void raw(const void* p, size_t n) { b.append(static_cast<const char*>(p), n); }
  void u8(uint8_t v) { raw(&v, 1); }
  void i32(int32_t v) { raw(&v, 4); }
  void i64(int64_t v) { raw(&v, 8); }
  void str(const std::string& s) {
    i32(static_cast<int32_t>(s.size()));
    raw(s.data(), s.size());
  }
  template <class T, class F>
  void opt(const std::optional<T>& o, F&& f) {
    u8(o ? 1 : 0);
    if (o) f(*o);
  }
};

uint64_t fnv(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

std::string serNh(const NextHopThrift& nh) {
  Ser s;
  s.str(nh.address.addr);
  s.opt(nh.address.ifName, [&](const std::string& x) { s.str(x); });
  s.i32(nh.weight);
  s.opt(nh.mplsAction, [&](const MplsAction& a) {
    s.i32(a.action);
    s.opt(a.swapLabel, [&](int32_t x) { s.i32(x); });
    s.opt(a.pushLabels, [&](const std::vector<int32_t>& l) {
      s.i32(static_cast<int32_t>(l.size()));
      for (int32_t x : l) s.i32(x);
    });
  });
  s.i32(nh.metric);
  s.opt(nh.area, [&](const std::string& x) { s.str(x); });
  s.opt(nh.neighborNodeName, [&](const std::string& x) { s.str(x); });
  return s.b;
}

void serNhs(Ser& s, const NextHopSet& nhs) {
  std::vector<std::string> v;
  for (const auto& nh : nhs) v.push_back(serNh(nh));
  std::sort(v.begin(), v.end());
  s.i32(static_cast<int32_t>(v.size()));
  for (const auto& x : v) s.str(x);
}

void serEntry(Ser& s, const PrefixEntry& e) {
  s.str(e.prefixAddr);
  s.i32(e.prefixLen);
  s.i32(e.type);
  s.i32(e.forwardingType);
  s.i32(e.forwardingAlgorithm);
  s.opt(e.minNexthop, [&](int64_t x) { s.i64(x); });
  s.opt(e.prependLabel, [&](int32_t x) { s.i32(x); });
  s.i32(e.metrics.path_preference);
  s.i32(e.metrics.source_preference);
  s.i32(e.metrics.distance);
  s.opt(e.mv, [&](const MetricVector& mv) {
    s.i64(mv.version);
    s.i32(static_cast<int32_t>(mv.metrics.size()));
    for (const auto& m : mv.metrics) {
      s.i64(m.type);
      s.i64(m.priority);
      s.i32(m.op);
      s.u8(m.isBestPathTieBreaker ? 1 : 0);
      s.i32(static_cast<int32_t>(m.metric.size()));
      for (int64_t x : m.metric) s.i64(x);
    }
  });
  s.opt(e.data, [&](const std::string& x) { s.str(x); });
  if (!e.tags.empty()) {  // sorted (std::set); absent for tag-free entries
    s.i32(static_cast<int32_t>(e.tags.size()));
    for (const auto& t : e.tags) s.str(t);
  }
}

// (n_unicast, n_mpls, per-route FNV digests as little-endian u64 bytes)
py::tuple routeDbDigest(const DecisionRouteDb& db) {
  std::vector<const RibUnicastEntry*> uc;
  for (const auto& kv : db.unicastRoutes) uc.push_back(&kv.second);
  std::sort(uc.begin(), uc.end(),
            [](const RibUnicastEntry* a, const RibUnicastEntry* b) { return a->prefix < b->prefix; });
  std::vector<const RibMplsEntry*> mp;
  for (const auto& kv : db.mplsRoutes) mp.push_back(&kv.second);
  std::sort(mp.begin(), mp.end(),
            [](const RibMplsEntry* a, const RibMplsEntry* b) { return a->label < b->label; });
  std::string out;
  out.reserve(8 * (uc.size() + mp.size()));
  for (const auto* e : uc) {
    Ser s;
    s.str(e->prefix.first);
    s.i32(e->prefix.second);
    s.u8(e->doNotInstall ? 1 : 0);
    s.str(e->bestArea);
    s.opt(e->bestPrefixEntry, [&](const PrefixEntry& p) { serEntry(s, p); });
    serNhs(s, e->nexthops);
    const uint64_t h = fnv(s.b);
    out.append(reinterpret_cast<const char*>(&h), 8);
  }
  for (const auto* e : mp) {
    Ser s;
    s.i32(e->label);
    serNhs(s, e->nexthops);
    const uint64_t h = fnv(s.b);
    out.append(reinterpret_cast<const char*>(&h), 8);
  }
  return py::make_tuple(uc.size(), mp.size(), py::bytes(out));
}

// std::unordered_map would be converted to a dict by pybind11/stl.h; wrap it
struct AreaMap {
  AreaLinkStates m;
};

// (name, prefixes | None, tags | None, (default, {area: w}, {nbr: w}) | None),
// the wire form openr_amd/rib_policy.py gives both backends
RibPolicyStatementSpec statementFromWire(const py::tuple& t) {
  RibPolicyStatementSpec s;
  s.name = t[0].cast<std::string>();
  if (!t[1].is_none()) {
    s.prefixes.emplace();
    for (auto p : t[1]) {
      auto pt = p.cast<py::tuple>();
      s.prefixes->emplace_back(bytesOf(pt[0]), pt[1].cast<int32_t>());
    }
  }
  if (!t[2].is_none()) s.tags = t[2].cast<std::vector<std::string>>();
  if (!t[3].is_none()) {
    auto w = t[3].cast<py::tuple>();
    RibRouteActionWeight a;
    a.default_weight = w[0].cast<int32_t>();
    a.area_to_weight = w[1].cast<std::map<std::string, int32_t>>();
    a.neighbor_to_weight = w[2].cast<std::map<std::string, int32_t>>();
    s.set_weight = std::move(a);
  }
  return s;
}

struct StatementProbe {  // a lone RibPolicyStatement (RibPolicyTest.cpp statement tests)
  RibPolicyStatement st;
  uint64_t invalidated{0};
};

}  // namespace

PYBIND11_MODULE(openr_oracle, m) {
  m.def("calculate_update", [](py::tuple old_db, py::tuple new_db) {
    return deltaToWire(routeDbFromWire(old_db).calculateUpdate(routeDbFromWire(new_db)));
  });
  m.def("apply_update", [](py::tuple db, py::tuple delta) {
    DecisionRouteDb d = routeDbFromWire(db);
    d.update(deltaFromWire(delta));
    return routeDbToWire(d);
  });
  m.doc() = "CPU oracle (test infrastructure): restatement of the OpenR Decision SPF / route build";

  py::class_<LinkState>(m, "LinkState")
      .def(py::init<const std::string&>())
      .def("update_adjacency_database",
           [](LinkState& s, py::tuple db, uint64_t up, uint64_t down) {
             return changeToWire(s.updateAdjacencyDatabase(adjDbFromWire(db), up, down));
           },
           py::arg("db"), py::arg("hold_up_ttl") = 0, py::arg("hold_down_ttl") = 0)
      .def("delete_adjacency_database",
           [](LinkState& s, const std::string& n) { return changeToWire(s.deleteAdjacencyDatabase(n)); })
      .def("decrement_holds", [](LinkState& s) { return changeToWire(s.decrementHolds()); })
      .def("has_holds", &LinkState::hasHolds)
      .def("has_node", &LinkState::hasNode)
      .def("is_node_overloaded", &LinkState::isNodeOverloaded)
      .def("num_links", &LinkState::numLinks)
      .def("num_nodes", &LinkState::numNodes)
      .def_property_readonly("spf_runs", [](const LinkState& s) { return s.spfRuns; })
      .def("links_from_node",
           [](const LinkState& s, const std::string& n) {
             py::list l;
             for (const auto& link : s.linksFromNode(n)) l.append(linkDesc(*link));
             return l;
           })
      .def("get_spf_result",
           [](const LinkState& s, const std::string& n, bool useLinkMetric) {
             py::dict d;
             for (const auto& [name, r] : s.getSpfResult(n, useLinkMetric)) {
               std::vector<std::string> nhs(r.nextHops().begin(), r.nextHops().end());
               std::sort(nhs.begin(), nhs.end());
               py::list pls;
               for (const auto& pl : r.pathLinks()) pls.append(py::make_tuple(linkDesc(*pl.link), pl.prevNode));
               d[py::str(name)] = py::make_tuple(r.metric(), nhs, pls);
             }
             return d;
           },
           py::arg("node"), py::arg("use_link_metric") = true)
      .def("run_spf_ignoring",
           [](const LinkState& s, const std::string& src, std::vector<py::tuple> ignore) {
             // runSpf(src, true, linksToIgnore) for links named by descriptor
             LinkSet ign;
             for (auto& t : ignore) {
               auto n1 = t[0].cast<std::string>();
               auto if1 = t[1].cast<std::string>();
               for (const auto& link : s.linksFromNode(n1))
                 if (link->getIfaceFromNode(n1) == if1 &&
                     link->getOtherNodeName(n1) == t[2].cast<std::string>())
                   ign.insert(link);
             }
             py::dict d;
             for (const auto& [name, r] : s.runSpf(src, true, ign)) {
               std::vector<std::string> nhs(r.nextHops().begin(), r.nextHops().end());
               std::sort(nhs.begin(), nhs.end());
               d[py::str(name)] = py::make_tuple(r.metric(), nhs);
             }
             return d;
           })
      .def("get_kth_paths",
           [](const LinkState& s, const std::string& a, const std::string& b, size_t k) {
             py::list out;
             for (const auto& p : s.getKthPaths(a, b, k)) out.append(pathToWire(p));
             return out;
           })
      .def("get_metric_from_a_to_b", &LinkState::getMetricFromAToB, py::arg("a"), py::arg("b"),
           py::arg("use_link_metric") = true)
      .def("get_hops_from_a_to_b", &LinkState::getHopsFromAToB)
      .def("get_max_hops_to_node", &LinkState::getMaxHopsToNode)
      .def("metric_from_node",
           [](const LinkState& s, const std::string& n1, const std::string& if1,
              const std::string& from) {
             for (const auto& link : s.linksFromNode(n1))
               if (link->getIfaceFromNode(n1) == if1) return link->getMetricFromNode(from);
             throw std::out_of_range("no such link");
           })
      .def("spf_tables",
           [](const LinkState& s, std::vector<std::string> srcs, std::vector<std::string> order,
              std::vector<std::vector<std::string>> nbrs, int threads,
              std::vector<std::vector<std::tuple<std::string, std::string, std::string>>> ignores) {
             // dist [S][N] (u32, 0xFFFFFFFF = absent) in `order`, and nexthop
             // sets as bitmasks [S][N][W] over each source's `nbrs` list;
             // runSpf(src, true, ignores[i]) per source on per-thread LinkState
             // copies (ignores: per source a list of link descriptors
             // (n1, if1, n2), or empty = no ignore sets)
             if (nbrs.size() != srcs.size()) throw std::invalid_argument("one nbr list per source");
             if (!ignores.empty() && ignores.size() != srcs.size())
               throw std::invalid_argument("one ignore list per source");
             const size_t S = srcs.size(), N = order.size();
             size_t W = 1;
             for (const auto& l : nbrs) W = std::max(W, (l.size() + 31) / 32);
             py::array_t<uint32_t> dist({S, N}), nh({S, N, W});
             uint32_t* pd = dist.mutable_data();
             uint32_t* pn = nh.mutable_data();
             std::string err;
             {
               py::gil_scoped_release rel;
               std::unordered_map<std::string, size_t> col;
               for (size_t i = 0; i < N; ++i) col.emplace(order[i], i);
               threads = std::max(1, std::min<int>(threads, static_cast<int>(S)));
               std::vector<LinkState> copies;
               copies.reserve(threads);
               for (int t = 0; t < threads; ++t) {
                 copies.emplace_back(s.getArea());
                 for (const auto& kv : s.getAdjacencyDatabases())
                   copies.back().updateAdjacencyDatabase(kv.second);
               }
               std::vector<std::thread> ws;
               std::vector<std::string> errs(threads);
               for (int t = 0; t < threads; ++t) {
                 ws.emplace_back([&, t] {
                   for (size_t i = t; i < S; i += threads) {
                     std::unordered_map<std::string, size_t> bit;
                     for (size_t k = 0; k < nbrs[i].size(); ++k) bit.emplace(nbrs[i][k], k);
                     uint32_t* d = pd + i * N;
                     uint32_t* m = pn + i * N * W;
                     std::fill(d, d + N, 0xFFFFFFFFu);
                     std::fill(m, m + N * W, 0u);
                     LinkSet ign;
                     if (!ignores.empty()) {
                       for (const auto& [n1, if1, n2] : ignores[i]) {
                         bool found = false;
                         for (const auto& link : copies[t].linksFromNode(n1))
                           if (link->getIfaceFromNode(n1) == if1 && link->getOtherNodeName(n1) == n2) {
                             ign.insert(link);
                             found = true;
                           }
                         if (!found) {
                           errs[t] = "ignored link " + n1 + "/" + if1 + " not found";
                           return;
                         }
                       }
                     }
                     for (const auto& [name, r] : copies[t].runSpf(srcs[i], true, ign)) {
                       auto c = col.find(name);
                       if (c == col.end()) {
                         errs[t] = "node " + name + " not in order";
                         return;
                       }
                       d[c->second] = static_cast<uint32_t>(r.metric());
                       for (const auto& h : r.nextHops()) {
                         auto b = bit.find(h);
                         if (b == bit.end()) {
                           errs[t] = "nexthop " + h + " of " + srcs[i] + " not a neighbour";
                           return;
                         }
                         m[c->second * W + b->second / 32] |= 1u << (b->second % 32);
                       }
                     }
                   }
                 });
               }
               for (auto& w : ws) w.join();
               for (auto& e : errs)
                 if (!e.empty()) err = e;
             }
             if (!err.empty()) throw std::runtime_error("spf_tables: " + err);
             return py::make_tuple(dist, nh);
           },
           py::arg("srcs"), py::arg("order"), py::arg("nbrs"), py::arg("threads") = 8,
           py::arg("ignores") = std::vector<std::vector<std::tuple<std::string, std::string, std::string>>>{})
      .def("kth_paths_threaded",
           [](const LinkState& s, std::vector<std::pair<std::string, std::string>> pairs, int threads,
              std::vector<std::string> replay) {
             // getKthPaths(src, dst, 1) and (src, dst, 2) per pair on per-thread
             // LinkState copies (the memo is not thread-safe), pairs of one
             // source on one thread (its SpfResult memoised there). The copies
             // replay the adjacency databases in `replay` order - the order the
             // caller loaded them - so every LinkSet has the original's
             // insertion sequence and iteration order (parallel-link ties).
             std::vector<std::vector<Path>> k1(pairs.size()), k2(pairs.size());
             {
               py::gil_scoped_release rel;
               threads = std::max(1, std::min<int>(threads, static_cast<int>(pairs.size())));
               const auto& dbs = s.getAdjacencyDatabases();
               for (const auto& n : replay)
                 if (!dbs.count(n)) throw std::invalid_argument("kth_paths_threaded: no database of " + n);
               std::map<std::string, int> owner;
               for (const auto& p : pairs) owner.emplace(p.first, static_cast<int>(owner.size()) % threads);
               std::vector<std::thread> ws;
               for (int t = 0; t < threads; ++t) {
                 ws.emplace_back([&, t] {
                   LinkState copy(s.getArea());  // built on its thread
                   for (const auto& n : replay) copy.updateAdjacencyDatabase(dbs.at(n));
                   for (size_t i = 0; i < pairs.size(); ++i) {
                     if (owner.at(pairs[i].first) != t) continue;
                     k1[i] = copy.getKthPaths(pairs[i].first, pairs[i].second, 1);
                     k2[i] = copy.getKthPaths(pairs[i].first, pairs[i].second, 2);
                   }
                 });
               }
               for (auto& w : ws) w.join();
             }
             py::list out;
             for (size_t i = 0; i < pairs.size(); ++i) {
               py::list a, b;
               for (const auto& p : k1[i]) a.append(pathToWire(p));
               for (const auto& p : k2[i]) b.append(pathToWire(p));
               out.append(py::make_tuple(a, b));
             }
             return out;
           },
           py::arg("pairs"), py::arg("threads"), py::arg("replay"))
      .def("time_spf_sources",
           [](const LinkState& s, std::vector<std::string> srcs, int threads) {
             // Timed all-sources SPF: one LinkState copy per thread (the memo is
             // not thread-safe, LinkState.h:279-301), no cross-source memo.
             py::gil_scoped_release rel;
             threads = std::max(1, threads);
             // deep copies (replayed adjacency databases): threads must not
             // share Link objects, whose shared_ptr refcounts runSpf bumps
             std::vector<LinkState> copies;
             copies.reserve(threads);
             for (int t = 0; t < threads; ++t) {
               copies.emplace_back(s.getArea());
               for (const auto& kv : s.getAdjacencyDatabases())
                 copies.back().updateAdjacencyDatabase(kv.second);
             }
             const auto t0 = std::chrono::steady_clock::now();
             std::vector<std::thread> ws;
             size_t checksum = 0;
             std::vector<size_t> sums(threads, 0);
             for (int t = 0; t < threads; ++t) {
               ws.emplace_back([&, t] {
                 for (size_t i = t; i < srcs.size(); i += threads) {
                   auto r = copies[t].runSpf(srcs[i], true);
                   sums[t] += r.size();
                 }
               });
             }
             for (auto& w : ws) w.join();
             const double sec =
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
             for (auto v : sums) checksum += v;
             return std::make_pair(sec, checksum);
           });

  // the independent fast checker (oracle_fast.h): parity at the configs'
  // full sizes, validated against the faithful LinkState above
  py::class_<FastChecker>(m, "FastChecker")
      .def(py::init<const LinkState&, const std::vector<std::string>&>(), py::arg("link_state"),
           py::arg("order"))
      .def_property_readonly("nodes", &FastChecker::nodes)
      .def_property_readonly("links", &FastChecker::links)
      .def("link_index", &FastChecker::linkIndex)
      .def("link_desc", &FastChecker::linkDesc)
      .def("neighbours", &FastChecker::neighbours)
      .def("spf_rows",  // dist [S][N] (u32, 0xFFFFFFFF absent) and first-hop masks [S][N][W]
           [](const FastChecker& f, std::vector<uint32_t> srcs, std::vector<std::vector<uint32_t>> ignores,
              int threads) {
             if (!ignores.empty() && ignores.size() != srcs.size())
               throw std::invalid_argument("spf_rows: one ignore list per source");
             const size_t S = srcs.size(), N = f.nodes();
             std::vector<FastChecker::Row> rows(S);
             {
               py::gil_scoped_release rel;
               parallelOver(S, threads, [&](size_t i) {
                 static const std::vector<uint32_t> none;
                 f.spf(srcs[i], ignores.empty() ? none : ignores[i], rows[i]);
               });
             }
             size_t W = 1;
             for (const auto& r : rows) W = std::max<size_t>(W, r.words);
             py::array_t<uint32_t> dist({S, N}), nh({S, N, W});
             uint32_t* pd = dist.mutable_data();
             uint32_t* pn = nh.mutable_data();
             std::fill(pn, pn + S * N * W, 0u);
             for (size_t i = 0; i < S; ++i)
               for (size_t v = 0; v < N; ++v) {
                 pd[i * N + v] = rows[i].dist[v] == ~0ull ? 0xFFFFFFFFu : static_cast<uint32_t>(rows[i].dist[v]);
                 for (uint32_t k = 0; k < rows[i].words; ++k)
                   pn[(i * N + v) * W + k] = rows[i].nh[v * rows[i].words + k];
               }
             return py::make_tuple(dist, nh);
           },
           py::arg("srcs"), py::arg("ignores") = std::vector<std::vector<uint32_t>>{}, py::arg("threads") = 8)
      .def("row_digests",  // orh_row_digest of each runSpf(srcs[i], true, ignores[i]) row
           [](const FastChecker& f, std::vector<uint32_t> srcs, std::vector<std::vector<uint32_t>> ignores,
              int threads) {
             if (!ignores.empty() && ignores.size() != srcs.size())
               throw std::invalid_argument("row_digests: one ignore list per source");
             py::array_t<uint64_t> out(srcs.size());
             uint64_t* po = out.mutable_data();
             {
               py::gil_scoped_release rel;
               parallelOver(srcs.size(), threads, [&](size_t i) {
                 static const std::vector<uint32_t> none;
                 FastChecker::Row r;
                 f.spf(srcs[i], ignores.empty() ? none : ignores[i], r);
                 po[i] = FastChecker::digest(r);
               });
             }
             return out;
           },
           py::arg("srcs"), py::arg("ignores") = std::vector<std::vector<uint32_t>>{}, py::arg("threads") = 8)
      .def("kth_paths",  // per pair (k = 1 paths, k = 2 paths), each path a list of link descriptors
           [](const FastChecker& f, std::vector<std::pair<uint32_t, uint32_t>> pairs, int threads) {
             std::vector<std::vector<std::vector<uint32_t>>> k1(pairs.size()), k2(pairs.size());
             {
               py::gil_scoped_release rel;
               parallelOver(pairs.size(), threads,
                            [&](size_t i) { f.kthPaths(pairs[i].first, pairs[i].second, k1[i], k2[i]); });
             }
             auto conv = [&](const std::vector<std::vector<uint32_t>>& ps) {
               py::list out;
               for (const auto& p : ps) {
                 py::list path;
                 for (uint32_t l : p) {
                   const auto& [a, ifa, b, ifb] = f.linkDesc(l);
                   path.append(py::make_tuple(a, ifa, b, ifb));
                 }
                 out.append(path);
               }
               return out;
             };
             py::list out;
             for (size_t i = 0; i < pairs.size(); ++i) out.append(py::make_tuple(conv(k1[i]), conv(k2[i])));
             return out;
           },
           py::arg("pairs"), py::arg("threads") = 8);

  m.def("path_a_in_path_b", [](std::vector<py::tuple> a, std::vector<py::tuple> b) {
    auto mk = [](const std::vector<py::tuple>& v) {
      Path p;
      for (auto& t : v)
        p.push_back(std::make_shared<Link>("a", t[0].cast<std::string>(), t[1].cast<std::string>(),
                                           t[2].cast<std::string>(), t[3].cast<std::string>()));
      return p;
    };
    return LinkState::pathAInPathB(mk(a), mk(b));
  });

  m.def("link_hash", [](const std::string& n1, const std::string& if1, const std::string& n2,
                        const std::string& if2) { return Link("a", n1, if1, n2, if2).hash; });

  m.def("unordered_int_order", [](std::vector<int> keys) {
    // iteration order of a libstdc++ std::unordered_map<int, ...> built by
    // inserting `keys` in order (the reference test helper's container,
    // DecisionTestUtils.cpp:18-43)
    std::unordered_map<int, int> mp;
    for (int k : keys) mp.emplace(k, 0);
    std::vector<int> order;
    for (auto& kv : mp) order.push_back(kv.first);
    return order;
  });

  py::class_<AreaMap>(m, "AreaLinkStates")
      .def(py::init<>())
      .def("add_area", [](AreaMap& a, const std::string& area) {
        a.m.emplace(area, LinkState(area));
      })
      .def("area", [](AreaMap& a, const std::string& area) -> LinkState& { return a.m.at(area); },
           py::return_value_policy::reference_internal)
      .def("areas", [](const AreaMap& a) {
        std::vector<std::string> v;
        for (auto& kv : a.m) v.push_back(kv.first);
        return v;
      });

  py::class_<PrefixState>(m, "PrefixState")
      .def(py::init<>())
      .def("update_prefix",
           [](PrefixState& s, const std::string& node, const std::string& area, py::tuple e) {
             py::list out;
             for (const auto& c : s.updatePrefix(node, area, entryFromWire(e)))
               out.append(py::make_tuple(py::bytes(c.first), c.second));
             return out;
           })
      .def("update_prefixes",  // [(node, area, entry)]: update_prefix in order, one call
           [](PrefixState& s, py::list items) {
             size_t n = 0;
             for (auto it : items) {
               auto t = it.cast<py::tuple>();
               n += s.updatePrefix(t[0].cast<std::string>(), t[1].cast<std::string>(),
                                   entryFromWire(t[2].cast<py::tuple>())).size();
             }
             return n;
           })
      .def("delete_prefix",
           [](PrefixState& s, const std::string& node, const std::string& area, py::bytes addr,
              int32_t len) {
             py::list out;
             for (const auto& c : s.deletePrefix(node, area, Cidr{std::string(addr), len}))
               out.append(py::make_tuple(py::bytes(c.first), c.second));
             return out;
           })
      .def("num_prefixes", [](const PrefixState& s) { return s.prefixes().size(); });

  py::class_<SpfSolver>(m, "SpfSolver")
      .def(py::init<const std::string&, bool, bool, bool, bool>(), py::arg("my_node"),
           py::arg("enable_v4"), py::arg("enable_ordered_fib") = false,
           py::arg("bgp_dry_run") = false, py::arg("enable_best_route_selection") = false)
      .def("build_route_db",
           [](SpfSolver& s, const std::string& me, const AreaMap& als,
              const PrefixState& ps) -> py::object {
             auto db = s.buildRouteDb(me, als.m, ps);
             if (!db) return py::none();
             return routeDbToWire(*db);
           })
      .def("build_route_db_digest",
           [](SpfSolver& s, const std::string& me, const AreaMap& als,
              const PrefixState& ps) -> py::object {
             std::optional<DecisionRouteDb> db;
             {
               py::gil_scoped_release rel;
               db = s.buildRouteDb(me, als.m, ps);
             }
             if (!db) return py::none();
             return routeDbDigest(*db);
           })
      .def("time_build_route_db",
           [](SpfSolver& s, const std::string& me, const AreaMap& als,
              const PrefixState& ps) {
             const auto t0 = std::chrono::steady_clock::now();
             auto db = s.buildRouteDb(me, als.m, ps);
             const double sec =
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
             size_t n = db ? db->unicastRoutes.size() + db->mplsRoutes.size() : 0;
             return std::make_pair(sec, n);
           })
      .def("create_route_for_prefix_or_get_static_route",
           [](SpfSolver& s, const std::string& me, const AreaMap& als,
              const PrefixState& ps, py::bytes addr, int32_t len) -> py::object {
             auto r = s.createRouteForPrefixOrGetStaticRoute(me, als.m, ps, Cidr{std::string(addr), len});
             if (!r) return py::none();
             return unicastToWire(*r);
           })
      .def("update_static_unicast_routes",
           [](SpfSolver& s, std::vector<py::tuple> upd, std::vector<py::tuple> del) {
             std::vector<std::pair<Cidr, std::vector<NextHopThrift>>> u;
             for (auto& t : upd) {
               std::vector<NextHopThrift> nhs;
               for (auto n : t[2].cast<py::list>()) nhs.push_back(nhFromWire(n.cast<py::tuple>()));
               u.push_back({Cidr{bytesOf(t[0]), t[1].cast<int32_t>()}, nhs});
             }
             std::vector<Cidr> d;
             for (auto& t : del) d.push_back(Cidr{bytesOf(t[0]), t[1].cast<int32_t>()});
             s.updateStaticUnicastRoutes(u, d);
           })
      .def("update_static_mpls_routes",
           [](SpfSolver& s, std::vector<py::tuple> upd, std::vector<int32_t> del) {
             std::vector<std::pair<int32_t, std::vector<NextHopThrift>>> u;
             for (auto& t : upd) {
               std::vector<NextHopThrift> nhs;
               for (auto n : t[1].cast<py::list>()) nhs.push_back(nhFromWire(n.cast<py::tuple>()));
               u.push_back({t[0].cast<int32_t>(), nhs});
             }
             s.updateStaticMplsRoutes(u, del);
           })
      // Decision::rebuildRoutes' full rebuild (Decision.cpp:1888-1900):
      // buildRouteDb, then RibPolicy::applyPolicy on its unicast routes
      .def("build_route_db_with_policy",
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              RibPolicy& policy) -> py::object {
             auto db = s.buildRouteDb(me, als.m, ps);
             if (!db) return py::none();
             policy.applyPolicy(db->unicastRoutes);
             return routeDbToWire(*db);
           })
      .def("build_route_db_with_policy_digest",
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              RibPolicy& policy) -> py::object {
             std::optional<DecisionRouteDb> db;
             {
               py::gil_scoped_release rel;
               db = s.buildRouteDb(me, als.m, ps);
               if (db) policy.applyPolicy(db->unicastRoutes);
             }
             if (!db) return py::none();
             return routeDbDigest(*db);
           })
      .def_property_readonly("route_build_runs", [](const SpfSolver& s) { return s.routeBuildRuns; });

  // RibPolicy (RibPolicy.cpp:19-247), the same Python surface as the
  // product's openr_amd._openr_host.RibPolicy
  py::class_<RibPolicy>(m, "RibPolicy")
      .def(py::init([](py::list statements, int64_t ttlSecs) {
             std::vector<RibPolicyStatementSpec> specs;
             for (auto st : statements) specs.push_back(statementFromWire(st.cast<py::tuple>()));
             try {
               return new RibPolicy(specs, ttlSecs);
             } catch (const std::invalid_argument& e) {
               throw py::value_error(e.what());
             }
           }),
           py::arg("statements"), py::arg("ttl_secs"))
      .def("is_active", &RibPolicy::isActive)
      .def("ttl_ms", [](const RibPolicy& p) { return p.getTtlDuration().count(); })
      .def("match", [](const RibPolicy& p, py::tuple r) { return p.match(unicastFromWire(r)); })
      .def("apply_action",
           [](RibPolicy& p, py::tuple r) {
             RibUnicastEntry e = unicastFromWire(r);
             const bool changed = p.applyAction(e);
             return py::make_tuple(changed, unicastToWire(e));
           })
      .def("apply_policy",  // (updated prefixes, deleted prefixes, transformed unicast routes)
           [](RibPolicy& p, py::list routes) {
             std::unordered_map<Cidr, RibUnicastEntry, CidrHash> m;
             for (auto r : routes) {
               RibUnicastEntry e = unicastFromWire(r.cast<py::tuple>());
               Cidr k = e.prefix;
               m.emplace(std::move(k), std::move(e));
             }
             auto ch = p.applyPolicy(m);
             py::list up, del, out;
             for (const auto& c : ch.updatedRoutes) up.append(py::make_tuple(py::bytes(c.first), c.second));
             for (const auto& c : ch.deletedRoutes) del.append(py::make_tuple(py::bytes(c.first), c.second));
             for (const auto& [_, e] : m) out.append(unicastToWire(e));
             return py::make_tuple(up, del, out);
           })
      .def_property_readonly("invalidated_routes", &RibPolicy::invalidatedRoutes);
  py::class_<StatementProbe>(m, "RibPolicyStatement")
      .def(py::init([](py::tuple st) {
        try {
          return new StatementProbe{RibPolicyStatement(statementFromWire(st))};
        } catch (const std::invalid_argument& e) {
          throw py::value_error(e.what());
        }
      }))
      .def("match", [](const StatementProbe& s, py::tuple r) { return s.st.match(unicastFromWire(r)); })
      .def("apply_action", [](StatementProbe& s, py::tuple r) {
        RibUnicastEntry e = unicastFromWire(r);
        const bool changed = s.st.applyAction(e, s.invalidated);
        return py::make_tuple(changed, unicastToWire(e));
      });
}
