// Python bindings of the drop-in Decision host library (module
// openr_amd._openr_host). The wire format (tuples) is shared with the test
// oracle so that openr_amd.facade can drive either one.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <limits>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <sys/resource.h>
#include <unistd.h>
#include <cstring>

#include "parallel.h"
#include "rib_policy.h"
#include "spf_solver.h"
#include "decision_ingest.h"
#include "multi_device.h"
#include "thrift_compact.h"

namespace py = pybind11;
using namespace openr_amd;

namespace {

py::bytes pyBytes(const AddrBytes& a) { return py::bytes(a.data(), a.size()); }

std::string str(const py::handle& h) { return h.cast<std::string>(); }

Adjacency adjFromWire(const py::tuple& t) {
  Adjacency a;
  a.otherNodeName = str(t[0]);
  a.ifName = str(t[1]);
  a.nextHopV6.addr = str(t[2]);
  a.nextHopV4.addr = str(t[3]);
  a.metric = t[4].cast<int32_t>();
  a.adjLabel = t[5].cast<int32_t>();
  a.isOverloaded = t[6].cast<bool>();
  a.rtt = t[7].cast<int32_t>();
  a.timestamp = t[8].cast<int64_t>();
  a.weight = t[9].cast<int64_t>();
  a.otherIfName = str(t[10]);
  return a;
}

AdjacencyDatabase adjDbFromWire(const py::tuple& t) {
  AdjacencyDatabase db;
  db.thisNodeName = str(t[0]);
  db.isOverloaded = t[1].cast<bool>();
  const auto adjs = t[2].cast<py::list>();
  db.adjacencies.reserve(adjs.size());
  for (auto a : adjs) db.adjacencies.push_back(adjFromWire(a.cast<py::tuple>()));
  db.nodeLabel = t[3].cast<int32_t>();
  db.area = str(t[4]);
  return db;
}

PrefixEntry entryFromWire(const py::tuple& t) {
  PrefixEntry e;
  e.addr = str(t[0]);
  e.len = t[1].cast<int32_t>();
  e.type = t[2].cast<int32_t>();
  e.forwardingType = t[3].cast<int32_t>();
  e.forwardingAlgorithm = t[4].cast<int32_t>();
  if (!t[5].is_none()) e.minNexthop = t[5].cast<int64_t>();
  if (!t[6].is_none()) e.prependLabel = t[6].cast<int32_t>();
  auto m = t[7].cast<py::tuple>();
  e.pathPreference = m[0].cast<int32_t>();
  e.sourcePreference = m[1].cast<int32_t>();
  e.distance = m[2].cast<int32_t>();
  if (!t[8].is_none()) {
    auto mvt = t[8].cast<py::tuple>();
    MetricVector mv;
    mv.version = mvt[0].cast<int64_t>();
    for (auto ent : mvt[1]) {
      auto et = ent.cast<py::tuple>();
      mv.metrics.push_back(MetricEntity{et[0].cast<int64_t>(), et[1].cast<int64_t>(),
                                        et[2].cast<int32_t>(), et[3].cast<bool>(),
                                        et[4].cast<std::vector<int64_t>>()});
    }
    e.mv = std::move(mv);
  }
  if (!t[9].is_none()) e.data = str(t[9]);
  if (t.size() > 10 && !t[10].is_none())
    for (auto tag : t[10]) e.tags.insert(tag.cast<std::string>());
  return e;
}

// entryFromWire over the CPython API for the bulk load (pybind's accessors
// and casts were most of its per-entry cost); false for what it does not
// take (metric vectors, out-of-range or unexpected values): entryFromWire then
bool strFast(PyObject* o, std::string& out) {
  const char* p;
  Py_ssize_t n;
  if (PyUnicode_Check(o)) {
    p = PyUnicode_AsUTF8AndSize(o, &n);
    if (!p) {
      PyErr_Clear();
      return false;
    }
  } else if (PyBytes_Check(o)) {
    p = PyBytes_AS_STRING(o);
    n = PyBytes_GET_SIZE(o);
  } else {
    return false;
  }
  out.assign(p, static_cast<size_t>(n));
  return true;
}

template <class T>
bool intFast(PyObject* o, T& out) {
  if (!PyLong_Check(o)) return false;
  int overflow = 0;
  const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
  if (overflow || (v == -1 && PyErr_Occurred()) || v < std::numeric_limits<T>::min() ||
      v > std::numeric_limits<T>::max()) {
    PyErr_Clear();
    return false;
  }
  out = static_cast<T>(v);
  return true;
}

bool entryFromWireFast(PyObject* t, PrefixEntry& e) {
  if (!PyTuple_Check(t) || PyTuple_GET_SIZE(t) < 10) return false;
  auto at = [t](Py_ssize_t i) { return PyTuple_GET_ITEM(t, i); };
  PyObject* a = at(0);
  if (!PyBytes_Check(a) || PyBytes_GET_SIZE(a) > static_cast<Py_ssize_t>(AddrBytes::kMax)) return false;
  e.addr.assign(PyBytes_AS_STRING(a), static_cast<size_t>(PyBytes_GET_SIZE(a)));
  if (!intFast(at(1), e.len) || !intFast(at(2), e.type) || !intFast(at(3), e.forwardingType) ||
      !intFast(at(4), e.forwardingAlgorithm))
    return false;
  if (at(5) != Py_None) {
    int64_t v;
    if (!intFast(at(5), v)) return false;
    e.minNexthop = v;
  }
  if (at(6) != Py_None) {
    int32_t v;
    if (!intFast(at(6), v)) return false;
    e.prependLabel = v;
  }
  PyObject* m = at(7);
  if (!PyTuple_Check(m) || PyTuple_GET_SIZE(m) < 3 || !intFast(PyTuple_GET_ITEM(m, 0), e.pathPreference) ||
      !intFast(PyTuple_GET_ITEM(m, 1), e.sourcePreference) || !intFast(PyTuple_GET_ITEM(m, 2), e.distance))
    return false;
  if (at(8) != Py_None) return false;  // metric vector: the pybind path
  if (at(9) != Py_None) {
    std::string d;
    if (!strFast(at(9), d)) return false;
    e.data = std::move(d);
  }
  if (PyTuple_GET_SIZE(t) > 10 && at(10) != Py_None) {
    PyObject* tags = at(10);
    if (!PyTuple_Check(tags) && !PyList_Check(tags)) return false;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(tags);
    for (Py_ssize_t i = 0; i < n; ++i) {
      std::string tag;
      if (!PyUnicode_Check(PySequence_Fast_GET_ITEM(tags, i)) || !strFast(PySequence_Fast_GET_ITEM(tags, i), tag))
        return false;
      e.tags.insert(std::move(tag));
    }
  }
  return true;
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
  return py::make_tuple(pyBytes(e.addr), e.len, e.type, e.forwardingType, e.forwardingAlgorithm,
                        py::cast(e.minNexthop), py::cast(e.prependLabel),
                        py::make_tuple(e.pathPreference, e.sourcePreference, e.distance), mv,
                        e.data ? py::object(py::bytes(*e.data)) : py::none(),
                        py::tuple(py::cast(std::vector<std::string>(e.tags.begin(), e.tags.end()))));
}

NextHopThrift nhFromWire(const py::tuple& t) {
  NextHopThrift nh;
  nh.address.addr = str(t[0]);
  if (!t[1].is_none()) nh.address.ifName = str(t[1]);
  nh.weight = t[2].cast<int32_t>();
  if (!t[3].is_none()) {
    auto a = t[3].cast<py::tuple>();
    MplsAction act;
    act.action = a[0].cast<int32_t>();
    if (!a[1].is_none()) act.swapLabel = a[1].cast<int32_t>();
    if (!a[2].is_none()) act.pushLabels = a[2].cast<std::vector<int32_t>>();
    nh.mplsAction = std::move(act);
  }
  nh.metric = t[4].cast<int32_t>();
  if (!t[5].is_none()) nh.area = str(t[5]);
  if (!t[6].is_none()) nh.neighborNodeName = str(t[6]);
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
  return py::make_tuple(pyBytes(nh.address.addr), py::cast(nh.address.ifName), nh.weight, act,
                        nh.metric, py::cast(nh.area), py::cast(nh.neighborNodeName));
}

py::list nhsToWire(const NextHopSet& s) {
  py::list l;
  for (const auto& nh : s) l.append(nhToWire(nh));
  return l;
}
py::list nhsToWire(const NextHops& s) { return nhsToWire(s.set()); }

py::tuple unicastToWire(const RibUnicastEntry& e) {
  return py::make_tuple(pyBytes(e.prefix.first), e.prefix.second, nhsToWire(e.nexthops),
                        e.doNotInstall, e.bestArea,
                        e.bestPrefixEntry ? entryToWire(*e.bestPrefixEntry) : py::none());
}

RibUnicastEntry unicastFromWire(const py::tuple& t) {
  RibUnicastEntry e;
  e.prefix = {str(t[0]), t[1].cast<int32_t>()};
  for (auto nh : t[2]) e.nexthops.insert(nhFromWire(nh.cast<py::tuple>()));
  e.doNotInstall = t[3].cast<bool>();
  e.bestArea = str(t[4]);
  if (!t[5].is_none()) e.bestPrefixEntry = entryFromWire(t[5].cast<py::tuple>());
  return e;
}

RibPolicyStatementSpec statementFromWire(const py::tuple& t) {
  // (name, prefixes | None, tags | None, (default, {area: w}, {nbr: w}) | None)
  RibPolicyStatementSpec s;
  s.name = str(t[0]);
  if (!t[1].is_none()) {
    s.prefixes.emplace();
    for (auto p : t[1]) {
      auto pt = p.cast<py::tuple>();
      s.prefixes->emplace_back(str(pt[0]), pt[1].cast<int32_t>());
    }
  }
  if (!t[2].is_none()) s.tags = t[2].cast<std::vector<std::string>>();
  if (!t[3].is_none()) {
    auto w = t[3].cast<py::tuple>();
    RibRouteActionWeight a;
    a.defaultWeight = w[0].cast<int32_t>();
    a.areaToWeight = w[1].cast<std::map<std::string, int32_t>>();
    a.neighborToWeight = w[2].cast<std::map<std::string, int32_t>>();
    s.setWeight = std::move(a);
  }
  return s;
}

py::tuple routeDbToWire(const DecisionRouteDb& db) {
  py::list uc, mp;
  for (const auto& [_, e] : db.unicastRoutes) uc.append(unicastToWire(e));
  for (const auto& [_, e] : db.mplsRoutes) mp.append(py::make_tuple(e.label, nhsToWire(e.nexthops)));
  return py::make_tuple(uc, mp);
}

DecisionRouteDb routeDbFromWire(const py::tuple& w) {
  DecisionRouteDb db;
  for (auto u : w[0]) {
    RibUnicastEntry e = unicastFromWire(u.cast<py::tuple>());
    auto key = e.prefix;
    db.unicastRoutes.emplace(std::move(key), std::move(e));
  }
  for (auto m : w[1]) {
    auto t = m.cast<py::tuple>();
    RibMplsEntry e;
    e.label = t[0].cast<int32_t>();
    for (auto nh : t[1]) e.nexthops.insert(nhFromWire(nh.cast<py::tuple>()));
    db.mplsRoutes.emplace(e.label, std::move(e));
  }
  return db;
}

// DecisionRouteUpdate as (unicast updates, unicast deletes (addr, len),
// mpls updates (label, nexthops), mpls deletes)
py::tuple deltaToWire(const DecisionRouteUpdate& d) {
  py::list uu, ud, mu;
  for (const auto& [_, e] : d.unicastRoutesToUpdate) uu.append(unicastToWire(e));
  for (const auto& p : d.unicastRoutesToDelete) ud.append(py::make_tuple(pyBytes(p.first), p.second));
  for (const auto& e : d.mplsRoutesToUpdate) mu.append(py::make_tuple(e.label, nhsToWire(e.nexthops)));
  return py::make_tuple(uu, ud, mu, py::cast(d.mplsRoutesToDelete));
}

DecisionRouteUpdate deltaFromWire(const py::tuple& w) {
  DecisionRouteUpdate d;
  for (auto u : w[0]) {
    RibUnicastEntry e = unicastFromWire(u.cast<py::tuple>());
    auto key = e.prefix;
    d.unicastRoutesToUpdate.emplace(std::move(key), std::move(e));
  }
  for (auto p : w[1]) {
    auto t = p.cast<py::tuple>();
    d.unicastRoutesToDelete.emplace_back(str(t[0]), t[1].cast<int32_t>());
  }
  for (auto m : w[2]) {
    auto t = m.cast<py::tuple>();
    RibMplsEntry e;
    e.label = t[0].cast<int32_t>();
    for (auto nh : t[1]) e.nexthops.insert(nhFromWire(nh.cast<py::tuple>()));
    d.mplsRoutesToUpdate.push_back(std::move(e));
  }
  d.mplsRoutesToDelete = w[3].cast<std::vector<int32_t>>();
  return d;
}

py::tuple changeToWire(const LinkStateChange& c) {
  return py::make_tuple(c.topologyChanged, c.linkAttributesChanged, c.nodeLabelChanged);
}

py::tuple linkDesc(const Link& l) { return py::make_tuple(l.on1, l.oif1, l.on2, l.oif2); }

std::optional<uint32_t> findLink(const LinkState& ls, const std::string& n1, const std::string& if1,
                                 const std::string& n2) {
  auto a = ls.nodeId(n1);
  if (!a) return std::nullopt;
  for (uint32_t lid : ls.linksFromNode(n1)) {
    const Link& l = ls.link(lid);
    if (l.ifFrom(*a) == if1 && ls.nodeName(l.other(*a)) == n2) return lid;
  }
  return std::nullopt;
}

py::dict rowToDict(const LinkState& ls, const SpfRow& row, bool withPaths) {
  py::dict d;
  if (!row.known) {
    d[py::str(row.srcName)] = py::make_tuple(0, py::list(), py::list());
    return d;
  }
  for (uint32_t v = 0; v < row.n; ++v) {
    if (!row.reachable(v)) continue;
    std::vector<std::string> nhs;
    row.forEachNextHop(v, [&](uint32_t nb) { nhs.push_back(ls.nodeName(nb)); });
    std::sort(nhs.begin(), nhs.end());
    py::list pls;
    if (withPaths) {
      for (const auto& [lid, prev] : ls.pathLinks(row, v))
        pls.append(py::make_tuple(linkDesc(ls.link(lid)), ls.nodeName(prev)));
    }
    d[py::str(ls.nodeName(v))] = py::make_tuple(static_cast<uint64_t>(row.metric(v)), nhs, pls);
  }
  return d;
}

py::tuple adjDbToWire(const AdjacencyDatabase& db) {
  py::list adjs;
  for (const auto& a : db.adjacencies)
    adjs.append(py::make_tuple(a.otherNodeName, a.ifName, pyBytes(a.nextHopV6.addr), pyBytes(a.nextHopV4.addr),
                               a.metric, a.adjLabel, a.isOverloaded, a.rtt, a.timestamp, a.weight,
                               a.otherIfName));
  return py::make_tuple(db.thisNodeName, db.isOverloaded, adjs, db.nodeLabel, db.area);
}

struct AreaMap {
  AreaLinkStates m;
  unsigned lane = 0;  // stream lane of every area's context (laneContext)
};

// all-sources sweep over a LinkState's device mirror (bench / parity tools):
// device-resident dist + first-hop rows for a fixed source list
class SpfSweep {
 public:
  SpfSweep(const LinkState& ls, const std::vector<std::string>& srcs, bool useLinkMetric,
           const std::vector<std::vector<uint32_t>>* ignore = nullptr, uint32_t minWords = 1)
      : ls_(ls), useLinkMetric_(useLinkMetric) {
    if (ignore) {
      if (ignore->size() != srcs.size())
        throw std::invalid_argument("SpfSweep: one ignore set per source");
      ignPtr_.push_back(0);
      for (const auto& set : *ignore) {
        ignLinks_.insert(ignLinks_.end(), set.begin(), set.end());
        ignPtr_.push_back(static_cast<uint32_t>(ignLinks_.size()));
      }
    }
    for (const auto& s : srcs) {
      auto id = ls.nodeId(s);
      if (!id) throw std::invalid_argument("SpfSweep: unknown source " + s);
      srcs_.push_back(*id);
    }
    graph_ = ls.deviceGraph();
    ctx_ = ls.context();
    uint32_t nn = 0, ne = 0;
    orh_graph_info(graph_, &nn, &ne);
    n_ = nn;
    edges_ = ne;
    if (orh_spf_words(graph_, srcs_.data(), static_cast<uint32_t>(srcs_.size()), &words_) != ORH_OK)
      throw std::runtime_error("orh_spf_words failed");
    words_ = std::max(words_, minWords);  // a shard padded to the whole batch's mask width
    const size_t nd = srcs_.size() * static_cast<size_t>(n_);
    if (orh_device_alloc(ctx_, nd * 4, reinterpret_cast<void**>(&dDist_)) != ORH_OK ||
        orh_device_alloc(ctx_, nd * 4 * words_, reinterpret_cast<void**>(&dNh_)) != ORH_OK)
      throw std::runtime_error("SpfSweep: device allocation failed");
  }
  ~SpfSweep() {
    orh_device_free(ctx_, dDist_);
    orh_device_free(ctx_, dNh_);
  }
  void run() {  // asynchronous
    orh_spf_request req{};
    req.h_srcs = srcs_.data();
    req.n_src = static_cast<uint32_t>(srcs_.size());
    req.use_link_metric = useLinkMetric_ ? 1 : 0;
    // a multi-source sweep's second phase on the context's second stream:
    // the next sweep on this context starts its search at once (sync(),
    // fetch() and copy_to() join it)
    req.flags = ORH_SPF_DEFER_HOPS;
    if (!ignPtr_.empty()) {
      req.h_ignore_ptr = ignPtr_.data();
      req.h_ignore_links = ignLinks_.empty() ? ignPtr_.data() : ignLinks_.data();
    }
    if (orh_spf_run(graph_, &req, words_, dDist_, dNh_) != ORH_OK)
      throw std::runtime_error(std::string("orh_spf_run: ") + orh_last_error(ctx_));
  }
  double lastMs() {
    double ms = 0;
    if (orh_last_spf_ms(ctx_, &ms) != ORH_OK) throw std::runtime_error("orh_last_spf_ms failed");
    return ms;
  }
  py::tuple phaseMs() {
    double a = 0, b = 0;
    if (orh_last_spf_phase_ms(ctx_, &a, &b) != ORH_OK)
      throw std::runtime_error("orh_last_spf_phase_ms failed");
    return py::make_tuple(a, b);
  }
  void sync() {
    if (orh_sync(ctx_) != ORH_OK) throw std::runtime_error(orh_last_error(ctx_));
  }
  py::dict info() const {  // kernel plan of the context's last run (orh_last_spf_info)
    orh_spf_info i{};
    orh_last_spf_info(ctx_, &i);
    py::dict d;
    d["variant"] = i.variant;
    d["rows"] = i.rows;
    d["mask_bits"] = i.mask_bits;
    d["batch_sources"] = i.batch_sources;
    d["hop_nodes"] = i.hop_nodes;
    d["hop_split"] = i.hop_split;
    d["ms_threads"] = i.ms_threads;
    d["ms_skip"] = i.ms_skip;
    d["ms_direct"] = i.ms_direct;
    return d;
  }
  py::tuple fetch(size_t i) {
    if (i >= srcs_.size()) throw std::out_of_range("SpfSweep.fetch");
    py::array_t<uint32_t> dist(n_), nh(static_cast<size_t>(n_) * words_);
    orh_memcpy_d2h(ctx_, dist.mutable_data(), dDist_ + i * n_, n_ * 4ull);
    orh_memcpy_d2h(ctx_, nh.mutable_data(), dNh_ + i * static_cast<size_t>(n_) * words_,
                   static_cast<size_t>(n_) * words_ * 4);
    return py::make_tuple(dist, nh);
  }
  // rows [0, sources) into caller-owned device buffers (e.g. torch tensors
  // feeding an RCCL all-gather): dist u32[S][N], nh u32[S][N][words]
  void copyTo(uintptr_t dDist, uintptr_t dNh) {
    const size_t nd = srcs_.size() * static_cast<size_t>(n_);
    if ((dDist && orh_memcpy_d2d(ctx_, reinterpret_cast<void*>(dDist), dDist_, nd * 4) != ORH_OK) ||
        (dNh && orh_memcpy_d2d(ctx_, reinterpret_cast<void*>(dNh), dNh_, nd * 4 * words_) != ORH_OK))
      throw std::runtime_error(std::string("SpfSweep.copy_to: ") + orh_last_error(ctx_));
  }
  uint32_t words() const { return words_; }
  uint32_t nodes() const { return n_; }
  uint32_t edges() const { return edges_; }
  size_t sources() const { return srcs_.size(); }

 private:
  const LinkState& ls_;
  bool useLinkMetric_;
  std::vector<uint32_t> srcs_;
  std::vector<uint32_t> ignPtr_, ignLinks_;  // per-source ignore sets (CSR), empty for none
  orh_graph* graph_{nullptr};
  orh_ctx* ctx_{nullptr};
  uint32_t n_{0}, edges_{0}, words_{1};
  uint32_t* dDist_{nullptr};
  uint32_t* dNh_{nullptr};
};

// ---- canonical route-db digest --------------------------------------------
// Per route: fields serialised in order (integers little-endian, strings and
// lists length-prefixed, optionals with a presence byte, nexthops sorted by
// their serialised bytes; PrefixEntry.tags, sorted, only when non-empty), hashed with
// FNV-1a 64. Routes in (prefix bytes, length) order, then labels. Lets a
// caller compare full-size route databases (C3, C5) without materialising
// them in Python.
class DigestWriter {
 public:
  std::string b;
  void raw(const void* p, size_t n) { b.append(static_cast<const char*>(p), n); }
  void u8(uint8_t v) { raw(&v, 1); }
  void i32(int32_t v) { raw(&v, 4); }
  void i64(int64_t v) { raw(&v, 8); }
  void str(const std::string& s) {
    i32(static_cast<int32_t>(s.size()));
    raw(s.data(), s.size());
  }
  void optStr(const std::optional<std::string>& o) {
    u8(o ? 1 : 0);
    if (o) str(*o);
  }
  void optI32(const std::optional<int32_t>& o) {
    u8(o ? 1 : 0);
    if (o) i32(*o);
  }
};

uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) {
    h ^= c;
    h *= 1099511628211ull;
  }
  return h;
}

std::string nexthopBytes(const NextHopThrift& nh) {
  DigestWriter w;
  w.str(nh.address.addr.str());
  w.optStr(nh.address.ifName);
  w.i32(nh.weight);
  w.u8(nh.mplsAction ? 1 : 0);
  if (nh.mplsAction) {
    w.i32(nh.mplsAction->action);
    w.optI32(nh.mplsAction->swapLabel);
    w.u8(nh.mplsAction->pushLabels ? 1 : 0);
    if (nh.mplsAction->pushLabels) {
      w.i32(static_cast<int32_t>(nh.mplsAction->pushLabels->size()));
      for (int32_t l : *nh.mplsAction->pushLabels) w.i32(l);
    }
  }
  w.i32(nh.metric);
  w.optStr(nh.area);
  w.optStr(nh.neighborNodeName);
  return w.b;
}

void writeNexthops(DigestWriter& w, const NextHopSet& nhs) {
  std::vector<std::string> v;
  v.reserve(nhs.size());
  for (const auto& nh : nhs) v.push_back(nexthopBytes(nh));
  std::sort(v.begin(), v.end());
  w.i32(static_cast<int32_t>(v.size()));
  for (const auto& x : v) w.str(x);
}
void writeNexthops(DigestWriter& w, const NextHops& nhs) { writeNexthops(w, nhs.set()); }

void writeEntry(DigestWriter& w, const PrefixEntry& e) {
  w.str(e.addr.str());
  w.i32(e.len);
  w.i32(e.type);
  w.i32(e.forwardingType);
  w.i32(e.forwardingAlgorithm);
  w.u8(e.minNexthop ? 1 : 0);
  if (e.minNexthop) w.i64(*e.minNexthop);
  w.optI32(e.prependLabel);
  w.i32(e.pathPreference);
  w.i32(e.sourcePreference);
  w.i32(e.distance);
  w.u8(e.mv ? 1 : 0);
  if (e.mv) {
    w.i64(e.mv->version);
    w.i32(static_cast<int32_t>(e.mv->metrics.size()));
    for (const auto& m : e.mv->metrics) {
      w.i64(m.type);
      w.i64(m.priority);
      w.i32(m.op);
      w.u8(m.isBestPathTieBreaker ? 1 : 0);
      w.i32(static_cast<int32_t>(m.metric.size()));
      for (int64_t x : m.metric) w.i64(x);
    }
  }
  w.optStr(e.data);
  if (!e.tags.empty()) {  // (absent for tag-free entries: older digests stand)
    w.i32(static_cast<int32_t>(e.tags.size()));
    for (const auto& t : e.tags) w.str(t);
  }
}

py::tuple routeDbDigest(const DecisionRouteDb& db) {
  std::vector<const RibUnicastEntry*> uc;
  uc.reserve(db.unicastRoutes.size());
  for (const auto& kv : db.unicastRoutes) uc.push_back(&kv.second);
  std::sort(uc.begin(), uc.end(),
            [](const RibUnicastEntry* a, const RibUnicastEntry* b) { return a->prefix < b->prefix; });
  std::vector<const RibMplsEntry*> mp;
  for (const auto& kv : db.mplsRoutes) mp.push_back(&kv.second);
  std::sort(mp.begin(), mp.end(),
            [](const RibMplsEntry* a, const RibMplsEntry* b) { return a->label < b->label; });
  std::string out(8 * (uc.size() + mp.size()), '\0');
  auto put = [&](size_t i, const std::string& bytes) {
    const uint64_t h = fnv1a(bytes);
    std::memcpy(&out[8 * i], &h, 8);
  };
  auto& pool = WorkerPool::instance();
  pool.parallelFor(uc.size(), [&](size_t, size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      DigestWriter w;
      w.str(uc[i]->prefix.first.str());
      w.i32(uc[i]->prefix.second);
      w.u8(uc[i]->doNotInstall ? 1 : 0);
      w.str(uc[i]->bestArea);
      w.u8(uc[i]->bestPrefixEntry ? 1 : 0);
      if (uc[i]->bestPrefixEntry) writeEntry(w, *uc[i]->bestPrefixEntry);
      writeNexthops(w, uc[i]->nexthops);
      put(i, w.b);
    }
  });
  for (size_t i = 0; i < mp.size(); ++i) {
    DigestWriter w;
    w.i32(mp[i]->label);
    writeNexthops(w, mp[i]->nexthops);
    put(uc.size() + i, w.b);
  }
  return py::make_tuple(uc.size(), mp.size(), py::bytes(out));
}

struct RibStatementProbe {  // a lone RibPolicyStatement (RibPolicyTest.cpp statement tests)
  RibPolicyStatement st;
};

}  // namespace

PYBIND11_MODULE(_openr_host, m) {
  m.doc() = "OpenR Decision SPF / route build on MI355X (host library over libopenr_hip)";

  py::class_<LinkState>(m, "LinkState")
      .def("update_adjacency_database",
           [](LinkState& s, py::tuple db, uint64_t up, uint64_t down) {
             return changeToWire(s.updateAdjacencyDatabase(adjDbFromWire(db), up, down));
           },
           py::arg("db"), py::arg("hold_up_ttl") = 0, py::arg("hold_down_ttl") = 0)
      .def("update_adjacency_databases",
           [](LinkState& s, py::list dbs) {
             py::list out;
             for (auto d : dbs) out.append(changeToWire(s.updateAdjacencyDatabase(adjDbFromWire(d.cast<py::tuple>()))));
             return out;
           })
      .def("delete_adjacency_database",
           [](LinkState& s, const std::string& n) { return changeToWire(s.deleteAdjacencyDatabase(n)); })
      .def("decrement_holds", [](LinkState& s) { return changeToWire(s.decrementHolds()); })
      .def("has_holds", &LinkState::hasHolds)
      .def("has_node", &LinkState::hasNode)
      .def("is_node_overloaded", &LinkState::isNodeOverloaded)
      .def("num_links", &LinkState::numLinks)
      .def("num_nodes", &LinkState::numNodes)
      .def_property_readonly("spf_runs", &LinkState::spfRuns)
      .def("links_from_node",
           [](const LinkState& s, const std::string& n) {
             py::list l;
             for (uint32_t lid : s.linksFromNode(n)) l.append(linkDesc(s.link(lid)));
             return l;
           })
      .def("get_spf_result",
           [](const LinkState& s, const std::string& n, bool useLinkMetric) {
             return rowToDict(s, s.getSpfRow(n, useLinkMetric), true);
           },
           py::arg("node"), py::arg("use_link_metric") = true)
      .def("get_spf_result_ref",  // the reference-shaped SpfResult (LinkState::getSpfResult)
           [](const LinkState& s, const std::string& n, bool useLinkMetric) {
             py::dict d;
             for (const auto& [name, r] : s.getSpfResult(n, useLinkMetric)) {
               std::vector<std::string> nhs(r.nextHops().begin(), r.nextHops().end());
               std::sort(nhs.begin(), nhs.end());
               py::list pls;
               for (const auto& pl : r.pathLinks())
                 pls.append(py::make_tuple(linkDesc(s.link(pl.link.id())), pl.prevNode));
               d[py::str(name)] = py::make_tuple(static_cast<uint64_t>(r.metric()), nhs, pls);
             }
             return d;
           },
           py::arg("node"), py::arg("use_link_metric") = true)
      .def("run_spf_ignoring",
           [](const LinkState& s, const std::string& src, std::vector<py::tuple> ignore) {
             std::vector<uint32_t> ign;
             for (auto& t : ignore) {
               if (auto lid = findLink(s, str(t[0]), str(t[1]), str(t[2]))) ign.push_back(*lid);
             }
             auto row = s.runSpf(src, true, ign);
             py::dict d;
             for (auto item : rowToDict(s, row, false)) {
               auto v = item.second.cast<py::tuple>();
               d[item.first] = py::make_tuple(v[0], v[1]);
             }
             return d;
           })
      .def("get_kth_paths",
           [](const LinkState& s, const std::string& a, const std::string& b, size_t k) {
             py::list out;
             for (const auto& p : s.getKthPathIds(a, b, k)) {
               py::list path;
               for (uint32_t lid : p) path.append(linkDesc(s.link(lid)));
               out.append(path);
             }
             return out;
           })
      .def("get_kth_path_ids",  // getKthPaths as LinkState link ids
           [](const LinkState& s, const std::string& a, const std::string& b, size_t k) {
             py::list out;
             for (const auto& p : s.getKthPathIds(a, b, k)) out.append(py::cast(p));
             return out;
           })
      .def("walk_kth_paths",  // the reference-typed getKthPaths (LinkRef handles) walked
                              // as selectBestPathsKsp2 does (Decision.cpp:1035-1076):
                              // per link from `src` (metric from the near end, near
                              // interface, far node, nhV6 from src on the first link)
           [](const LinkState& s, const std::string& a, const std::string& b, size_t k) {
             py::list out;
             for (const auto& path : s.getKthPaths(a, b, k)) {
               py::list hops;
               std::string cur = a;
               for (auto& link : path) {
                 hops.append(py::make_tuple(link->getMetricFromNode(cur), link->getIfaceFromNode(cur),
                                            link->getOtherNodeName(cur), link->getArea(), link->isUp()));
                 cur = link->getOtherNodeName(cur);
               }
               const auto& first = path.front();
               out.append(py::make_tuple(hops, pyBytes(first->getNhV6FromNode(a).addr),
                                         first->getIfaceFromNode(a)));
             }
             return out;
           })
      .def("mirror_stats", &LinkState::mirrorStats)
      .def("last_spf_info",  // kernel plan of the last SPF launch on this LinkState's context
           [](const LinkState& s) {
             orh_spf_info i{};
             orh_last_spf_info(s.context(), &i);
             py::dict d;
             d["variant"] = i.variant;
             d["rows"] = i.rows;
             d["batch_sources"] = i.batch_sources;
             return d;
           })
      .def("ksp2_abi",  // orh_ksp2 straight through the C ABI: per dst (k = 1 paths, k = 2 paths)
           [](const LinkState& s, const std::string& a, const std::vector<std::string>& dsts) {
             auto src = s.nodeId(a);
             if (!src) throw std::invalid_argument("ksp2_abi: unknown source " + a);
             std::vector<uint32_t> ids;
             for (const auto& d : dsts) {
               auto id = s.nodeId(d);
               if (!id) throw std::invalid_argument("ksp2_abi: unknown destination " + d);
               ids.push_back(*id);
             }
             orh_graph* g = s.deviceGraph();
             size_t need = 0;
             if (orh_ksp2(g, *src, ids.data(), static_cast<uint32_t>(ids.size()), nullptr, 0, &need) != ORH_OK)
               throw std::runtime_error(std::string("orh_ksp2: ") + orh_last_error(s.context()));
             std::vector<uint32_t> buf(need);
             if (orh_ksp2(g, *src, ids.data(), static_cast<uint32_t>(ids.size()), buf.data(), buf.size(),
                          &need) != ORH_OK)
               throw std::runtime_error(std::string("orh_ksp2: ") + orh_last_error(s.context()));
             py::list out;
             size_t w = 0;
             for (size_t i = 0; i < ids.size(); ++i) {
               py::list ks;
               for (int k = 0; k < 2; ++k) {
                 py::list paths;
                 const uint32_t np = buf[w++];
                 for (uint32_t p = 0; p < np; ++p) {
                   py::list path;
                   const uint32_t len = buf[w++];
                   for (uint32_t l = 0; l < len; ++l) path.append(linkDesc(s.link(buf[w++])));
                   paths.append(path);
                 }
                 ks.append(paths);
               }
               out.append(ks);
             }
             return out;
           })
      .def("get_metric_from_a_to_b", &LinkState::getMetricFromAToB, py::arg("a"), py::arg("b"),
           py::arg("use_link_metric") = true)
      .def("get_hops_from_a_to_b",
           [](const LinkState& s, const std::string& a, const std::string& b) {
             return s.getMetricFromAToB(a, b, false);
           })
      .def("get_max_hops_to_node", &LinkState::getMaxHopsToNode)
      .def("metric_from_node",
           [](const LinkState& s, const std::string& n1, const std::string& if1,
              const std::string& from) {
             auto a = s.nodeId(n1);
             auto f = s.nodeId(from);
             if (a && f) {
               for (uint32_t lid : s.linksFromNode(n1))
                 if (s.link(lid).ifFrom(*a) == if1) return s.link(lid).metricFrom(*f);
             }
             throw std::out_of_range("no such link");
           })
      .def("neighbors",  // distinct neighbours of src in first-hop bit order (orh_graph_neighbors)
           [](const LinkState& s, const std::string& src) {
             auto id = s.nodeId(src);
             if (!id) throw std::invalid_argument("neighbors: unknown node " + src);
             orh_graph* g = s.deviceGraph();
             uint32_t n = 0;
             orh_graph_neighbors(g, *id, nullptr, 0, &n);
             std::vector<uint32_t> ids(n);
             orh_graph_neighbors(g, *id, ids.data(), n, &n);
             std::vector<std::string> out;
             for (uint32_t v : ids) out.push_back(s.nodeName(v));
             return out;
           })
      .def("node_names",
           [](const LinkState& s) {
             std::vector<std::string> v;
             for (uint32_t i = 0; i < s.numNodeIds(); ++i) v.push_back(s.nodeName(i));
             return v;
           })
      .def("link_ids",
           [](const LinkState& s) {  // every link id, with its (n1, if1, n2, if2)
             py::list out;
             for (uint32_t lid = 0; lid < s.numLinkSlots(); ++lid)
               if (s.linkAlive(lid)) out.append(py::make_tuple(lid, linkDesc(s.link(lid))));
             return out;
           })
      .def("what_if_sweep",  // runSpf(src, true, {links}) for many (src, ignore set) pairs
           [](const LinkState& s, const std::vector<std::string>& srcs,
              const std::vector<std::vector<uint32_t>>& ignore) {
             return new SpfSweep(s, srcs, true, &ignore);
           },
           py::keep_alive<0, 1>())
      .def("what_if_batch",  // a what-if job over `srcs`: request i = (srcs[src_idx[i]], ignore[i])
           [](const LinkState& s, const std::vector<std::string>& srcs, const std::vector<uint32_t>& srcIdx,
              const std::vector<std::vector<uint32_t>>& ignore, uint32_t chunk, bool useLinkMetric,
              bool shareBase, bool searchLarge) {
             return new WhatIfBatch(s, srcs, srcIdx, ignore, chunk, useLinkMetric, shareBase, searchLarge);
           },
           py::arg("srcs"), py::arg("src_idx"), py::arg("ignore"), py::arg("chunk") = 4096,
           py::arg("use_link_metric") = true, py::arg("share_base") = false, py::arg("search_large") = false,
           py::return_value_policy::take_ownership, py::keep_alive<0, 1>())
      .def("run_spf_batch",
           [](const LinkState& s, const std::vector<std::string>& srcs,
              const std::vector<std::vector<uint32_t>>& ignore, bool useLinkMetric) {
             std::vector<uint32_t> ids;
             for (const auto& n : srcs) {
               auto id = s.nodeId(n);
               if (!id) throw std::invalid_argument("run_spf_batch: unknown source " + n);
               ids.push_back(*id);
             }
             py::list out;
             for (const auto& row : s.runSpfBatch(ids, useLinkMetric, ignore.empty() ? nullptr : &ignore)) {
               py::dict d;
               for (auto item : rowToDict(s, row, false)) {
                 auto v = item.second.cast<py::tuple>();
                 d[item.first] = py::make_tuple(v[0], v[1]);
               }
               out.append(d);
             }
             return out;
           },
           py::arg("srcs"), py::arg("ignore"), py::arg("use_link_metric") = true)
      .def("prefetch_spf_results", &LinkState::prefetchSpfResults, py::arg("nodes"),
           py::arg("use_link_metric") = true)
      .def("prefetch_kth_paths", &LinkState::prefetchKthPaths)
      .def("time_prefetch_kth_paths",  // wall seconds of each cold prefetchKthPaths call (memo dropped first)
           [](const LinkState& ls, const std::vector<std::pair<std::string, std::string>>& pairs, int reps) {
             std::vector<double> out;
             for (int r = 0; r < reps; ++r) {
               ls.dropMemo();
               const auto t0 = std::chrono::steady_clock::now();
               ls.prefetchKthPaths(pairs);
               out.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
             }
             return out;
           })
      .def("ksp_stats", [](const LinkState& s) {  // pairs traced on the device / host
        return py::make_tuple(s.kspDevicePairs_, s.kspHostPairs_);
      })
      .def("spf_words",  // first-hop mask words a batch over these sources needs
           [](const LinkState& s, const std::vector<std::string>& srcs) {
             std::vector<uint32_t> ids;
             for (const auto& n : srcs) {
               auto id = s.nodeId(n);
               if (!id) throw std::invalid_argument("spf_words: unknown source " + n);
               ids.push_back(*id);
             }
             uint32_t w = 1;
             if (orh_spf_words(s.deviceGraph(), ids.data(), static_cast<uint32_t>(ids.size()), &w) != ORH_OK)
               throw std::runtime_error(std::string("orh_spf_words: ") + orh_last_error(s.context()));
             return w;
           })
      .def("sweep", [](const LinkState& s, const std::vector<std::string>& srcs, bool useLinkMetric,
                       uint32_t minWords) {
             return new SpfSweep(s, srcs, useLinkMetric, nullptr, minWords);
           },
           py::arg("srcs"), py::arg("use_link_metric") = true, py::arg("min_words") = 1,
           py::return_value_policy::take_ownership, py::keep_alive<0, 1>());

  py::class_<SpfSweep>(m, "SpfSweep")
      .def("run", &SpfSweep::run)
      .def("last_ms", &SpfSweep::lastMs)
      .def("phase_ms", &SpfSweep::phaseMs)
      .def("sync", &SpfSweep::sync)
      .def("info", &SpfSweep::info)
      .def("fetch", &SpfSweep::fetch)
      .def("copy_to", &SpfSweep::copyTo, py::arg("dist_ptr"), py::arg("nh_ptr"))
      .def_property_readonly("words", &SpfSweep::words)
      .def_property_readonly("nodes", &SpfSweep::nodes)
      .def_property_readonly("edges", &SpfSweep::edges)
      .def_property_readonly("sources", &SpfSweep::sources);

  // one topology on several devices, the all-sources SPF split over them
  // (multi_device.h; SURVEY.md §8e inside the library, no torch)
  py::class_<ReplicatedLinkState>(m, "ReplicatedLinkState")
      .def(py::init<const std::string&, const std::vector<int>&>(), py::arg("area"), py::arg("devices"))
      .def("update_adjacency_database",
           [](ReplicatedLinkState& s, py::tuple db, uint64_t up, uint64_t down) {
             return changeToWire(s.updateAdjacencyDatabase(adjDbFromWire(db), up, down));
           },
           py::arg("db"), py::arg("hold_up_ttl") = 0, py::arg("hold_down_ttl") = 0)
      .def("delete_adjacency_database",
           [](ReplicatedLinkState& s, const std::string& n) { return changeToWire(s.deleteAdjacencyDatabase(n)); })
      .def("decrement_holds", [](ReplicatedLinkState& s) { return changeToWire(s.decrementHolds()); })
      .def_property_readonly("replicas", &ReplicatedLinkState::replicas)
      .def("replica", &ReplicatedLinkState::replica, py::return_value_policy::reference_internal)
      .def("sweep",
           [](const ReplicatedLinkState& s, const std::vector<std::string>& srcs, bool useLinkMetric) {
             return new MultiDeviceSweep(s, srcs, useLinkMetric);
           },
           py::arg("srcs"), py::arg("use_link_metric") = true, py::return_value_policy::take_ownership,
           py::keep_alive<0, 1>())
      .def("what_if_batch",
           [](const ReplicatedLinkState& s, const std::vector<std::string>& srcs, const std::vector<uint32_t>& srcIdx,
              const std::vector<std::vector<uint32_t>>& ignore, uint32_t chunk, bool useLinkMetric,
              bool shareBase) {
             return new MultiDeviceWhatIf(s, srcs, srcIdx, ignore, chunk, useLinkMetric, shareBase);
           },
           py::arg("srcs"), py::arg("src_idx"), py::arg("ignore"), py::arg("chunk") = 4096,
           py::arg("use_link_metric") = true, py::arg("share_base") = false,
           py::return_value_policy::take_ownership, py::keep_alive<0, 1>())
      .def("kth_paths_batch",
           [](const ReplicatedLinkState& s, const std::vector<std::pair<std::string, std::string>>& pairs) {
             return new MultiDeviceKthPaths(s, pairs);
           },
           py::arg("pairs"), py::return_value_policy::take_ownership, py::keep_alive<0, 1>());
  py::class_<MultiDeviceSweep>(m, "MultiDeviceSweep")
      .def("run", &MultiDeviceSweep::run)
      .def("run_block", &MultiDeviceSweep::runBlock, py::arg("block"))
      .def("sync", &MultiDeviceSweep::sync)
      .def("last_ms", &MultiDeviceSweep::lastMs, py::arg("block"))
      .def("block", &MultiDeviceSweep::block)
      .def_property_readonly("blocks", &MultiDeviceSweep::blocks)
      .def_property_readonly("sources", &MultiDeviceSweep::sources)
      .def_property_readonly("nodes", &MultiDeviceSweep::nodes)
      .def_property_readonly("words", &MultiDeviceSweep::words)
      .def("fetch",
           [](const MultiDeviceSweep& s, size_t i) {
             py::array_t<uint32_t> dist(s.nodes()), nh(static_cast<size_t>(s.nodes()) * s.words());
             s.fetch(i, dist.mutable_data(), nh.mutable_data());
             return py::make_tuple(dist, nh);
           })
      .def("gather", [](const MultiDeviceSweep& s) {
        py::array_t<uint32_t> dist({s.sources(), static_cast<size_t>(s.nodes())});
        py::array_t<uint32_t> nh({s.sources(), static_cast<size_t>(s.nodes()) * s.words()});
        s.gather(dist.mutable_data(), nh.mutable_data());
        return py::make_tuple(dist, nh);
      });

  // every area on several devices, the route build sharded over them by
  // prefix (multi_device.h)
  py::class_<ReplicatedAreaLinkStates>(m, "ReplicatedAreaLinkStates")
      .def(py::init<const std::vector<int>&>(), py::arg("devices"))
      .def("update_adjacency_database",
           [](ReplicatedAreaLinkStates& s, py::tuple db, uint64_t up, uint64_t down) {
             return changeToWire(s.updateAdjacencyDatabase(adjDbFromWire(db), up, down));
           },
           py::arg("db"), py::arg("hold_up_ttl") = 0, py::arg("hold_down_ttl") = 0)
      .def("delete_adjacency_database",
           [](ReplicatedAreaLinkStates& s, const std::string& area, const std::string& n) {
             return changeToWire(s.deleteAdjacencyDatabase(area, n));
           })
      .def_property_readonly("replicas", &ReplicatedAreaLinkStates::replicas)
      .def("route_builder",
           [](const ReplicatedAreaLinkStates& s, const std::string& me, bool v4, bool orderedFib, bool bgpDryRun,
              bool bestRoute) { return new ShardedRouteBuilder(s, me, v4, orderedFib, bgpDryRun, bestRoute); },
           py::arg("my_node"), py::arg("enable_v4"), py::arg("enable_ordered_fib") = false,
           py::arg("bgp_dry_run") = false, py::arg("enable_best_route_selection") = false,
           py::return_value_policy::take_ownership, py::keep_alive<0, 1>());
  py::class_<ShardedRouteBuilder>(m, "ShardedRouteBuilder")
      .def_property_readonly("shards", &ShardedRouteBuilder::shards)
      .def("build_route_db_digest",
           [](ShardedRouteBuilder& b, const std::string& me, const PrefixState& ps) -> py::object {
             auto db = b.buildRouteDb(me, ps);
             if (!db) return py::none();
             return routeDbDigest(*db);
           })
      .def("build_route_db",
           [](ShardedRouteBuilder& b, const std::string& me, const PrefixState& ps) -> py::object {
             auto db = b.buildRouteDb(me, ps);
             if (!db) return py::none();
             return routeDbToWire(*db);
           })
      .def("time_build_route_db",  // (seconds, routes, per-shard ms, merge ms)
           [](ShardedRouteBuilder& b, const std::string& me, const PrefixState& ps) {
             double sec = 0;
             size_t n = 0;
             {
               py::gil_scoped_release nogil;
               const auto t0 = std::chrono::steady_clock::now();
               auto db = b.buildRouteDb(me, ps);
               sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
               n = db ? db->unicastRoutes.size() + db->mplsRoutes.size() : 0;
             }
             std::vector<double> shardMs;
             for (size_t r = 0; r < b.shards(); ++r) shardMs.push_back(b.lastShardMs(r));
             return py::make_tuple(sec, n, shardMs, b.lastMergeMs());
           })
      .def("release_prefix_mirrors", &ShardedRouteBuilder::releasePrefixMirrors, py::arg("prefix_state"))
      .def("time_build_shard",  // shard r alone: (seconds, routes)
           [](ShardedRouteBuilder& b, size_t r, const std::string& me, const PrefixState& ps) {
             py::gil_scoped_release nogil;
             const auto t0 = std::chrono::steady_clock::now();
             auto db = b.buildShard(r, me, ps);
             const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
             const size_t n = db ? db->unicastRoutes.size() + db->mplsRoutes.size() : 0;
             return std::make_pair(sec, n);
           });

  // batched link-failure what-if SPFs (whatif_batch.h)
  py::class_<WhatIfBatch>(m, "WhatIfBatch")
      .def("run", &WhatIfBatch::run)
      .def("last_ms", &WhatIfBatch::lastMs)
      .def("sync", &WhatIfBatch::sync)
      .def("release", &WhatIfBatch::release)
      .def("set_digests", &WhatIfBatch::setDigests, py::arg("on") = true)
      .def("info",
           [](const WhatIfBatch& b) {
             py::array_t<uint32_t> out(b.requests());
             b.info(out.mutable_data());
             return out;
           })
      .def("digests",
           [](const WhatIfBatch& b) {
             py::array_t<uint64_t> out(b.requests());
             b.digests(out.mutable_data());
             return out;
           })
      .def("fetch",
           [](const WhatIfBatch& b, size_t i) {
             py::array_t<uint32_t> dist(b.nodes()), nh(b.nodes());
             b.fetch(i, dist.mutable_data(), nh.mutable_data());
             return py::make_tuple(dist, nh);
           })
      .def_property_readonly("requests", &WhatIfBatch::requests)
      .def_property_readonly("chunk", &WhatIfBatch::chunk)
      .def_property_readonly("nodes", &WhatIfBatch::nodes)
      .def_property_readonly("edges", &WhatIfBatch::edges);

  // a what-if job / KSP2 batch split over devices by source (multi_device.h)
  py::class_<MultiDeviceWhatIf>(m, "MultiDeviceWhatIf")
      .def("run", &MultiDeviceWhatIf::run, py::call_guard<py::gil_scoped_release>())
      .def("run_block", &MultiDeviceWhatIf::runBlock, py::arg("block"))
      .def("sync", &MultiDeviceWhatIf::sync)
      .def("release", &MultiDeviceWhatIf::release, py::arg("block"))
      .def("set_digests", &MultiDeviceWhatIf::setDigests, py::arg("on") = true)
      .def("last_ms", &MultiDeviceWhatIf::lastMs, py::arg("block"))
      .def("source_block", &MultiDeviceWhatIf::sourceBlock)
      .def("block_requests", &MultiDeviceWhatIf::blockRequests)
      .def_property_readonly("blocks", &MultiDeviceWhatIf::blocks)
      .def_property_readonly("requests", &MultiDeviceWhatIf::requests)
      .def("info",
           [](const MultiDeviceWhatIf& b) {
             py::array_t<uint32_t> out(b.requests());
             b.info(out.mutable_data());
             return out;
           })
      .def("digests", [](const MultiDeviceWhatIf& b) {
        py::array_t<uint64_t> out(b.requests());
        b.digests(out.mutable_data());
        return out;
      });
  py::class_<MultiDeviceKthPaths>(m, "MultiDeviceKthPaths")
      .def("run", &MultiDeviceKthPaths::run, py::call_guard<py::gil_scoped_release>())
      .def("run_block", &MultiDeviceKthPaths::runBlock, py::arg("block"))
      .def("last_ms", &MultiDeviceKthPaths::lastMs, py::arg("block"))
      .def("block_pairs", &MultiDeviceKthPaths::blockPairs)
      .def_property_readonly("blocks", &MultiDeviceKthPaths::blocks)
      .def_property_readonly("pairs", &MultiDeviceKthPaths::pairs)
      .def_property_readonly("device_pairs", &MultiDeviceKthPaths::devicePairs)
      .def("paths", [](const MultiDeviceKthPaths& b, size_t i, size_t k) {
        py::list out;
        for (const auto& p : b.paths(i, k)) out.append(py::cast(p));
        return out;
      });

  // DecisionRouteDb::calculateUpdate / update (Decision.cpp:108-160)
  // the bulk ingest's parser against the general one (tests): (whether the
  // CPython-API path took the entry, the entry as each path reads it)
  m.def("parse_prefix_entry", [](py::tuple t) {
    PrefixEntry fast;
    const bool ok = entryFromWireFast(t.ptr(), fast);
    return py::make_tuple(ok, ok ? entryToWire(fast) : py::none(), entryToWire(entryFromWire(t)));
  });
  m.def("host_threads", [] { return WorkerPool::instance().size(); },
        "threads of the host worker pool (the caller included)");
  // ---- thrift Compact wire -----------------------
  m.def("route_db_thrift", [](py::tuple db, const std::string& node) {  // DecisionRouteDb::toThrift
    return py::bytes(compact::routeDatabase(routeDbFromWire(db), node));
  });
  m.def("route_delta_thrift", [](py::tuple old_db, py::tuple new_db) {  // calculateUpdate -> toThrift
    return py::bytes(compact::routeDatabaseDelta(routeDbFromWire(old_db).calculateUpdate(routeDbFromWire(new_db))));
  });
  m.def("adj_db_to_compact", [](py::tuple db) { return py::bytes(compact::adjacencyDatabaseBytes(adjDbFromWire(db))); });
  m.def("adj_db_from_compact", [](py::bytes b) { return adjDbToWire(compact::adjacencyDatabase(std::string(b))); });
  m.def("prefix_db_to_compact",
        [](const std::string& node, const std::string& area, std::vector<py::tuple> entries, bool del,
           std::vector<std::vector<std::string>> areaStacks) {
          compact::PrefixDatabase db;
          db.thisNodeName = node;
          db.area = area;
          db.deletePrefix = del;
          for (auto& e : entries) db.prefixEntries.push_back(entryFromWire(e));
          db.areaStacks = std::move(areaStacks);
          return py::bytes(compact::prefixDatabaseBytes(db));
        },
        py::arg("node"), py::arg("area"), py::arg("entries"), py::arg("delete_prefix") = false,
        py::arg("area_stacks") = std::vector<std::vector<std::string>>{});
  m.def("prefix_db_from_compact", [](py::bytes b) {
    const auto db = compact::prefixDatabase(std::string(b));
    py::list entries;
    for (const auto& e : db.prefixEntries) entries.append(entryToWire(e));
    return py::make_tuple(db.thisNodeName, db.area, entries, db.deletePrefix, db.areaStacks);
  });
  // publication: {key: (version, originatorId, value bytes | None, ttl, ttlVersion)}
  m.def("publication_to_compact", [](const std::string& area, py::dict keyVals, std::vector<std::string> expired) {
    Publication p;
    p.area = area;
    p.expiredKeys = std::move(expired);
    for (auto kv : keyVals) {
      auto t = kv.second.cast<py::tuple>();
      KvValue v;
      v.version = t[0].cast<int64_t>();
      v.originatorId = str(t[1]);
      if (!t[2].is_none()) v.value = std::string(t[2].cast<py::bytes>());
      v.ttl = t[3].cast<int64_t>();
      v.ttlVersion = t[4].cast<int64_t>();
      p.keyVals[str(kv.first)] = std::move(v);
    }
    return py::bytes(publicationToCompact(p));
  });
  // (area, {key: (version, originatorId, value bytes | None, ttl, ttlVersion)}, expiredKeys)
  m.def("publication_from_compact", [](py::bytes b) {
    const Publication p = publicationFromCompact(std::string(b));
    py::dict kv;
    for (const auto& [k, v] : p.keyVals)
      kv[py::str(k)] = py::make_tuple(v.version, v.originatorId,
                                      v.value ? py::object(py::bytes(*v.value)) : py::object(py::none()),
                                      v.ttl, v.ttlVersion);
    return py::make_tuple(p.area, kv, p.expiredKeys);
  });
  m.def("parse_prefix_key", [](const std::string& key) -> py::object {  // PrefixKey::fromStr
    auto k = parsePrefixKey(key);
    if (!k) return py::none();
    return py::make_tuple(k->node, k->area, pyBytes(k->prefix.first), k->prefix.second);
  });

  m.def("calculate_update", [](py::tuple old_db, py::tuple new_db) {
    return deltaToWire(routeDbFromWire(old_db).calculateUpdate(routeDbFromWire(new_db)));
  });
  m.def("apply_update", [](py::tuple db, py::tuple delta) {
    DecisionRouteDb d = routeDbFromWire(db);
    d.update(deltaFromWire(delta));
    return routeDbToWire(d);
  });
  m.def("path_a_in_path_b", [](std::vector<py::tuple>, std::vector<py::tuple>) -> bool {
    throw std::runtime_error("path_a_in_path_b: use LinkState paths (ids are per LinkState)");
  });

  py::class_<AreaMap>(m, "AreaLinkStates")
      .def(py::init([](unsigned lane) {
             laneContext(lane);  // validate (and create) before any area uses it
             auto* a = new AreaMap();
             a->lane = lane;
             return a;
           }),
           py::arg("lane") = 0u)
      .def("add_area",
           [](AreaMap& a, const std::string& area) {
             a.m.emplace(std::piecewise_construct, std::forward_as_tuple(area),
                         std::forward_as_tuple(area, laneContext(a.lane)));
           })
      .def("area", [](AreaMap& a, const std::string& area) -> LinkState& { return a.m.at(area); },
           py::return_value_policy::reference_internal)
      .def("areas", [](const AreaMap& a) {
        std::vector<std::string> v;
        for (const auto& kv : a.m) v.push_back(kv.first);
        return v;
      });

  // Decision::processPublication state: pending updates, fib times, counters
  struct Ingest {
    std::string me;
    bool orderedFib;
    DecisionPendingUpdates pending;
    std::unordered_map<std::string, int64_t> fibTimes;
    IngestStats stats;
    Ingest(const std::string& n, bool o) : me(n), orderedFib(o), pending(n) {}
  };
  py::class_<Ingest>(m, "DecisionIngest")
      .def(py::init<const std::string&, bool>(), py::arg("my_node"), py::arg("ordered_fib") = false)
      .def("process_publication",  // thrift::Publication in Compact bytes
           [](Ingest& g, py::bytes pub, AreaMap& als, PrefixState& ps) {
             processPublication(publicationFromCompact(std::string(pub)), g.me, g.orderedFib, als.m, ps,
                                g.pending, g.fibTimes, g.stats, als.lane);
           })
      .def("pending", [](const Ingest& g) {
        py::list pfx;
        for (const auto& c : g.pending.updatedPrefixes()) pfx.append(py::make_tuple(pyBytes(c.first), c.second));
        py::dict d;
        d["needs_full_rebuild"] = g.pending.needsFullRebuild();
        d["needs_route_update"] = g.pending.needsRouteUpdate();
        d["updated_prefixes"] = pfx;
        d["count"] = g.pending.count();
        return d;
      })
      .def("reset", [](Ingest& g) { g.pending.reset(); })
      .def("fib_times", [](const Ingest& g) { return g.fibTimes; })
      .def("stats", [](const Ingest& g) {
        py::dict d;
        d["adj_db_update"] = g.stats.adjDbUpdates;
        d["prefix_db_update"] = g.stats.prefixDbUpdates;
        d["error"] = g.stats.errors;
        d["ttl_refresh"] = g.stats.ttlRefreshes;
        return d;
      });

  // Decision::routeDb_ + rebuildRoutes (Decision.cpp:1865-1930); returns
  // (delta wire, seconds)
  py::class_<DecisionRib>(m, "DecisionRib")
      .def(py::init<>())
      .def("rebuild_routes",
           [](DecisionRib& r, SpfSolver& solver, const std::string& me, const AreaMap& als,
              const PrefixState& ps, bool full, std::vector<py::tuple> prefixes, RibPolicy* policy,
              bool wire) {
             std::vector<Cidr> pfx;
             pfx.reserve(prefixes.size());
             for (auto& t : prefixes) pfx.emplace_back(AddrBytes(str(t[0])), t[1].cast<int32_t>());
             const auto t0 = std::chrono::steady_clock::now();
             py::object out;
             {
               auto u = r.rebuildRoutes(solver, me, als.m, ps, full, pfx, policy);
               if (wire) {
                 out = deltaToWire(u);
               } else {  // sizes only: (unicast updated, deleted, mpls updated, deleted)
                 out = py::make_tuple(u.unicastRoutesToUpdate.size(), u.unicastRoutesToDelete.size(),
                                      u.mplsRoutesToUpdate.size(), u.mplsRoutesToDelete.size());
               }
             }  // the delta is freed inside the timed call, as Decision's would be
             const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
             return py::make_tuple(out, sec);
           },
           py::arg("solver"), py::arg("me"), py::arg("als"), py::arg("ps"), py::arg("full"),
           py::arg("prefixes"), py::arg("policy") = nullptr, py::arg("wire") = true)
      .def("rebuild_routes_thrift",  // the same; the update as thrift::RouteDatabaseDelta bytes
           [](DecisionRib& r, SpfSolver& solver, const std::string& me, const AreaMap& als,
              const PrefixState& ps, bool full, std::vector<py::tuple> prefixes, RibPolicy* policy) {
             std::vector<Cidr> pfx;
             pfx.reserve(prefixes.size());
             for (auto& t : prefixes) pfx.emplace_back(AddrBytes(str(t[0])), t[1].cast<int32_t>());
             return py::bytes(compact::routeDatabaseDelta(r.rebuildRoutes(solver, me, als.m, ps, full, pfx, policy)));
           },
           py::arg("solver"), py::arg("me"), py::arg("als"), py::arg("ps"), py::arg("full"),
           py::arg("prefixes"), py::arg("policy") = nullptr)
      .def("route_db_thrift",  // routeDb_ as thrift::RouteDatabase bytes
           [](const DecisionRib& r, const std::string& me) {
             return py::bytes(compact::routeDatabase(r.routeDb(), me));
           })
      .def_property_readonly("delta_rebuilds", &DecisionRib::deltaRebuilds)
      .def_property_readonly("whole_rebuilds", &DecisionRib::wholeRebuilds)
      .def("rebuild_routes_pending",  // from a DecisionIngest's pending updates (then reset)
           [](DecisionRib& r, SpfSolver& solver, const std::string& me, const AreaMap& als,
              const PrefixState& ps, Ingest& g, RibPolicy* policy) {
             return deltaToWire(r.rebuildRoutes(solver, me, als.m, ps, g.pending, policy));
           },
           py::arg("solver"), py::arg("me"), py::arg("als"), py::arg("ps"), py::arg("ingest"),
           py::arg("policy") = nullptr)
      .def("route_db", [](const DecisionRib& r) { return routeDbToWire(r.routeDb()); });

  py::class_<PrefixState>(m, "PrefixState")
      .def(py::init<>())
      .def("update_prefix",
           [](PrefixState& s, const std::string& node, const std::string& area, py::tuple e) {
             py::list out;
             for (const auto& c : s.updatePrefix(node, area, entryFromWire(e)))
               out.append(py::make_tuple(pyBytes(c.first), c.second));
             return out;
           })
      .def("update_prefixes",  // [(node, area, entry wire)]: changed prefixes counted
           [](PrefixState& s, py::list items) {
             s.reserve(items.size());
             size_t n = 0;
             std::string node, area;
             for (auto it : items) {
               PyObject* t = it.ptr();
               PrefixEntry e;
               if (!(PyTuple_Check(t) && PyTuple_GET_SIZE(t) == 3 && strFast(PyTuple_GET_ITEM(t, 0), node) &&
                     strFast(PyTuple_GET_ITEM(t, 1), area) && entryFromWireFast(PyTuple_GET_ITEM(t, 2), e))) {
                 auto tt = it.cast<py::tuple>();
                 node = str(tt[0]);
                 area = str(tt[1]);
                 e = entryFromWire(tt[2].cast<py::tuple>());
               }
               n += s.upsertPrefix(node, area, std::move(e));
             }
             return n;
           })
      .def("set_tag_set_id_limit", &PrefixState::setTagSetIdLimit)
      .def_property_readonly("num_tag_sets", &PrefixState::numTagSets)
      .def("delete_prefix",
           [](PrefixState& s, const std::string& node, const std::string& area, py::bytes addr,
              int32_t len) {
             py::list out;
             for (const auto& c : s.deletePrefix(node, area, Cidr{std::string(addr), len}))
               out.append(py::make_tuple(pyBytes(c.first), c.second));
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
      .def("build_route_db_thrift",  // thrift::RouteDatabase in Compact bytes (canonical order)
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps) -> py::object {
             auto db = s.buildRouteDb(me, als.m, ps);
             if (!db) return py::none();
             return py::bytes(compact::routeDatabase(*db, me));
           })
      .def("build_route_db_digest",
           [](SpfSolver& s, const std::string& me, const AreaMap& als,
              const PrefixState& ps) -> py::object {
             auto db = s.buildRouteDb(me, als.m, ps);
             if (!db) return py::none();
             return routeDbDigest(*db);
           })
      .def("time_build_route_db",
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps) {
             const auto t0 = std::chrono::steady_clock::now();
             auto db = s.buildRouteDb(me, als.m, ps);
             const double sec =
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
             const size_t n = db ? db->unicastRoutes.size() + db->mplsRoutes.size() : 0;
             return std::make_pair(sec, n);
           })
      .def("time_build_route_db_phases",  // (seconds, routes, [(phase, ms)], minor faults, major faults, RSS delta bytes)
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps) {
             auto rss = [] {
               long pages = 0, resident = 0;
               if (FILE* f = std::fopen("/proc/self/statm", "r")) {
                 if (std::fscanf(f, "%ld %ld", &pages, &resident) != 2) resident = 0;
                 std::fclose(f);
               }
               return static_cast<int64_t>(resident) * sysconf(_SC_PAGESIZE);
             };
             RoutePhaseCapture cap;
             struct rusage r0{}, r1{};
             const int64_t m0 = rss();
             getrusage(RUSAGE_SELF, &r0);
             const auto t0 = std::chrono::steady_clock::now();
             auto db = s.buildRouteDb(me, als.m, ps);
             const double sec =
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
             getrusage(RUSAGE_SELF, &r1);
             const int64_t m1 = rss();
             const size_t n = db ? db->unicastRoutes.size() + db->mplsRoutes.size() : 0;
             py::list ph;
             for (const auto& [name, ms] : cap.phases) ph.append(py::make_tuple(std::string(name), ms));
             return py::make_tuple(sec, n, ph, static_cast<int64_t>(r1.ru_minflt - r0.ru_minflt),
                                   static_cast<int64_t>(r1.ru_majflt - r0.ru_majflt), m1 - m0);
           })
      .def("time_build_route_db_with_policy",  // Decision::rebuildRoutes: build + RibPolicy
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              RibPolicy& policy) {
             // (seconds, routes, updated, invalidated, routes decided on the
             // device, device policy ms)
             SpfSolver::PolicyStats st;
             const auto t0 = std::chrono::steady_clock::now();
             auto db = s.buildRouteDbWithPolicy(me, als.m, ps, &policy, &st);
             const auto t1 = std::chrono::steady_clock::now();
             return py::make_tuple(std::chrono::duration<double>(t1 - t0).count(),
                                   db ? db->unicastRoutes.size() : 0, st.updated, st.invalidated,
                                   st.onDevice, st.deviceMs);
           })
      .def("time_host_apply_policy",  // A/B: buildRouteDb, then applyPolicy over the map on the host
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              RibPolicy& policy) {
             auto db = s.buildRouteDb(me, als.m, ps);
             const auto t0 = std::chrono::steady_clock::now();
             size_t updated = 0;
             if (db) updated = policy.applyPolicy(db->unicastRoutes).updatedRoutes.size();
             const auto t1 = std::chrono::steady_clock::now();
             return py::make_tuple(std::chrono::duration<double>(t1 - t0).count(), updated);
           })
      .def("build_route_db_with_policy",
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              RibPolicy& policy) -> py::object {
             auto db = s.buildRouteDbWithPolicy(me, als.m, ps, &policy);
             if (!db) return py::none();
             return routeDbToWire(*db);
           })
      .def("build_route_db_with_policy_digest",
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              RibPolicy& policy) -> py::object {
             auto db = s.buildRouteDbWithPolicy(me, als.m, ps, &policy);
             if (!db) return py::none();
             return routeDbDigest(*db);
           })
      .def("create_route_for_prefix_or_get_static_route",
           [](SpfSolver& s, const std::string& me, const AreaMap& als, const PrefixState& ps,
              py::bytes addr, int32_t len) -> py::object {
             auto r = s.createRouteForPrefixOrGetStaticRoute(me, als.m, ps,
                                                             Cidr{std::string(addr), len});
             if (!r) return py::none();
             return unicastToWire(*r);
           })
      .def("update_static_unicast_routes",
           [](SpfSolver& s, std::vector<py::tuple> upd, std::vector<py::tuple> del) {
             std::vector<std::pair<Cidr, std::vector<NextHopThrift>>> u;
             for (auto& t : upd) {
               std::vector<NextHopThrift> nhs;
               for (auto n : t[2].cast<py::list>()) nhs.push_back(nhFromWire(n.cast<py::tuple>()));
               u.push_back({Cidr{str(t[0]), t[1].cast<int32_t>()}, nhs});
             }
             std::vector<Cidr> d;
             for (auto& t : del) d.push_back(Cidr{str(t[0]), t[1].cast<int32_t>()});
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
      .def_property_readonly("route_build_runs", &SpfSolver::routeBuildRuns)
      .def("set_prefix_shard", &SpfSolver::setPrefixShard, py::arg("rank"), py::arg("world"))
      .def_property_readonly("last_select_ms", &SpfSolver::lastSelectMs)
      .def_property_readonly("last_select_bytes", &SpfSolver::lastSelectBytes)
      .def_property_readonly("device_selected", &SpfSolver::deviceSelected)
      .def_property_readonly("host_selected", &SpfSolver::hostSelected);

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
             UnicastRouteMap m;
             for (auto r : routes) {
               RibUnicastEntry e = unicastFromWire(r.cast<py::tuple>());
               Cidr k = e.prefix;
               m.emplace(std::move(k), std::move(e));
             }
             auto ch = p.applyPolicy(m);
             py::list up, del, out;
             for (const auto& c : ch.updatedRoutes) up.append(py::make_tuple(pyBytes(c.first), c.second));
             for (const auto& c : ch.deletedRoutes) del.append(py::make_tuple(pyBytes(c.first), c.second));
             for (const auto& [_, e] : m) out.append(unicastToWire(e));
             return py::make_tuple(up, del, out);
           })
      .def_property_readonly("invalidated_routes", &RibPolicy::invalidatedRoutes);
  py::class_<RibStatementProbe>(m, "RibPolicyStatement")
      .def(py::init([](py::tuple st) {
        try {
          return new RibStatementProbe{RibPolicyStatement(statementFromWire(st))};
        } catch (const std::invalid_argument& e) {
          throw py::value_error(e.what());
        }
      }))
      .def("match", [](const RibStatementProbe& s, py::tuple r) { return s.st.match(unicastFromWire(r)); })
      .def("apply_action", [](const RibStatementProbe& s, py::tuple r) {
        RibUnicastEntry e = unicastFromWire(r);
        const bool changed = s.st.applyAction(e);
        return py::make_tuple(changed, unicastToWire(e));
      });

  m.def("device_count", [] {
    int n = 0;
    orh_device_count(&n);
    return n;
  });
  // distance-kernel selection on the default context (ORH_SPF_AUTO /
  // ORH_SPF_PER_SOURCE / ORH_SPF_GLOBAL); results are identical in every mode
  // what-if repair on the default context (ORH_REPAIR_OFF / _AUTO / _ALWAYS)
  m.def("set_repair_mode", [](int mode) {
    if (orh_set_repair_mode(defaultContext(), mode) != ORH_OK)
      throw std::invalid_argument("set_repair_mode: bad mode");
  });
  m.def("set_spf_mode", [](int mode) {
    if (orh_set_spf_mode(defaultContext(), mode) != ORH_OK)
      throw std::invalid_argument("set_spf_mode: mode must be 0, 1, 2 or 3");
  });
}
