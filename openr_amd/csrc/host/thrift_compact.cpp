// Thrift Compact protocol for the Decision path's wire types; see
// thrift_compact.h for the schemas and the ordering rules.
#include "thrift_compact.h"

#include <algorithm>
#include <tuple>

namespace openr_amd {
namespace compact {

// ---- protocol -----------------------------------------------------------------
void Writer::field(int16_t id, Type t) {
  int16_t& last = last_.back();
  const int d = id - last;
  if (d > 0 && d <= 15) {
    out_.push_back(static_cast<char>((d << 4) | t));
  } else {
    out_.push_back(static_cast<char>(t));
    varint(zigzag32(id));
  }
  last = id;
}

void Writer::listBegin(Type elem, size_t n) {
  if (n < 15) {
    out_.push_back(static_cast<char>((n << 4) | elem));
  } else {
    out_.push_back(static_cast<char>(0xF0 | elem));
    varint(n);
  }
}

uint64_t Reader::varint() {
  uint64_t v = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    need(1);
    const uint8_t b = *p_++;
    v |= static_cast<uint64_t>(b & 0x7F) << shift;
    if (!(b & 0x80)) return v;
  }
  throw std::invalid_argument("compact: varint too long");
}

bool Reader::field(int16_t* id, Type* t) {
  const uint8_t h = byte();
  if (h == kStop) return false;
  *t = static_cast<Type>(h & 0x0F);
  const uint8_t d = h >> 4;
  int16_t& last = last_.back();
  *id = d ? static_cast<int16_t>(last + d) : i16();
  last = *id;
  return true;
}

std::string Reader::binary() {
  const uint64_t n = varint();
  need(n);
  std::string s(reinterpret_cast<const char*>(p_), n);
  p_ += n;
  return s;
}

void Reader::listBegin(Type* elem, uint32_t* n) {
  const uint8_t h = byte();
  *elem = static_cast<Type>(h & 0x0F);
  const uint32_t s = h >> 4;
  const uint64_t c = s == 15 ? varint() : s;
  if (c > remaining()) throw std::invalid_argument("compact: list size beyond the input");
  *n = static_cast<uint32_t>(c);
}

// one open list / set / map level of skip(), bounded together with the open
// structs by kMaxDepth
struct ContainerLevel {
  explicit ContainerLevel(Reader& r) : r_(r) {
    if (r.last_.size() + r.containers_ >= Reader::kMaxDepth)
      throw std::invalid_argument("compact: nesting too deep");
    ++r.containers_;
  }
  ~ContainerLevel() { --r_.containers_; }
  Reader& r_;
};

void Reader::skip(Type t) {
  switch (t) {
    case kTrue: case kFalse: return;  // value in the header (field) or a byte (list element)
    case kByte: byte(); return;
    case kI16: case kI32: case kI64: varint(); return;
    case kDouble: need(8); p_ += 8; return;
    case kBinary: binary(); return;
    case kList: case kSet: {
      ContainerLevel level(*this);
      Type e;
      uint32_t n;
      listBegin(&e, &n);
      for (uint32_t i = 0; i < n; ++i) {
        if (e == kTrue || e == kFalse) byte();
        else skip(e);
      }
      return;
    }
    case kMap: {
      ContainerLevel level(*this);
      Type k, v;
      uint32_t n;
      mapBegin(&k, &v, &n);
      // a bool inside a map is a one-byte value, as in a list
      auto elem = [this](Type e) {
        if (e == kTrue || e == kFalse) byte();
        else skip(e);
      };
      for (uint32_t i = 0; i < n; ++i) {
        elem(k);
        elem(v);
      }
      return;
    }
    case kStruct: {
      structBegin();
      int16_t id;
      Type ft;
      while (field(&id, &ft)) skip(ft);
      structEnd();
      return;
    }
    default: throw std::invalid_argument("compact: unknown type " + std::to_string(int(t)));
  }
}

namespace {

bool readBool(Type t) {
  if (t != kTrue && t != kFalse) throw std::invalid_argument("compact: bool field of another type");
  return t == kTrue;
}

void expect(Type got, Type want, const char* what) {
  if (got != want) throw std::invalid_argument(std::string("compact: unexpected type for ") + what);
}

// ---- Network.thrift ---------------------------------------------------------
void writeBinaryAddress(Writer& w, const AddrBytes& addr, const std::optional<std::string>& ifName) {
  w.structBegin();
  w.field(1, kBinary);
  w.binary(addr.str());
  if (ifName) w.fieldBinary(3, *ifName);
  w.structEnd();
}

void writeIpPrefix(Writer& w, const Cidr& c) {  // Network.thrift:61-64
  w.structBegin();
  w.field(1, kStruct);
  writeBinaryAddress(w, c.first, std::nullopt);
  w.fieldI16(2, static_cast<int16_t>(c.second));
  w.structEnd();
}

void writeMplsAction(Writer& w, const MplsAction& a) {  // Network.thrift:48-54
  w.structBegin();
  w.fieldI32(1, a.action);
  if (a.swapLabel) w.fieldI32(2, *a.swapLabel);
  if (a.pushLabels) {
    w.field(3, kList);
    w.listBegin(kI32, a.pushLabels->size());
    for (int32_t l : *a.pushLabels) w.i32(l);
  }
  w.structEnd();
}

void writeNextHop(Writer& w, const NextHopThrift& nh) {  // Network.thrift:66-97
  w.structBegin();
  w.field(1, kStruct);
  writeBinaryAddress(w, nh.address.addr, nh.address.ifName);
  w.fieldI32(2, nh.weight);
  if (nh.mplsAction) {
    w.field(3, kStruct);
    writeMplsAction(w, *nh.mplsAction);
  }
  w.fieldI32(51, nh.metric);
  if (nh.area) w.fieldBinary(53, *nh.area);
  if (nh.neighborNodeName) w.fieldBinary(54, *nh.neighborNodeName);
  w.structEnd();
}

void writeNextHops(Writer& w, int16_t id, const NextHopSet& s) {
  std::vector<const NextHopThrift*> v;
  v.reserve(s.size());
  for (const auto& nh : s) v.push_back(&nh);
  std::sort(v.begin(), v.end(), [](const NextHopThrift* a, const NextHopThrift* b) { return nextHopLess(*a, *b); });
  w.field(id, kList);
  w.listBegin(kStruct, v.size());
  for (const auto* nh : v) writeNextHop(w, *nh);
}

// RibUnicastEntry::toThrift (RibEntry.h:77-90)
void writeUnicastRoute(Writer& w, const RibUnicastEntry& e) {  // Network.thrift:122-131
  w.structBegin();
  w.field(1, kStruct);
  writeIpPrefix(w, e.prefix);
  writeNextHops(w, 4, e.nexthops.set());
  const bool bgp = e.bestPrefixEntry && e.bestPrefixEntry->type == kPrefixTypeBgp;
  if (bgp) {
    w.fieldI32(5, kPrefixTypeBgp);
    if (e.bestPrefixEntry->data) w.fieldBinary(6, *e.bestPrefixEntry->data);
  }
  w.fieldBool(7, e.doNotInstall);
  w.structEnd();
}

// RibMplsEntry::toThrift (RibEntry.h:130-136)
void writeMplsRoute(Writer& w, const RibMplsEntry& e) {  // Network.thrift:99-103
  w.structBegin();
  w.fieldI32(1, e.label);
  writeNextHops(w, 4, e.nexthops.set());
  w.structEnd();
}

bool cidrLess(const Cidr& a, const Cidr& b) {
  return a.first != b.first ? a.first < b.first : a.second < b.second;
}

template <class Map>
std::vector<const RibUnicastEntry*> sortedUnicast(const Map& m) {
  std::vector<const RibUnicastEntry*> v;
  v.reserve(m.size());
  for (const auto& kv : m) v.push_back(&kv.second);
  std::sort(v.begin(), v.end(),
            [](const RibUnicastEntry* a, const RibUnicastEntry* b) { return cidrLess(a->prefix, b->prefix); });
  return v;
}

// ---- Types.thrift: adjacency / prefix databases ------------------------------
BinaryAddress readBinaryAddress(Reader& r) {
  BinaryAddress a;
  r.structBegin();
  int16_t id;
  Type t;
  while (r.field(&id, &t)) {
    if (id == 1 && t == kBinary) a.addr = AddrBytes(r.binary());
    else if (id == 3 && t == kBinary) a.ifName = r.binary();
    else r.skip(t);
  }
  r.structEnd();
  return a;
}

Adjacency readAdjacency(Reader& r) {  // Types.thrift:74-142
  Adjacency a;
  r.structBegin();
  int16_t id;
  Type t;
  while (r.field(&id, &t)) {
    switch (id) {
      case 1: expect(t, kBinary, "otherNodeName"); a.otherNodeName = r.binary(); break;
      case 2: expect(t, kBinary, "ifName"); a.ifName = r.binary(); break;
      case 3: expect(t, kStruct, "nextHopV6"); a.nextHopV6 = readBinaryAddress(r); break;
      case 5: expect(t, kStruct, "nextHopV4"); a.nextHopV4 = readBinaryAddress(r); break;
      case 4: expect(t, kI32, "metric"); a.metric = r.i32(); break;
      case 6: expect(t, kI32, "adjLabel"); a.adjLabel = r.i32(); break;
      case 7: a.isOverloaded = readBool(t); break;
      case 8: expect(t, kI32, "rtt"); a.rtt = r.i32(); break;
      case 9: expect(t, kI64, "timestamp"); a.timestamp = r.i64(); break;
      case 10: expect(t, kI64, "weight"); a.weight = r.i64(); break;
      case 11: expect(t, kBinary, "otherIfName"); a.otherIfName = r.binary(); break;
      default: r.skip(t);
    }
  }
  r.structEnd();
  return a;
}

MetricVector readMetricVector(Reader& r) {  // Types.thrift:237-296
  MetricVector mv;
  r.structBegin();
  int16_t id;
  Type t;
  while (r.field(&id, &t)) {
    if (id == 1 && t == kI64) {
      mv.version = r.i64();
    } else if (id == 2 && t == kList) {
      Type e;
      uint32_t n;
      r.listBegin(&e, &n);
      expect(e, kStruct, "MetricVector.metrics");
      for (uint32_t i = 0; i < n; ++i) {
        MetricEntity me;
        r.structBegin();
        int16_t fid;
        Type ft;
        while (r.field(&fid, &ft)) {
          if (fid == 1 && ft == kI64) me.type = r.i64();
          else if (fid == 2 && ft == kI64) me.priority = r.i64();
          else if (fid == 3 && ft == kI32) me.op = r.i32();
          else if (fid == 4) me.isBestPathTieBreaker = readBool(ft);
          else if (fid == 5 && ft == kList) {
            Type le;
            uint32_t ln;
            r.listBegin(&le, &ln);
            expect(le, kI64, "MetricEntity.metric");
            for (uint32_t k = 0; k < ln; ++k) me.metric.push_back(r.i64());
          } else {
            r.skip(ft);
          }
        }
        r.structEnd();
        mv.metrics.push_back(std::move(me));
      }
    } else {
      r.skip(t);
    }
  }
  r.structEnd();
  return mv;
}

PrefixEntry readPrefixEntry(Reader& r, std::vector<std::string>* areaStack) {  // Types.thrift:350-429
  PrefixEntry p;
  r.structBegin();
  int16_t id;
  Type t;
  while (r.field(&id, &t)) {
    switch (id) {
      case 1: {  // IpPrefix
        expect(t, kStruct, "prefix");
        r.structBegin();
        int16_t fid;
        Type ft;
        while (r.field(&fid, &ft)) {
          if (fid == 1 && ft == kStruct) p.addr = readBinaryAddress(r).addr;
          else if (fid == 2 && ft == kI16) p.len = r.i16();
          else r.skip(ft);
        }
        r.structEnd();
        break;
      }
      case 2: expect(t, kI32, "type"); p.type = r.i32(); break;
      case 3: expect(t, kBinary, "data"); p.data = r.binary(); break;
      case 4: expect(t, kI32, "forwardingType"); p.forwardingType = r.i32(); break;
      case 7: expect(t, kI32, "forwardingAlgorithm"); p.forwardingAlgorithm = r.i32(); break;
      case 6: expect(t, kStruct, "mv"); p.mv = readMetricVector(r); break;
      case 8: expect(t, kI64, "minNexthop"); p.minNexthop = r.i64(); break;
      case 9: expect(t, kI32, "prependLabel"); p.prependLabel = r.i32(); break;
      case 10: {  // PrefixMetrics
        expect(t, kStruct, "metrics");
        r.structBegin();
        int16_t fid;
        Type ft;
        while (r.field(&fid, &ft)) {
          if (fid == 2 && ft == kI32) p.pathPreference = r.i32();
          else if (fid == 3 && ft == kI32) p.sourcePreference = r.i32();
          else if (fid == 4 && ft == kI32) p.distance = r.i32();
          else r.skip(ft);
        }
        r.structEnd();
        break;
      }
      case 11: {  // set<string> tags
        Type e;
        uint32_t n;
        r.listBegin(&e, &n);
        expect(e, kBinary, "tags");
        for (uint32_t i = 0; i < n; ++i) p.tags.insert(r.binary());
        break;
      }
      case 12: {  // list<string> area_stack
        Type e;
        uint32_t n;
        r.listBegin(&e, &n);
        if (n) expect(e, kBinary, "area_stack");
        for (uint32_t i = 0; i < n; ++i) areaStack->push_back(r.binary());
        break;
      }
      default: r.skip(t);
    }
  }
  r.structEnd();
  // toIPNetwork (folly createNetwork) throws on a malformed CIDR, and
  // Decision counts the entry as failed to deserialise: same rule as parseCidr
  const size_t nb = p.addr.size();
  if ((nb != 4 && nb != 16) || p.len < 0 || p.len > static_cast<int>(8 * nb))
    throw std::invalid_argument("compact: malformed prefix (address of " + std::to_string(nb) +
                                " bytes, length " + std::to_string(p.len) + ")");
  // the reference keys prefixes by the masked network (folly::CIDRNetwork)
  for (size_t i = 0; i < nb; ++i) {
    const int keep = std::clamp(p.len - static_cast<int>(8 * i), 0, 8);
    p.addr[i] = static_cast<char>(static_cast<uint8_t>(p.addr[i]) & static_cast<uint8_t>(0xFF00u >> keep));
  }
  return p;
}

void writePrefixEntry(Writer& w, const PrefixEntry& p, const std::vector<std::string>& areaStack) {
  w.structBegin();
  w.field(1, kStruct);
  writeIpPrefix(w, Cidr{p.addr, p.len});
  w.fieldI32(2, p.type);
  if (p.data) w.fieldBinary(3, *p.data);
  w.fieldI32(4, p.forwardingType);
  if (p.mv) {
    w.field(6, kStruct);
    w.structBegin();
    w.fieldI64(1, p.mv->version);
    w.field(2, kList);
    w.listBegin(kStruct, p.mv->metrics.size());
    for (const auto& me : p.mv->metrics) {
      w.structBegin();
      w.fieldI64(1, me.type);
      w.fieldI64(2, me.priority);
      w.fieldI32(3, me.op);
      w.fieldBool(4, me.isBestPathTieBreaker);
      w.field(5, kList);
      w.listBegin(kI64, me.metric.size());
      for (int64_t x : me.metric) w.i64(x);
      w.structEnd();
    }
    w.structEnd();
  }
  w.fieldI32(7, p.forwardingAlgorithm);
  if (p.minNexthop) w.fieldI64(8, *p.minNexthop);
  if (p.prependLabel) w.fieldI32(9, *p.prependLabel);
  w.field(10, kStruct);
  w.structBegin();
  w.fieldI32(1, 1);
  w.fieldI32(2, p.pathPreference);
  w.fieldI32(3, p.sourcePreference);
  w.fieldI32(4, p.distance);
  w.structEnd();
  w.field(11, kSet);
  w.listBegin(kBinary, p.tags.size());
  for (const auto& tag : p.tags) w.binary(tag);
  w.field(12, kList);
  w.listBegin(kBinary, areaStack.size());
  for (const auto& a : areaStack) w.binary(a);
  w.structEnd();
}

}  // namespace

bool nextHopLess(const NextHopThrift& a, const NextHopThrift& b) {
  auto key = [](const NextHopThrift& n) {
    return std::make_tuple(n.address.addr.view(), n.address.ifName.has_value(),
                           n.address.ifName ? std::string_view(*n.address.ifName) : std::string_view(),
                           n.weight, n.mplsAction.has_value());
  };
  const auto ka = key(a), kb = key(b);
  if (ka != kb) return ka < kb;
  if (a.mplsAction && b.mplsAction) {
    const auto& x = *a.mplsAction;
    const auto& y = *b.mplsAction;
    if (x.action != y.action) return x.action < y.action;
    if (x.swapLabel != y.swapLabel) return x.swapLabel < y.swapLabel;  // nullopt first
    if (x.pushLabels != y.pushLabels) return x.pushLabels < y.pushLabels;
  }
  if (a.metric != b.metric) return a.metric < b.metric;
  if (a.area != b.area) return a.area < b.area;
  return a.neighborNodeName < b.neighborNodeName;
}

std::string routeDatabase(const DecisionRouteDb& db, const std::string& thisNodeName) {
  // DecisionRouteDb::toThrift (Decision.h:93-104); thisNodeName is written
  // because the field is not optional (Types.thrift:1003-1025)
  Writer w;
  w.structBegin();
  w.fieldBinary(1, thisNodeName);
  const auto uc = sortedUnicast(db.unicastRoutes);
  w.field(4, kList);
  w.listBegin(kStruct, uc.size());
  for (const auto* e : uc) writeUnicastRoute(w, *e);
  std::vector<const RibMplsEntry*> mp;
  mp.reserve(db.mplsRoutes.size());
  for (const auto& kv : db.mplsRoutes) mp.push_back(&kv.second);
  std::sort(mp.begin(), mp.end(), [](const RibMplsEntry* a, const RibMplsEntry* b) { return a->label < b->label; });
  w.field(5, kList);
  w.listBegin(kStruct, mp.size());
  for (const auto* e : mp) writeMplsRoute(w, *e);
  w.structEnd();
  return w.take();
}

std::string routeDatabaseDelta(const DecisionRouteUpdate& d) {
  // DecisionRouteUpdate::toThrift (RouteUpdate.h:45-63), Types.thrift:1031-1060
  Writer w;
  w.structBegin();
  const auto uu = sortedUnicast(d.unicastRoutesToUpdate);
  w.field(2, kList);
  w.listBegin(kStruct, uu.size());
  for (const auto* e : uu) writeUnicastRoute(w, *e);
  std::vector<Cidr> del(d.unicastRoutesToDelete);
  std::sort(del.begin(), del.end(), cidrLess);
  w.field(3, kList);
  w.listBegin(kStruct, del.size());
  for (const auto& c : del) writeIpPrefix(w, c);
  std::vector<const RibMplsEntry*> mu;
  for (const auto& e : d.mplsRoutesToUpdate) mu.push_back(&e);
  std::sort(mu.begin(), mu.end(), [](const RibMplsEntry* a, const RibMplsEntry* b) { return a->label < b->label; });
  w.field(4, kList);
  w.listBegin(kStruct, mu.size());
  for (const auto* e : mu) writeMplsRoute(w, *e);
  std::vector<int32_t> md(d.mplsRoutesToDelete);
  std::sort(md.begin(), md.end());
  w.field(5, kList);
  w.listBegin(kI32, md.size());
  for (int32_t l : md) w.i32(l);
  w.structEnd();
  return w.take();
}

AdjacencyDatabase adjacencyDatabase(const std::string& bytes) {  // Types.thrift:144-180
  Reader r(bytes);
  AdjacencyDatabase db;
  r.structBegin();
  int16_t id;
  Type t;
  while (r.field(&id, &t)) {
    switch (id) {
      case 1: expect(t, kBinary, "thisNodeName"); db.thisNodeName = r.binary(); break;
      case 2: db.isOverloaded = readBool(t); break;
      case 3: {
        expect(t, kList, "adjacencies");
        Type e;
        uint32_t n;
        r.listBegin(&e, &n);
        expect(e, kStruct, "adjacencies element");
        for (uint32_t i = 0; i < n; ++i) db.adjacencies.push_back(readAdjacency(r));
        break;
      }
      case 4: expect(t, kI32, "nodeLabel"); db.nodeLabel = r.i32(); break;
      case 6: expect(t, kBinary, "area"); db.area = r.binary(); break;
      default: r.skip(t);
    }
  }
  r.structEnd();
  if (!r.atEnd()) throw std::invalid_argument("compact: trailing bytes after AdjacencyDatabase");
  return db;
}

PrefixDatabase prefixDatabase(const std::string& bytes) {  // Types.thrift:431-460
  Reader r(bytes);
  PrefixDatabase db;
  r.structBegin();
  int16_t id;
  Type t;
  while (r.field(&id, &t)) {
    switch (id) {
      case 1: expect(t, kBinary, "thisNodeName"); db.thisNodeName = r.binary(); break;
      case 3: {
        expect(t, kList, "prefixEntries");
        Type e;
        uint32_t n;
        r.listBegin(&e, &n);
        expect(e, kStruct, "prefixEntries element");
        // containers grow as elements parse (the count is peer-supplied)
        for (uint32_t i = 0; i < n; ++i) {
          db.areaStacks.emplace_back();
          db.prefixEntries.push_back(readPrefixEntry(r, &db.areaStacks.back()));
        }
        break;
      }
      case 5: db.deletePrefix = readBool(t); break;
      case 7: expect(t, kBinary, "area"); db.area = r.binary(); break;
      default: r.skip(t);
    }
  }
  r.structEnd();
  if (!r.atEnd()) throw std::invalid_argument("compact: trailing bytes after PrefixDatabase");
  return db;
}

std::string adjacencyDatabaseBytes(const AdjacencyDatabase& db) {
  Writer w;
  w.structBegin();
  w.fieldBinary(1, db.thisNodeName);
  w.fieldBool(2, db.isOverloaded);
  w.field(3, kList);
  w.listBegin(kStruct, db.adjacencies.size());
  for (const auto& a : db.adjacencies) {
    w.structBegin();
    w.fieldBinary(1, a.otherNodeName);
    w.fieldBinary(2, a.ifName);
    w.field(3, kStruct);
    writeBinaryAddress(w, a.nextHopV6.addr, a.nextHopV6.ifName);
    w.fieldI32(4, a.metric);
    w.field(5, kStruct);
    writeBinaryAddress(w, a.nextHopV4.addr, a.nextHopV4.ifName);
    w.fieldI32(6, a.adjLabel);
    w.fieldBool(7, a.isOverloaded);
    w.fieldI32(8, a.rtt);
    w.fieldI64(9, a.timestamp);
    w.fieldI64(10, a.weight);
    w.fieldBinary(11, a.otherIfName);
    w.structEnd();
  }
  w.fieldI32(4, db.nodeLabel);
  w.fieldBinary(6, db.area);
  w.structEnd();
  return w.take();
}

std::string prefixDatabaseBytes(const PrefixDatabase& db) {
  Writer w;
  w.structBegin();
  w.fieldBinary(1, db.thisNodeName);
  w.field(3, kList);
  w.listBegin(kStruct, db.prefixEntries.size());
  for (size_t i = 0; i < db.prefixEntries.size(); ++i)
    writePrefixEntry(w, db.prefixEntries[i], i < db.areaStacks.size() ? db.areaStacks[i] : std::vector<std::string>{});
  w.fieldBool(5, db.deletePrefix);
  w.fieldBinary(7, db.area);
  w.structEnd();
  return w.take();
}

}  // namespace compact
}  // namespace openr_amd
