// Thrift Compact protocol for the Decision path's wire types (SURVEY.md §8f
// rows f1 / f3): the route database Decision hands to Fib, and the
// adjacency / prefix databases it reads from KvStore publications.
//
// Schemas follow openr/if/Types.thrift and openr/if/Network.thrift field by
// field (ids, types, optional vs default fields); encoding follows the
// Apache Thrift Compact protocol (field headers as id deltas, zigzag
// varints, lists with an inline size nibble, bool values in the field
// header). Fields that are not `optional` are always written, as fbthrift
// does; optional fields only when set.
//
// List order: the reference's DecisionRouteDb::toThrift / RibUnicastEntry::
// toThrift walk unordered containers (Decision.h:93-104, RibEntry.h:77-90),
// so its byte order is unspecified. Here routes are
// written in ascending (prefix bytes, length) / label order and every
// nexthop list in the thrift operator< order of NextHopThrift (field by
// field, unset optionals first) - the order createUnicastRoute /
// createMplsRoute give (Util.cpp:813-847) - so equal databases serialize to
// equal bytes.
#pragma once

#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_types.h"

namespace openr_amd {
namespace compact {

enum Type : uint8_t {
  kStop = 0, kTrue = 1, kFalse = 2, kByte = 3, kI16 = 4, kI32 = 5, kI64 = 6, kDouble = 7,
  kBinary = 8, kList = 9, kSet = 10, kMap = 11, kStruct = 12
};

class Writer {
 public:
  void structBegin() { last_.push_back(0); }
  void structEnd() {
    out_.push_back(static_cast<char>(kStop));
    last_.pop_back();
  }
  void field(int16_t id, Type t);
  void fieldBool(int16_t id, bool v) { field(id, v ? kTrue : kFalse); }
  void fieldI16(int16_t id, int16_t v) { field(id, kI16); varint(zigzag32(v)); }
  void fieldI32(int16_t id, int32_t v) { field(id, kI32); varint(zigzag32(v)); }
  void fieldI64(int16_t id, int64_t v) { field(id, kI64); varint(zigzag64(v)); }
  void fieldBinary(int16_t id, const std::string& s) { field(id, kBinary); binary(s); }
  void listBegin(Type elem, size_t n);
  void mapBegin(Type key, Type val, size_t n) {
    varint(n);
    if (n) out_.push_back(static_cast<char>((key << 4) | val));
  }
  void i32(int32_t v) { varint(zigzag32(v)); }
  void i64(int64_t v) { varint(zigzag64(v)); }
  void binary(const std::string& s) {
    varint(s.size());
    out_.append(s);
  }
  const std::string& bytes() const { return out_; }
  std::string take() { return std::move(out_); }

 private:
  static uint64_t zigzag32(int32_t v) {
    return static_cast<uint32_t>((static_cast<uint32_t>(v) << 1) ^ static_cast<uint32_t>(v >> 31));
  }
  static uint64_t zigzag64(int64_t v) {
    return (static_cast<uint64_t>(v) << 1) ^ static_cast<uint64_t>(v >> 63);
  }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      out_.push_back(static_cast<char>((v & 0x7F) | 0x80));
      v >>= 7;
    }
    out_.push_back(static_cast<char>(v));
  }
  std::string out_;
  std::vector<int16_t> last_;  // last field id per open struct
};

class Reader {
 public:
  explicit Reader(const std::string& b) : p_(reinterpret_cast<const uint8_t*>(b.data())), e_(p_ + b.size()) {}
  Reader(const uint8_t* p, size_t n) : p_(p), e_(p + n) {}
  // nesting bound: peer-supplied bytes must not drive skip() into unbounded
  // recursion (fbthrift rejects such input as a deserialisation error)
  // (structs, lists, sets and maps count alike: a list level costs the peer
  // one byte, so containers are bounded as structs are)
  static constexpr size_t kMaxDepth = 64;
  void structBegin() {
    if (last_.size() + containers_ >= kMaxDepth) throw std::invalid_argument("compact: nesting too deep");
    last_.push_back(0);
  }
  void structEnd() { last_.pop_back(); }
  // next field header: false at the stop field; bool values arrive in the type
  bool field(int16_t* id, Type* t);
  int32_t i32() { return unzigzag32(static_cast<uint32_t>(varint())); }
  int16_t i16() { return static_cast<int16_t>(i32()); }
  int64_t i64() {
    const uint64_t u = varint();
    return static_cast<int64_t>((u >> 1) ^ (~(u & 1) + 1));
  }
  uint8_t byte() {
    need(1);
    return *p_++;
  }
  std::string binary();
  // list header: element type and size (every element takes at least one
  // byte, so a count beyond the remaining input is rejected before any
  // container is sized from it)
  void listBegin(Type* elem, uint32_t* n);
  // map header: key / value types (unset when empty) and size
  void mapBegin(Type* key, Type* val, uint32_t* n) {
    const uint64_t c = varint();
    if (c > remaining()) throw std::invalid_argument("compact: map size beyond the input");
    *n = static_cast<uint32_t>(c);
    *key = *val = kStop;
    if (*n) {
      const uint8_t kv = byte();
      *key = static_cast<Type>(kv >> 4);
      *val = static_cast<Type>(kv & 0x0F);
    }
  }
  // skip a value of type t (unknown fields)
  void skip(Type t);
  bool atEnd() const { return p_ == e_; }
  size_t remaining() const { return static_cast<size_t>(e_ - p_); }

 private:
  void need(size_t n) const {
    if (static_cast<size_t>(e_ - p_) < n) throw std::invalid_argument("compact: truncated input");
  }
  static int32_t unzigzag32(uint32_t u) { return static_cast<int32_t>((u >> 1) ^ (~(u & 1) + 1)); }
  uint64_t varint();
  const uint8_t* p_;
  const uint8_t* e_;
  std::vector<int16_t> last_;
  size_t containers_ = 0;  // list / set / map levels open inside skip()
  friend struct ContainerLevel;
};

// ---- Decision -> Fib (Types.thrift:1003-1060, Network.thrift:48-131) -------
std::string routeDatabase(const DecisionRouteDb& db, const std::string& thisNodeName);
std::string routeDatabaseDelta(const DecisionRouteUpdate& delta);
// NextHopThrift's generated operator< (fields in id order, unset optional first)
bool nextHopLess(const NextHopThrift& a, const NextHopThrift& b);

// ---- KvStore -> Decision (Types.thrift:263-343, :479-605) -------------------
AdjacencyDatabase adjacencyDatabase(const std::string& bytes);
struct PrefixDatabase {
  std::string thisNodeName;
  std::vector<PrefixEntry> prefixEntries;
  std::vector<std::vector<std::string>> areaStacks;  // PrefixEntry.area_stack, per entry
  bool deletePrefix{false};
  std::string area;
};
PrefixDatabase prefixDatabase(const std::string& bytes);
std::string adjacencyDatabaseBytes(const AdjacencyDatabase& db);  // encoder (tests, tools)
std::string prefixDatabaseBytes(const PrefixDatabase& db);

}  // namespace compact
}  // namespace openr_amd
