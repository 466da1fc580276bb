// Compiled and run by tests/test_abi.py::test_route_map_unordered_map_api:
// the reference's own call patterns on DecisionRouteDb::unicastRoutes /
// DecisionRouteUpdate::unicastRoutesToUpdate (std::unordered_map there)
// compile and behave the same against the product's 64-shard map.
#include <cassert>
#include <cstdio>
#include <stdexcept>

#include "host_types.h"

using namespace openr_amd;

static Cidr pfx(int i) { return Cidr{AddrBytes(std::string(16, static_cast<char>(i))), 64}; }

int main() {
  DecisionRouteDb db;
  DecisionRouteUpdate upd;
  for (int i = 0; i < 200; ++i) {
    RibUnicastEntry e;
    e.prefix = pfx(i);
    // Decision.h:110  CHECK(unicastRoutes.emplace(key, std::move(entry)).second)
    auto key = e.prefix;
    if (!db.unicastRoutes.emplace(key, std::move(e)).second) return 1;
  }
  // RouteUpdate.h:34 / :41
  RibUnicastEntry r;
  r.prefix = pfx(7);
  upd.unicastRoutesToUpdate.emplace(r.prefix, r);
  // NetlinkSocket.cpp:386  emplace(std::make_pair(dest, std::move(route)))
  RibUnicastEntry r2;
  r2.prefix = pfx(201);
  if (!db.unicastRoutes.emplace(std::make_pair(r2.prefix, std::move(r2))).second) return 2;
  // Fib.cpp:304  unicastRoutes.at(prefix)
  if (db.unicastRoutes.at(pfx(3)).prefix != pfx(3)) return 3;
  bool threw = false;
  try {
    db.unicastRoutes.at(pfx(250));
  } catch (const std::out_of_range&) {
    threw = true;
  }
  if (!threw) return 4;
  // Decision.cpp:148 erase(prefix); count / find / insert_or_assign / size
  if (db.unicastRoutes.erase(pfx(5)) != 1 || db.unicastRoutes.count(pfx(5)) != 0) return 5;
  if (db.unicastRoutes.find(pfx(6)) == db.unicastRoutes.end()) return 6;
  db.unicastRoutes.insert_or_assign(pfx(6), RibUnicastEntry{pfx(6), {}, std::nullopt, "x", false});
  if (db.unicastRoutes.at(pfx(6)).bestArea != "x") return 7;
  // Fib.cpp:357-361  for (auto i = m.begin(); i != m.end();) i = m.erase(i) (some)
  size_t kept = 0;
  for (auto i = db.unicastRoutes.begin(); i != db.unicastRoutes.end();) {
    if (i->first.first[0] % 2) {
      i = db.unicastRoutes.erase(i);
    } else {
      ++kept;
      ++i;
    }
  }
  if (kept != db.unicastRoutes.size() || kept != 100) return 8;
  for (const auto& [p, e] : db.unicastRoutes)
    if (p != e.prefix || p.first[0] % 2) return 9;
  db.unicastRoutes[pfx(9)].bestArea = "y";  // operator[]
  if (!db.unicastRoutes.try_emplace(pfx(11)).second || db.unicastRoutes.try_emplace(pfx(11)).second) return 10;
  if (!db.unicastRoutes.insert({pfx(13), RibUnicastEntry{}}).second) return 11;
  if (upd.unicastRoutesToUpdate.empty() || upd.unicastRoutesToUpdate.size() != 1) return 12;
  upd.unicastRoutesToUpdate.clear();
  std::printf("ok %zu\n", db.unicastRoutes.size());
  return 0;
}
