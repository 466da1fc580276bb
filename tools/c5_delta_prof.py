"""Phase times (ORH_ROUTE_PROF) of the C5 Decision rebuilds: the first full
rebuild, then the delta rebuild after the leg's incremental stress.
python tools/c5_delta_prof.py"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.rib_policy import RibPolicy, RibPolicyStatement, RibRouteActionWeight  # noqa: E402
from openr_amd.types import PrefixEntry, PrefixMetrics  # noqa: E402
from openr_amd.workloads import C5_AREAS, C5_TAG, c5_multi_area  # noqa: E402

hip = host_backend()
areas, pfx = c5_multi_area()
t0 = time.perf_counter()
als, ps = load_topology(hip, [db for a in C5_AREAS for db in areas[a]], pfx)
print(f"load {time.perf_counter() - t0:.3f} s", flush=True)
solver = hip.spf_solver("me", True, enable_best_route_selection=True)
policy = RibPolicy([RibPolicyStatement("ucmp", None, [C5_TAG], RibRouteActionWeight(
    0, {"A": 1, "B": 2, "C": 3, "D": 4}, {}))], 3600)
rib = hip.module.DecisionRib()
os.environ["ORH_ROUTE_PROF"] = "1"
for rep in range(3):  # buildRouteDb alone (the leg's build_route_db_ms)
    print("build", rep, solver._impl.time_build_route_db("me", als._impl, ps._impl), flush=True)
print("first", rib.rebuild_routes(solver._impl, "me", als._impl, ps._impl, True, [], policy._impl, wire=False),
      flush=True)
rng = random.Random(55)
changed = set()
for i in range(10_000):
    node, area, e = pfx[rng.randrange(len(pfx))]
    got = (ps.delete_prefix(node, area, e.prefix) if i % 2 else ps.update_prefix(node, area, PrefixEntry(
        e.prefix, metrics=PrefixMetrics(1, rng.randint(0, 3), rng.randint(0, 3), rng.randint(0, 3)), tags=e.tags)))
    changed |= {(p.prefixAddress.addr, p.prefixLength) for p in got}
for _ in range(100):
    a = rng.choice(C5_AREAS)
    db = areas[a][rng.randrange(len(areas[a]) - 1)]
    db.adjacencies[rng.randrange(len(db.adjacencies))].metric = rng.randint(1, 4)
    als[a].update_adjacency_database(db)
for rep in range(3):
    t0 = time.perf_counter()
    r = rib.rebuild_routes(solver._impl, "me", als._impl, ps._impl, True, sorted(changed), policy._impl, wire=False)
    print("delta", rep, r, "wall", time.perf_counter() - t0, "delta_rebuilds", rib.delta_rebuilds, flush=True)
    changed = set()
