"""C2 buildRouteDb (grid 100x100, me = "1") cold / warm, every sample printed:
the run-to-run spread of the bench's build_route_db_runs, and what sets it.
  python tools/c2_build_spread.py [reps]   (env knobs, e.g. ORH_HOST_THREADS, apply)"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.topology import bench_grid  # noqa: E402
from openr_amd.types import K_TESTING_AREA  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
hip = host_backend()
n = 100
adj, pfx = bench_grid(n, 1)
als, ps = load_topology(hip, adj, pfx)
ls = als[K_TESTING_AREA]
solver = hip.spf_solver("1", True)
solver.build_route_db("1", als, ps)
db = adj[n * n // 2]
flip = [0]


def cold():
    flip[0] ^= 1
    db.adjacencies[0].metric = 1 + flip[0]
    ls.update_adjacency_database(db)
    return solver._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3


for pause in (0.0, 0.05):
    c = []
    for _ in range(reps):
        if pause:
            time.sleep(pause)  # the pool's threads go idle between builds
        c.append(cold())
    w = [solver._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3 for _ in range(reps)]
    for name, xs in (("cold", c), ("warm", w)):
        m = statistics.median(xs)
        print(f"threads {hip.module.host_threads()} pause {pause:.2f} s {name}: median {m:.3f} min {min(xs):.3f} "
              f"max {max(xs):.3f} spread {(max(xs) - min(xs)) / m:.2f} | {[round(x, 2) for x in xs]}", flush=True)
