#!/usr/bin/env python3
"""buildRouteDb phase profile on the C2 grid (GPU box): ORH_ROUTE_PROF=1."""
import os
import sys
import time

os.environ["ORH_ROUTE_PROF"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.topology import bench_grid  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
adj, pfx = bench_grid(n, 1)
hip = host_backend()
als, ps = load_topology(hip, adj, pfx)
solver = hip.spf_solver("1", True)
for i in range(3):
    print("--- run", i, file=sys.stderr)
    t = time.perf_counter()
    sec, nr = solver._impl.time_build_route_db("1", als._impl, ps._impl)
    print(f"total {sec*1e3:.3f} ms, {nr} routes, wall {(time.perf_counter()-t)*1e3:.3f}", file=sys.stderr)
