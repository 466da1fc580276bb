#!/usr/bin/env python3
"""buildRouteDb phase profile (GPU box): ORH_ROUTE_PROF=1.
usage: route_prof.py [grid N | c3]"""
import os
import sys
import time

os.environ["ORH_ROUTE_PROF"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402

hip = host_backend()
if len(sys.argv) > 1 and sys.argv[1] == "c3":
    from openr_amd.workloads import c3_fabric  # noqa: E402
    adj, pfx = c3_fabric()
    me = "2-0-0"
else:
    from openr_amd.topology import bench_grid  # noqa: E402
    adj, pfx = bench_grid(int(sys.argv[1]) if len(sys.argv) > 1 else 100, 1)
    me = "1"
als, ps = load_topology(hip, adj, pfx)
solver = hip.spf_solver(me, True)
for i in range(4):
    print("--- run", i, file=sys.stderr)
    t = time.perf_counter()
    sec, nr = solver._impl.time_build_route_db(me, als._impl, ps._impl)
    print(f"total {sec*1e3:.3f} ms, {nr} routes, wall {(time.perf_counter()-t)*1e3:.3f}", file=sys.stderr)
