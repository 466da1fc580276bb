#!/usr/bin/env python3
"""Same-box A/B of route-build host knobs (round 6): C2 (grid, me = "1")
warm / cold, C3 (Clos, 100k prefixes) and C5 (4 areas, 1M prefixes,
best-route) buildRouteDb medians, each env spec in its own child process,
alternating, twice:
  python tools/route_ab_r06.py "ORH_NODE_POOL=1" "ORH_NODE_POOL=0" "ORH_MERGE_DYN=0"
A child prints one JSON line; the parent prints them with the spec."""
import json
import os
import statistics
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.setdefault("ORH_MALLOC_TUNE", "1")  # as bench.py
    from openr_amd import host_backend
    from openr_amd.facade import load_topology
    from openr_amd.topology import bench_grid
    from openr_amd.types import K_TESTING_AREA
    from openr_amd.workloads import C5_AREAS, c3_fabric, c5_multi_area
    hip = host_backend()
    out = {}
    adj, pfx = bench_grid(100, 1)
    als, ps = load_topology(hip, adj, pfx)
    s2 = hip.spf_solver("1", True)
    for _ in range(3):
        s2._impl.time_build_route_db("1", als._impl, ps._impl)
    out["c2_warm"] = statistics.median(s2._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3
                                       for _ in range(9))
    db = adj[5050]
    cold = []
    for i in range(11):
        db.adjacencies[0].metric = 1 + (i & 1)
        als[K_TESTING_AREA].update_adjacency_database(db)
        cold.append(s2._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3)
    out["c2_cold"] = statistics.median(cold[2:])
    del als, ps, s2
    adj3, pfx3 = c3_fabric()
    als3, ps3 = load_topology(hip, adj3, pfx3)
    s3 = hip.spf_solver("2-0-0", True)
    for _ in range(2):
        s3._impl.time_build_route_db("2-0-0", als3._impl, ps3._impl)
    out["c3"] = statistics.median(s3._impl.time_build_route_db("2-0-0", als3._impl, ps3._impl)[0] * 1e3
                                  for _ in range(9))
    del als3, ps3, s3
    areas, pfx5 = c5_multi_area()
    als5, ps5 = load_topology(hip, [d for a in C5_AREAS for d in areas[a]], pfx5)
    s5 = hip.spf_solver("me", True, enable_best_route_selection=True)
    ms = [s5._impl.time_build_route_db("me", als5._impl, ps5._impl)[0] * 1e3 for _ in range(7)]
    out["c5"] = statistics.median(ms[2:])
    print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)
    sys.exit(0)

specs = sys.argv[1:] or [""]
for rep in range(2):
    for spec in specs:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                           capture_output=True, text=True, timeout=600)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else f"FAILED rc={r.returncode} {r.stderr[-300:]}"
        print(f"[{spec or 'default'} rep{rep + 1}] {line}", flush=True)
