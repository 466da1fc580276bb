"""C2 (grid, me = "1") and C3 (Clos, 100k prefixes, best-route) buildRouteDb
under env A/B specs, each spec in its own child process, alternating, twice:
  python tools/route_build_ab.py "ORH_ROUTE_TWO_PHASE=1" "ORH_ROUTE_TWO_PHASE=0"
Per child: medians of 9 warm builds each, C2 cold (after a metric flip) too."""
import os
import statistics
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from openr_amd import host_backend
    from openr_amd.facade import load_topology
    from openr_amd.topology import bench_grid
    from openr_amd.types import K_TESTING_AREA
    from openr_amd.workloads import c3_fabric
    hip = host_backend()
    adj, pfx = bench_grid(100, 1)
    als, ps = load_topology(hip, adj, pfx)
    s2 = hip.spf_solver("1", True)
    for _ in range(3):
        s2._impl.time_build_route_db("1", als._impl, ps._impl)
    warm2 = [s2._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3 for _ in range(9)]
    db = adj[5050]
    cold2 = []
    for i in range(11):
        db.adjacencies[0].metric = 1 + (i & 1)
        als[K_TESTING_AREA].update_adjacency_database(db)
        cold2.append(s2._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3)
    adj3, pfx3 = c3_fabric()
    als3, ps3 = load_topology(hip, adj3, pfx3)
    me3 = "2-0-0"  # the bench's C3 node
    s3 = hip.spf_solver(me3, True)
    for _ in range(3):
        s3._impl.time_build_route_db(me3, als3._impl, ps3._impl)
    c3 = [s3._impl.time_build_route_db(me3, als3._impl, ps3._impl)[0] * 1e3 for _ in range(9)]
    print(f"C2 warm {statistics.median(warm2):.2f} cold {statistics.median(cold2[2:]):.2f} ms | "
          f"C3 {statistics.median(c3):.2f} ms {[round(x, 2) for x in c3]}", flush=True)
    sys.exit(0)
for rep in range(2):
    for spec in sys.argv[1:]:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                           timeout=400)
        print(f"[{spec}] {r.stdout.strip()} {r.stderr.strip()[-300:] if r.returncode else ''}", flush=True)
