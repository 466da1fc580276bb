"""C5 buildRouteDb (1M prefixes, 4 areas, best-route) under env A/B specs on
one box: python tools/c5_build_ab.py "ORH_ROUTE_BUCKETS=0" "ORH_ROUTE_BUCKETS=1"
(each spec in its own child process, alternating, twice)."""
import os
import statistics
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from openr_amd import host_backend
    from openr_amd.facade import load_topology
    from openr_amd.workloads import C5_AREAS, c5_multi_area
    hip = host_backend()
    areas, pfx = c5_multi_area()
    als, ps = load_topology(hip, [db for a in C5_AREAS for db in areas[a]], pfx)
    solver = hip.spf_solver("me", True, enable_best_route_selection=True)
    ms = [solver._impl.time_build_route_db("me", als._impl, ps._impl)[0] * 1e3 for _ in range(7)]
    print(f"build ms {[round(x, 1) for x in ms]} median of the last 5 {statistics.median(ms[2:]):.2f}", flush=True)
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
