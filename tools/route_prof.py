"""buildRouteDb phase profile on C2 (GPU box): median per phase over warm
builds (memoized SPF) and cold builds (a metric flip clears the memo), from
the product's ORH_ROUTE_PROF stderr lines. Prints one JSON line per mode.

  python tools/route_prof.py [--n 100] [--reps 9]
"""
import argparse
import collections
import json
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--reps", type=int, default=9)
    args = ap.parse_args()
    os.environ["ORH_ROUTE_PROF"] = "1"
    from openr_amd import host_backend
    from openr_amd.facade import load_topology
    from openr_amd.topology import bench_grid
    from openr_amd.types import K_TESTING_AREA

    hip = host_backend()
    n = args.n
    adj_dbs, prefixes = bench_grid(n, 1)
    als, ps = load_topology(hip, adj_dbs, prefixes)
    ls = als[K_TESTING_AREA]
    solver = hip.spf_solver("1", True)
    db = adj_dbs[n * n // 2]
    flip = [0]

    def build(cold):
        if cold:
            flip[0] ^= 1
            db.adjacencies[0].metric = 1 + flip[0]
            ls.update_adjacency_database(db)
        return solver._impl.time_build_route_db("1", als._impl, ps._impl)[0] * 1e3

    # capture fd 2 (the C++ fprintf lines) around each mode
    for mode in ("warm", "cold"):
        build(mode == "cold")  # settle
        with tempfile.TemporaryFile(mode="w+") as tmp:
            saved = os.dup(2)
            os.dup2(tmp.fileno(), 2)
            try:
                totals = [build(mode == "cold") for _ in range(args.reps)]
            finally:
                os.dup2(saved, 2)
                os.close(saved)
            tmp.seek(0)
            phases = collections.defaultdict(list)
            for line in tmp:
                if line.startswith("route-prof "):
                    name, ms = line[len("route-prof "):].rsplit(None, 2)[0].strip(), line.split()[-2]
                    phases[name].append(float(ms))
        print(json.dumps({"mode": mode, "total_ms": round(statistics.median(totals), 3),
                          "phases_ms": {k: round(statistics.median(v), 3) for k, v in phases.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
