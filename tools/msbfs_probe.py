"""MS-BFS timing probe on the C2 grid (GPU box): the distance-phase time of
all-sources sweeps and of source subsets (one corner batch, one centre batch,
the first 8,192 / 10,000 sources), to separate per-workgroup latency from
co-residence and tail effects. Prints one JSON line per case.

  python tools/msbfs_probe.py [--n 100] [--reps 7]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.topology import bench_grid  # noqa: E402
from openr_amd.types import K_TESTING_AREA  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--cases", default="all,first8192,corner32,center32,corner256x32")
    args = ap.parse_args()
    n = args.n
    hip = host_backend()
    adj_dbs, _ = bench_grid(n)
    als, _ = load_topology(hip, adj_dbs, [])
    ls = als[K_TESTING_AREA]

    def node(x, y):
        return str(y * n + x)

    by_l1 = sorted(((x + y, x, y) for x in range(n) for y in range(n)))
    corner = [node(x, y) for _, x, y in by_l1[:32]]
    c = n // 2
    by_c = sorted(((abs(x - c) + abs(y - c), x, y) for x in range(n) for y in range(n)))
    center = [node(x, y) for _, x, y in by_c[:32]]
    cases = {
        "all": [str(i) for i in range(n * n)],
        "first8192": [str(i) for i in range(min(8192, n * n))],
        "corner32": corner,
        "center32": center,
        # the corner batch repeated: 256 identical workgroups, one per CU
        "corner256x32": corner * 256,
        "one": [node(1, 0)],
        "one_center": [node(c, c)],
    }
    for name in args.cases.split(","):
        srcs = cases[name]
        sweep = ls._impl.sweep(srcs, True)
        dist_ms, hop_ms = [], []
        for _ in range(args.reps + 1):
            sweep.run()
            sweep.sync()
            d, h = sweep.phase_ms()
            dist_ms.append(d)
            hop_ms.append(h)
        print(json.dumps({"case": name, "sources": len(srcs), "info": sweep.info(),
                          "dist_ms": round(statistics.median(dist_ms[1:]), 4),
                          "hop_ms": round(statistics.median(hop_ms[1:]), 4),
                          "env": {k: v for k, v in os.environ.items() if k.startswith("ORH_")}}),
              flush=True)


if __name__ == "__main__":
    main()
