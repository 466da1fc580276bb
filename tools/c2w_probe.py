#!/usr/bin/env python3
"""C2w probe: all-sources sweep of the weighted 100x100 grid
(workloads.c2_weighted_grid, metrics 1..64): wall ms per sweep over --reps
back-to-back sweeps, the HIP-event device ms of one sweep alone, the plan.
Env knobs pass through (ORH_LDS_NH=0: the two-phase LDS plan; ORH_LDS_NH_BLOCK,
ORH_DELTA_PCT)."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--lanes", type=int, default=1)
    args = p.parse_args()
    from openr_amd import host_backend
    from openr_amd.facade import load_topology
    from openr_amd.types import K_TESTING_AREA as A
    from openr_amd.workloads import c2_weighted_grid
    hip = host_backend()
    adj, pfx = c2_weighted_grid(args.n)
    names = [db.thisNodeName for db in adj]
    sweeps = []
    for lane in range(args.lanes):
        als, _ = load_topology(hip, adj, pfx, lane=lane)
        sweeps.append((als, als[A]._impl.sweep(names, True)))
    for _, sw in sweeps:
        sw.run()
    for _, sw in sweeps:
        sw.sync()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        for _, sw in sweeps:
            sw.run()
    for _, sw in sweeps:
        sw.sync()
    wall = (time.perf_counter() - t0) / (args.reps * len(sweeps))
    sw = sweeps[0][1]
    dev, ph = [], []
    for _ in range(5):
        sw.run()
        dev.append(sw.last_ms())
        ph.append(sw.phase_ms())
    out = {"nodes": sw.nodes, "edges": sw.edges, "sources": len(names), "lanes": args.lanes,
           "wall_ms_per_sweep": round(wall * 1e3, 4), "device_ms": round(statistics.median(dev), 4),
           "phase_ms": [round(statistics.median(p[i] for p in ph), 4) for i in (0, 1)],
           "spf_sources_per_s": round(len(names) / wall, 1), "info": sw.info(),
           "env": {k: v for k, v in os.environ.items() if k.startswith("ORH_")}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
