#!/usr/bin/env python3
"""Host cost of keeping one topology on N device replicas (verdict r05 item 7:
one host graph store for N device mirrors). For N = 1 and 8 replicas
(contexts on this GPU standing in for devices) of the C3 Clos and the C4 WAN:
  load      every adjacency database applied once (updateAdjacencyDatabase)
  updates   1,000 seeded single-adjacency metric changes, host side only
            (LinkState.cpp:564-719 once; each replica's mirror marked dirty)
  flush     each replica's device mirror brought up to date (per device; on
            N GPUs these run in parallel, here one after another)
Prints one JSON line per (workload, N)."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from openr_amd import host_backend
    from openr_amd.types import K_TESTING_AREA as A
    from openr_amd.workloads import c3_fabric, c4_wan
    hip = host_backend()
    for name, (adj, _) in (("C3", c3_fabric(num_prefixes=0)), ("C4", c4_wan())):
        wires = [db.to_wire() for db in adj]
        for n in (1, 8):
            rls = hip.module.ReplicatedLinkState(A, [0] * n)
            t0 = time.perf_counter()
            for w in wires:
                rls.update_adjacency_database(w)
            load = time.perf_counter() - t0
            t0 = time.perf_counter()
            for r in range(n):
                rls.replica(r).mirror_stats()  # no flush; warm the binding
            rng = random.Random(7)
            upd = []
            for _ in range(1000):
                db = adj[rng.randrange(len(adj))]
                db.adjacencies[rng.randrange(len(db.adjacencies))].metric = rng.randint(1, 9)
                upd.append(db.to_wire())
            t0 = time.perf_counter()
            for w in upd:
                rls.update_adjacency_database(w)
            updates = time.perf_counter() - t0
            t0 = time.perf_counter()
            for r in range(n):
                rls.replica(r).spf_words([adj[0].thisNodeName])  # flushes the replica's mirror
            flush = time.perf_counter() - t0
            print(json.dumps({"workload": name, "replicas": n, "nodes": len(adj),
                              "load_ms": round(load * 1e3, 2), "updates_1000_ms": round(updates * 1e3, 2),
                              "flush_all_ms": round(flush * 1e3, 2)}), flush=True)
            del rls


if __name__ == "__main__":
    main()
