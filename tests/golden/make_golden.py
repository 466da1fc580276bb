#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference Decision path cannot be built or run here (folly / fbthrift /
fb303 are absent), so these vectors are produced by the CPU
oracle (oracle/, test infrastructure), which is itself pinned by the
reference's own known-answer tests (tests/test_ka_link_state.py,
tests/test_ka_decision.py). They freeze that pinned behaviour on larger,
seeded inputs so both the oracle (``-m "not gpu"``) and the HIP product
(``-m gpu``) are checked against committed data, not only against each other.

Fixtures
  spf_random.json   getSpfResult (metric, sorted nextHops) for every source of
                    seeded random graphs (parallel links, directional metrics,
                    drained nodes and adjacencies), link metric and hop count
  route_db_c1.json  buildRouteDb on config C1 (createGrid(10, 1, SP_ECMP),
                    RoutingBenchmarkUtils.cpp:271-313): the full canonical route
                    DB of myNode "1" plus a sha256 of every node's route DB
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SPF_SEEDS = (0, 1, 2, 3)


def spf_table(ls, names):
    out = {}
    for src in names:
        for metric in (True, False):
            res = ls.get_spf_result(src, metric)
            out[f"{src}|{int(metric)}"] = {d: [r.metric, sorted(r.nextHops)]
                                           for d, r in sorted(res.items())}
    return out


def route_db_json(db):
    uni, mpls = db.canonical()
    return {"unicast": {k: [sorted(repr(nh) for nh in nhs), dni]
                        for k, (nhs, dni) in sorted(uni.items())},
            "mpls": {str(k): sorted(repr(nh) for nh in nhs) for k, nhs in sorted(mpls.items())}}


def route_db_digest(db):
    return hashlib.sha256(json.dumps(route_db_json(db), sort_keys=True).encode()).hexdigest()


def main():
    from conftest import _load_oracle
    from openr_amd.facade import Backend, load_topology
    from openr_amd.topology import bench_grid
    from openr_amd.types import K_TESTING_AREA as A
    from test_gpu_parity import random_topology

    oracle = Backend(_load_oracle(), "oracle")
    spf = {}
    for seed in SPF_SEEDS:
        dbs = random_topology(seed)
        als, _ = load_topology(oracle, dbs, [])
        spf[str(seed)] = spf_table(als[A], sorted(db.thisNodeName for db in dbs))
    with open(os.path.join(HERE, "spf_random.json"), "w") as f:
        json.dump({"generator": "tests/test_gpu_parity.py:random_topology(seed)", "seeds": spf},
                  f, sort_keys=True, separators=(",", ":"))

    adj, pfx = bench_grid(10)
    als, ps = load_topology(oracle, adj, pfx)
    digests = {}
    full = None
    for i in range(100):
        me = str(i)
        db = oracle.spf_solver(me, True).build_route_db(me, als, ps)
        digests[me] = route_db_digest(db)
        if me == "1":
            full = route_db_json(db)
    with open(os.path.join(HERE, "route_db_c1.json"), "w") as f:
        json.dump({"generator": "openr_amd/topology.py:bench_grid(10)", "my_node_1": full,
                   "sha256_by_node": digests}, f, sort_keys=True, indent=0)


if __name__ == "__main__":
    main()
