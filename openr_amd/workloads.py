"""Benchmark workloads of BASELINE.json's configs.

  C1  createGrid(10, 1 prefix, SP_ECMP)                      topology.bench_grid(10)
  C2  createGrid(100): all-sources SPF                       topology.bench_grid(100)
  C3  3-tier Clos of ~2.5k nodes (full spine mesh) + 100k /64s over the
      RSWs (~54 each) and a seeded 5% anycast subset (2-8 advertisers),
      default and best-route selection                       c3_fabric()
  C4  50k-node WAN, log-normal metrics: single-link what-if SPFs and KSP2
      (src, dst) pairs                                       c4_wan()
  C5  4 areas x ~2.5k nodes, myNode in all four, 1M prefixes with random
      PrefixMetrics, best-route selection, RibPolicy area weights
                                                             c5_multi_area()
All seeded; nothing is read from disk.
"""
from __future__ import annotations

import random
from typing import List, Tuple

from .topology import _hex2, bench_grid, fabric, wan
from .types import (K_TESTING_AREA, Adjacency, BinaryAddress, IpPrefix, PrefixEntry,
                    PrefixMetrics, PrefixType, create_adj_db)

C3_SEED, C4_SEED, C5_SEED = 3003, 4004, 5005
# C4 batch shape (SURVEY.md §8d / BASELINE.md): 4,096 sampled links x 64
# sources of runSpf(src, true, {link}), and 1,024 KSP2 (src, dst) pairs
C4_WHATIF_LINKS, C4_WHATIF_SRCS, C4_KSP2_PAIRS = 4096, 64, 1024
# requests per what-if run: two alternating device row buffers of
# CHUNK x N x 8 bytes (2 x 26 GB at N = 50,000 of the 288 GB HBM), so the
# large repairs of one chunk overlap the next chunk's copy
C4_WHATIF_CHUNK = 65536


def _metrics(rng):
    return PrefixMetrics(1, rng.randint(0, 3), rng.randint(0, 3), rng.randint(0, 3))


def c3_fabric(num_nodes: int = 2500, num_prefixes: int = 100_000, anycast: float = 0.05,
              seed: int = C3_SEED, area: str = K_TESTING_AREA):
    """Full-mesh Clos (N = 2,472 at 2,500) + prefixes (node, area, entry)."""
    adj_dbs, _ = fabric(num_nodes, bug_compatible=False, area=area)
    rsws = [db.thisNodeName for db in adj_dbs if db.thisNodeName.startswith("3-")]
    rng = random.Random(seed)
    prefixes = []
    for i in range(num_prefixes):
        addr = BinaryAddress(bytes([0xfd, 0x00, (i >> 24) & 255, (i >> 16) & 255,
                                    (i >> 8) & 255, i & 255, 0, 0] + [0] * 8))
        p = IpPrefix(addr, 64)
        if rng.random() < anycast:
            owners = rng.sample(rsws, rng.randint(2, 8))
        else:
            owners = [rsws[i % len(rsws)]]
        for o in owners:
            prefixes.append((o, area, PrefixEntry(p, PrefixType.LOOPBACK,
                                                  metrics=_metrics(rng))))
    return adj_dbs, prefixes


C2W_SEED, C2W_MAX_METRIC = 2002, 64


def c2_weighted_grid(n: int = 100, max_metric: int = C2W_MAX_METRIC, seed: int = C2W_SEED):
    """C2 with integer metrics (the weighted all-sources leg): the benchmark
    grid createGrid(n) (topology.bench_grid) with every link given a seeded
    metric uniform in [1, max_metric], the same in both directions (an IGP
    cost per link). Returns (adj_dbs, prefixes) like bench_grid."""
    adj_dbs, prefixes = bench_grid(n, 1)
    rng = random.Random(seed)
    metric = {}
    for db in adj_dbs:
        a = int(db.thisNodeName)
        for adj in db.adjacencies:
            b = int(adj.otherNodeName)
            key = (min(a, b), max(a, b))
            if key not in metric:
                metric[key] = rng.randint(1, max_metric)
            adj.metric = metric[key]
    return adj_dbs, prefixes


def c4_wan(num_nodes: int = 50_000, seed: int = C4_SEED):
    return wan(num_nodes, seed=seed)


def c4_what_if_pairs(link_ids: List[int], node_names: List[str], n_links: int, n_srcs: int,
                     seed: int = C4_SEED) -> List[Tuple[str, int]]:
    """(source, ignored link) pairs: n_links sampled links x n_srcs sampled sources."""
    rng = random.Random(seed + 1)
    links = rng.sample(link_ids, min(n_links, len(link_ids)))
    srcs = rng.sample(node_names, min(n_srcs, len(node_names)))
    return [(s, l) for l in links for s in srcs]


def c4_what_if_job(link_ids: List[int], node_names: List[str], n_links: int = C4_WHATIF_LINKS,
                   n_srcs: int = C4_WHATIF_SRCS, seed: int = C4_SEED):
    """The same (source, link) requests as c4_what_if_pairs, as a what-if job:
    (sources, per request its source index, per request its ignore set)."""
    rng = random.Random(seed + 1)
    links = rng.sample(link_ids, min(n_links, len(link_ids)))
    srcs = rng.sample(node_names, min(n_srcs, len(node_names)))
    idx = [i for _ in links for i in range(len(srcs))]
    sets = [[l] for l in links for _ in srcs]
    return srcs, idx, sets


def c4_ksp2_pairs(node_names: List[str], n_pairs: int, seed: int = C4_SEED):
    rng = random.Random(seed + 2)
    out = []
    while len(out) < n_pairs:
        a, b = rng.sample(node_names, 2)
        out.append((a, b))
    return out


C5_AREAS = ("A", "B", "C", "D")
C5_TAG = "C5:UCMP"  # every C5 prefix carries it; the RibPolicy statement matches on it


def c5_multi_area(side: int = 50, num_prefixes: int = 1_000_000, seed: int = C5_SEED,
                  me: str = "me"):
    """Four grid areas of side x side nodes (2,500 at side 50); `me` is in all
    four, attached to one corner node of each grid (metric 1). Prefixes are
    /64s spread over all nodes with random PrefixMetrics; 5% anycast across
    areas. Returns ({area: adj_dbs}, prefixes)."""
    rng = random.Random(seed)
    areas = {}
    names_by_area = {}
    for ai, area in enumerate(C5_AREAS):
        dbs, _ = bench_grid(side, 0, area=area)
        # rename nodes per area so areas do not share node names (except me)
        ren = {db.thisNodeName: f"{area}{db.thisNodeName}" for db in dbs}
        for db in dbs:
            db.thisNodeName = ren[db.thisNodeName]
            for adj in db.adjacencies:
                adj.otherNodeName = ren[adj.otherNodeName]
            db.nodeLabel = (ai + 1) * 10000 + db.nodeLabel
        corner = dbs[0]
        up = Adjacency(corner.thisNodeName, f"me-{area}", BinaryAddress.of(f"fe80::{ai + 1}:1"),
                       BinaryAddress.of(f"10.250.{ai}.1"), 1, 0, False, 100, 10000, 1,
                       f"{corner.thisNodeName}-me")
        down = Adjacency(me, f"{corner.thisNodeName}-me", BinaryAddress.of(f"fe80::{ai + 1}:2"),
                         BinaryAddress.of(f"10.250.{ai}.2"), 1, 0, False, 100, 10000, 1,
                         f"me-{area}")
        corner.adjacencies.append(down)
        dbs.append(create_adj_db(me, [up], 1, False, area))
        areas[area] = dbs
        names_by_area[area] = [db.thisNodeName for db in dbs if db.thisNodeName != me]
    prefixes = []
    for i in range(num_prefixes):
        addr = BinaryAddress(bytes([0xfc, 0x05, (i >> 24) & 255, (i >> 16) & 255,
                                    (i >> 8) & 255, i & 255, 0, 0] + [0] * 8))
        p = IpPrefix(addr, 64)
        if rng.random() < 0.05:
            owners = [(a, rng.choice(names_by_area[a])) for a in rng.sample(C5_AREAS, 2)]
        else:
            a = C5_AREAS[i % 4]
            owners = [(a, names_by_area[a][(i // 4) % len(names_by_area[a])])]
        for a, o in owners:
            prefixes.append((o, a, PrefixEntry(p, metrics=_metrics(rng), tags=(C5_TAG,))))
    return areas, prefixes
