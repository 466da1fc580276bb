"""Topology generators with the reference's naming, addressing and labels.

Each generator returns ``(adj_dbs, prefixes)``: a list of AdjacencyDatabase in
the order they are fed to ``LinkState.updateAdjacencyDatabase`` and a list of
``(node, area, PrefixEntry)`` advertisements.

  bench_grid      RoutingBenchmarkUtils.cpp:148-313 (createGrid, benchmark)
  unittest_grid       DecisionTest.cpp:4386-4443 (createGrid, unit tests)
  ring            DecisionTest.cpp:45-118, :1766-1856 (SimpleRingTopology)
  fabric          RoutingBenchmarkUtils.cpp:320-474 (createFabric)
  int_topology    DecisionTestUtils.cpp:17-56 (getLinkState)
  wan             build-defined seeded WAN for SURVEY config C4
"""
from __future__ import annotations

import math
import random
from typing import Dict, List, Sequence, Tuple

from .types import (K_TESTING_AREA, AdjacencyDatabase, Adjacency, BinaryAddress,
                    IpPrefix, PrefixEntry, PrefixForwardingAlgorithm,
                    PrefixForwardingType, PrefixType, create_adj_db,
                    create_adjacency, create_prefix_entry)


def _hex2(v: int) -> str:
    return f"{v:02x}"


# ---------------------------------------------------------------------------
# Benchmark grid (BM_DecisionGridInitialUpdate)
# ---------------------------------------------------------------------------

def bench_grid(n: int, num_prefixes: int = 1,
               algo: int = PrefixForwardingAlgorithm.SP_ECMP,
               area: str = K_TESTING_AREA):
    """n x n grid; node id = row*n + col, adjacency order right, left, up,
    down (RoutingBenchmarkUtils.cpp:229-269), unit metrics, adjLabel
    100001+neighbour, nodeLabel = id, one /128 per node per prefix index."""
    adj_dbs: List[AdjacencyDatabase] = []
    prefixes = []
    fwd_type = (PrefixForwardingType.SR_MPLS
                if algo == PrefixForwardingAlgorithm.KSP2_ED_ECMP
                else PrefixForwardingType.IP)
    for row in range(n):
        for col in range(n):
            node = row * n + col
            adjs = []
            for (r, c) in ((row, col + 1), (row, col - 1), (row - 1, col),
                           (row + 1, col)):
                if r < 0 or r >= n or c < 0 or c >= n:
                    continue
                other = r * n + c
                adjs.append(Adjacency(
                    str(other), f"if_{node}_{other}",
                    BinaryAddress.of(f"fe80:{_hex2(other >> 16)}::{_hex2(other & 0xffff)}"),
                    BinaryAddress.of(f"10.{other >> 16}.{(other >> 8) & 0xff}.{other & 0xff}"),
                    1, 100001 + other, False, 100, 10000, 1,
                    f"if_{other}_{node}"))
            adj_dbs.append(create_adj_db(str(node), adjs, node, False, area))
            for i in range(num_prefixes):
                pid = node + i
                pfx = IpPrefix.of(f"fc00:{_hex2(pid >> 16)}::{_hex2(pid & 0xffff)}/128")
                prefixes.append((str(node), area, create_prefix_entry(
                    pfx, PrefixType.LOOPBACK, fwd_type, algo)))
    return adj_dbs, prefixes


# ---------------------------------------------------------------------------
# Unit-test grid (GridTopologyFixture)
# ---------------------------------------------------------------------------

def unittest_grid_prefix(node: int) -> IpPrefix:
    """nodeToPrefixV6 (DecisionTest.cpp:4412-4415)."""
    return IpPrefix.of(f"::ffff:10.1.{node // 256}.{node % 256}/128")


def unittest_grid(n: int, area: str = K_TESTING_AREA):
    adj_dbs, prefixes = [], []

    def add(i, j, if_name, adjs, other_if):
        if i < 0 or i >= n or j < 0 or j >= n:
            return
        nb = i * n + j
        adjs.append(Adjacency(str(nb), if_name, BinaryAddress.of(f"fe80::{nb}"),
                              BinaryAddress.of(f"192.168.{nb // 256}.{nb % 256}"),
                              1, 100001 + nb, False, 100, 10000, 1, other_if))

    for i in range(n):
        for j in range(n):
            node = i * n + j
            adjs: List[Adjacency] = []
            add(i, j + 1, "0/1", adjs, "0/3")
            add(i - 1, j, "0/2", adjs, "0/4")
            add(i, j - 1, "0/3", adjs, "0/1")
            add(i + 1, j, "0/4", adjs, "0/2")
            adj_dbs.append(create_adj_db(str(node), adjs, node + 1, False, area))
            prefixes.append((str(node), area, create_prefix_entry(unittest_grid_prefix(node))))
    return adj_dbs, prefixes


# ---------------------------------------------------------------------------
# Four-node ring / mesh adjacencies of DecisionTest.cpp:45-85
# ---------------------------------------------------------------------------

def _adj(other, ifn, rif, nh6, nh4, metric, label):
    return create_adjacency(other, ifn, rif, nh6, nh4, metric, label)


RING_ADJ = {
    "adj12": lambda: _adj("2", "1/2", "2/1", "fe80::2", "192.168.0.2", 10, 100002),
    "adj13": lambda: _adj("3", "1/3", "3/1", "fe80::3", "192.168.0.3", 10, 100003),
    "adj14": lambda: _adj("4", "1/4", "4/1", "fe80::4", "192.168.0.4", 10, 100004),
    "adj21": lambda: _adj("1", "2/1", "1/2", "fe80::1", "192.168.0.1", 10, 100001),
    "adj23": lambda: _adj("3", "2/3", "3/2", "fe80::3", "192.168.0.3", 10, 100003),
    "adj24": lambda: _adj("4", "2/4", "4/2", "fe80::4", "192.168.0.4", 10, 100004),
    "adj31": lambda: _adj("1", "3/1", "1/3", "fe80::1", "192.168.0.1", 10, 100001),
    "adj32": lambda: _adj("2", "3/2", "2/3", "fe80::2", "192.168.0.2", 10, 100002),
    "adj34": lambda: _adj("4", "3/4", "4/3", "fe80::4", "192.168.0.4", 10, 100004),
    "adj41": lambda: _adj("1", "4/1", "1/4", "fe80::1", "192.168.0.1", 10, 100001),
    "adj42": lambda: _adj("2", "4/2", "2/4", "fe80::2", "192.168.0.2", 10, 100002),
    "adj43": lambda: _adj("3", "4/3", "3/4", "fe80::3", "192.168.0.3", 10, 100003),
}


def adj(name: str) -> Adjacency:
    return RING_ADJ[name]()


RING_ADDR_V6 = {i: IpPrefix.of(f"::ffff:10.{i}.{i}.{i}/128") for i in range(1, 5)}
RING_ADDR_V4 = {i: IpPrefix.of(f"10.{i}.{i}.{i}/32") for i in range(1, 5)}


def ring(v4: bool = False, area: str = K_TESTING_AREA, algo=None):
    """SimpleRingTopologyFixture::CustomSetUp (DecisionTest.cpp:1774-1856):
    1-2, 1-3, 2-4, 3-4 with metric 10; nodeLabel = node id."""
    adj_dbs = [
        create_adj_db("1", [adj("adj12"), adj("adj13")], 1, False, area),
        create_adj_db("2", [adj("adj21"), adj("adj24")], 2, False, area),
        create_adj_db("3", [adj("adj31"), adj("adj34")], 3, False, area),
        create_adj_db("4", [adj("adj42"), adj("adj43")], 4, False, area),
    ]
    addrs = RING_ADDR_V4 if v4 else RING_ADDR_V6
    prefixes = []
    for i in range(1, 5):
        e = create_prefix_entry(addrs[i])
        if algo == PrefixForwardingAlgorithm.KSP2_ED_ECMP:
            e.forwardingType = PrefixForwardingType.SR_MPLS
            e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
        prefixes.append((str(i), area, e))
    return adj_dbs, prefixes


# ---------------------------------------------------------------------------
# Integer-named topologies (DecisionTestUtils.cpp:17-56)
# ---------------------------------------------------------------------------

def int_topology(adj_map: Dict[int, Sequence], area: str = K_TESTING_AREA,
                 order: Sequence[int] = None) -> List[AdjacencyDatabase]:
    """getLinkState(adjMap): entries are neighbour ids or (neighbour, metric);
    parallel adjacencies get ifName "{node}/{adj}/{k}"; adjLabel is
    (node << 16) + adj; nodeLabel is the node id.  ``order`` gives the
    sequence of updateAdjacencyDatabase calls (the reference iterates an
    std::unordered_map<int, ...>)."""
    dbs = []
    for node in (order if order is not None else adj_map.keys()):
        adjs = []
        num_parallel: Dict[int, int] = {}
        for ent in adj_map[node]:
            nb, w = (ent if isinstance(ent, tuple) else (ent, 1))
            k = num_parallel.get(nb, 0)
            num_parallel[nb] = k + 1
            lo, hi = nb & 0xFF, (nb & 0xFF00) >> 8
            adjs.append(create_adjacency(
                str(nb), f"{node}/{nb}/{k}", f"{nb}/{node}/{k}",
                f"fe80::{hi:02x}{lo:02x}", f"192.168.{hi}.{lo}", w,
                (node << 16) + nb))
        dbs.append(create_adj_db(str(node), adjs, node, False, area))
    return dbs


# ---------------------------------------------------------------------------
# Clos fabric (BM_DecisionFabric)
# ---------------------------------------------------------------------------

SSW, FSW, RSW = 1, 2, 3
SSWS_PER_PLANE, FSWS_PER_POD, RSWS_PER_POD = 36, 8, 48


def fabric_pods(num_nodes: int) -> int:
    """numOfPods = (numOfGivenNodes - numOfSsws) / numOfFswsAndRswsPerPod
    (DecisionBenchmark.cpp:80-86)."""
    return (num_nodes - SSWS_PER_PLANE * FSWS_PER_POD) // (FSWS_PER_POD + RSWS_PER_POD)


def _fname(marker, pod, sw):
    return f"{marker}-{pod}-{sw}"


def _fabric_adj(src: str, marker: int, pod: int, sw: int) -> Adjacency:
    other = _fname(marker, pod, sw)
    return Adjacency(
        other, f"if_{src}_{other}",
        BinaryAddress.of(f"fe80:{_hex2(marker)}:{_hex2(pod)}::{_hex2(sw)}"),
        BinaryAddress.of(f"{marker}.{pod >> 8}.{pod & 0xff}.{sw}"),
        1, marker * 100000 + pod * 100 + sw, False, 100, 10000, 1,
        f"if_{other}_{src}")


def fabric(num_nodes: int, bug_compatible: bool = True,
           area: str = K_TESTING_AREA):
    """3-tier Clos. With ``bug_compatible`` each spine keeps only its pod-0
    adjacency, exactly as createSswsAdjacencies' repeated
    unordered_map::emplace on one key does (RoutingBenchmarkUtils.cpp:329-348);
    otherwise every spine connects to its plane's FSW in every pod.
    nodeLabel is 0 (createAdjValue, RoutingBenchmarkUtils.h:120-138)."""
    pods = fabric_pods(num_nodes)
    planes = FSWS_PER_POD
    dbs = []
    for plane in range(planes):
        for s in range(SSWS_PER_PLANE):
            name = _fname(SSW, plane, s)
            pod_list = [0] if bug_compatible else range(pods)
            adjs = [_fabric_adj(name, FSW, pod, plane) for pod in pod_list]
            dbs.append(create_adj_db(name, adjs, 0, False, area))
    for pod in range(pods):
        for f in range(FSWS_PER_POD):
            name = _fname(FSW, pod, f)
            adjs = [_fabric_adj(name, SSW, f, s) for s in range(SSWS_PER_PLANE)]
            adjs += [_fabric_adj(name, RSW, pod, r) for r in range(RSWS_PER_POD)]
            dbs.append(create_adj_db(name, adjs, 0, False, area))
    for pod in range(pods):
        for r in range(RSWS_PER_POD):
            name = _fname(RSW, pod, r)
            adjs = [_fabric_adj(name, FSW, pod, f) for f in range(FSWS_PER_POD)]
            dbs.append(create_adj_db(name, adjs, 0, False, area))
    return dbs, []


# ---------------------------------------------------------------------------
# Ladder (deep BFS: every level count the device level encoding can hold)
# ---------------------------------------------------------------------------

def ladder(length: int, metric: int = 1, area: str = K_TESTING_AREA):
    """Two rails a0..a{length-1}, b0..b{length-1} with rungs a_i-b_i; every
    link has the same metric, so the BFS depth from one end is ~length."""
    adjs: Dict[str, List[Adjacency]] = {}

    def link(x, y):
        for (p, q) in ((x, y), (y, x)):
            adjs.setdefault(p, []).append(Adjacency(
                q, f"{p}>{q}", BinaryAddress.of("fe80::1"), BinaryAddress.of("10.0.0.1"),
                metric, 0, False, 0, 0, 1, f"{q}>{p}"))

    for i in range(length):
        link(f"a{i}", f"b{i}")
        if i + 1 < length:
            link(f"a{i}", f"a{i + 1}")
            link(f"b{i}", f"b{i + 1}")
    return [create_adj_db(n, a, 0, False, area) for n, a in adjs.items()], []


# ---------------------------------------------------------------------------
# Seeded WAN
# ---------------------------------------------------------------------------

def wan(num_nodes: int, mean_degree: float = 4.0, seed: int = 4,
        area: str = K_TESTING_AREA):
    """Connected random graph: a random spanning tree plus extra random links
    up to ``mean_degree``; metrics log-normal(ln 100, 1.5) clipped to
    [1, 65535], independent per direction."""
    rng = random.Random(seed)
    links = set()
    order = list(range(num_nodes))
    rng.shuffle(order)
    for i in range(1, num_nodes):
        a, b = order[i], order[rng.randrange(i)]
        links.add((min(a, b), max(a, b)))
    target = int(num_nodes * mean_degree / 2)
    while len(links) < target:
        a, b = rng.randrange(num_nodes), rng.randrange(num_nodes)
        if a != b:
            links.add((min(a, b), max(a, b)))

    def metric():
        return int(min(65535, max(1, round(rng.lognormvariate(math.log(100), 1.5)))))

    adjs: Dict[int, List[Adjacency]] = {i: [] for i in range(num_nodes)}
    for a, b in sorted(links):
        for (x, y) in ((a, b), (b, a)):
            adjs[x].append(Adjacency(
                f"w{y}", f"w{x}-w{y}", BinaryAddress.of(f"fe80::{x:x}:{y:x}"),
                BinaryAddress.of(f"10.{(y >> 16) & 255}.{(y >> 8) & 255}.{y & 255}"),
                metric(), 0, False, 0, 0, 1, f"w{y}-w{x}"))
    dbs = [create_adj_db(f"w{i}", adjs[i], i + 1, False, area)
           for i in range(num_nodes)]
    return dbs, []
