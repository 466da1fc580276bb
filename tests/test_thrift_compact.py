"""Thrift Compact wire format of the Decision path.

The product's C++ codec (openr_amd/csrc/host/thrift_compact.cpp) writes
thrift::RouteDatabase / RouteDatabaseDelta (Types.thrift:1003-1060,
Network.thrift:48-131) and reads AdjacencyDatabase / PrefixDatabase /
Publication (Types.thrift:74-180, :350-460, :555-605, :897-936). Pins:
  - hand-derived known-answer bytes from the Compact protocol specification
    (field-id deltas, the long field header for id 51, zigzag varints,
    list headers, bool in the field header);
  - an independent schema-less Python decoder (tests/compact_decode.py)
    reading the product's bytes of route databases built by the oracle;
  - encode -> decode round trips of the KvStore-side structs.
These are host-code tests (no GPU): the oracle builds the route databases.
"""
import random

import pytest

from compact_decode import decode
from openr_amd import host_module
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import (BinaryAddress, IpPrefix, K_TESTING_AREA, PrefixForwardingAlgorithm,
                             PrefixForwardingType, PrefixMetrics, create_prefix_entry)

from test_gpu_parity import random_topology


@pytest.fixture(scope="module")
def mod():
    return host_module()


def _nh_wire(addr, ifname, metric, area=None, nbr=None, weight=0, mpls=None):
    return (addr, ifname, weight, mpls, metric, area, nbr)


def test_route_database_known_bytes(mod):
    """Hand-encoded from the Compact spec (see the comments per byte run)."""
    empty = (([], []))
    assert mod.route_db_thrift(empty, "a") == bytes.fromhex(
        "18 01 61"      # 1: string thisNodeName = "a"
        "39 0c"         # 4: list<UnicastRoute>, 0 elements
        "19 0c"         # 5: list<MplsRoute>, 0 elements
        "00")
    nh = _nh_wire(bytes([10, 0, 0, 1]), "eth0", 1, "A", "n1")
    route = (bytes([10, 0, 0, 0]), 8, [nh], False, "A", None)
    assert mod.route_db_thrift(([route], []), "a") == bytes.fromhex(
        "18 01 61"
        "39 1c"                         # 4: list, 1 struct
        "1c"                            #   UnicastRoute 1: IpPrefix dest
        "1c 18 04 0a000000 00"          #     1: BinaryAddress{1: addr}
        "14 10 00"                      #     2: i16 prefixLength = 8 (zigzag 16)
        "39 1c"                         #   4: list<NextHopThrift>, 1 struct
        "1c 18 04 0a000001 28 04 65746830 00"  # 1: BinaryAddress{1: addr, 3: ifName "eth0"}
        "15 00"                         #     2: i32 weight = 0
        "05 66 02"                      #     51: i32 metric = 1 (long header: id 51 zigzag = 0x66)
        "28 01 41"                      #     53: string area = "A"
        "18 02 6e31"                    #     54: string neighborNodeName = "n1"
        "00"
        "32"                            #   7: bool doNotInstall = false
        "00"
        "19 0c"
        "00")
    # MPLS route with a PUSH action (Network.thrift:48-54): label 100001 zigzag 200002
    push = (0, None, (16001, 16002))
    mnh = _nh_wire(bytes(16), "eth1", 0, None, None, mpls=push)
    got = mod.route_db_thrift(([], [(100001, [mnh])]), "")
    assert got == bytes.fromhex(
        "18 00" "39 0c"
        "19 1c"                         # 5: list<MplsRoute>, 1 struct
        "15 c29a0c"                     #   1: i32 topLabel = 100001
        "39 1c"                         #   4: list<NextHopThrift>
        "1c 18 10" + "00" * 16 + "28 04 65746831 00"
        "15 00"
        "1c 15 00 29 25 82fa01 84fa01 00"  # 3: MplsAction{1: PUSH, 3: list<i32>[16001, 16002]}
        "05 66 00"                      #   51: metric 0
        "00"                            # end NextHopThrift
        "00"                            # end MplsRoute
        "00")


def test_prefix_key_parse(mod):
    """PrefixKey::fromStr (Types.cpp:57-77, getPrefixRE2 Types.h:354-362)."""
    assert mod.parse_prefix_key("prefix:node-1:area.0:[fc00:1::/64]") == \
        ("node-1", "area.0", bytes.fromhex("fc000001000000000000000000000000"), 64)
    assert mod.parse_prefix_key("prefix:n:a:[10.1.2.3/16]") == ("n", "a", bytes([10, 1, 0, 0]), 16)
    for bad in ("prefix:n:a:10.0.0.0/8", "adj:n", "prefix:n:a:[10.0.0.0/33]", "prefix:n:[10.0.0.0/8]"):
        assert mod.parse_prefix_key(bad) is None, bad


def _expect_unicast(w):
    addr, plen, nhs, dni, _best_area, best = w
    out = {1: {1: {1: addr}, 2: plen}, 4: sorted((_expect_nh(n) for n in nhs), key=repr), 7: dni}
    if best is not None and best[2] == 3:  # BGP: prefixType + data (RibEntry.h:83-88)
        out[5] = 3
        if best[9] is not None:
            out[6] = best[9]
    return out


def _expect_nh(n):
    addr, ifname, weight, mpls, metric, area, nbr = n
    d = {1: {1: addr} | ({3: ifname.encode()} if ifname is not None else {}), 2: weight, 51: metric}
    if mpls is not None:
        act, swap, push = mpls
        d[3] = {1: act} | ({2: swap} if swap is not None else {}) | \
            ({3: list(push)} if push is not None else {})
    if area is not None:
        d[53] = area.encode()
    if nbr is not None:
        d[54] = nbr.encode()
    return d


def _check_db_bytes(mod, wire, me):
    data = mod.route_db_thrift(wire, me)
    got = decode(data)
    assert got[1] == me.encode()
    ucast = [_expect_unicast(w) for w in wire[0]]
    exp_u = sorted(ucast, key=lambda d: (d[1][1][1], d[1][2]))
    got_u = got[4]
    assert [(g[1][1][1], g[1][2]) for g in got_u] == [(e[1][1][1], e[1][2]) for e in exp_u]
    for g, e in zip(got_u, exp_u):
        assert sorted(g[4], key=repr) == e[4]
        assert {k: v for k, v in g.items() if k != 4} == {k: v for k, v in e.items() if k != 4}
    exp_m = sorted(wire[1], key=lambda m: m[0])
    assert [m[1] for m in got[5]] == [m[0] for m in exp_m]
    for g, (label, nhs) in zip(got[5], exp_m):
        assert sorted(g[4], key=repr) == sorted((_expect_nh(n) for n in nhs), key=repr)
    assert mod.route_db_thrift(wire, me) == data  # deterministic
    return data


def test_route_db_bytes_grid(mod, oracle):
    """Every route of the C1 grid's route DB (SP_ECMP + node / adj labels),
    decoded independently."""
    dbs, pfx = bench_grid(10, 2)
    als, ps = load_topology(oracle, dbs, pfx)
    wire = oracle.spf_solver("1", True)._impl.build_route_db("1", als._impl, ps._impl)
    data = _check_db_bytes(mod, wire, "1")
    assert len(decode(data)[4]) == len(wire[0]) > 0


@pytest.mark.parametrize("seed", range(3))
def test_route_db_bytes_random(mod, oracle, seed):
    """Random anycast topologies with SR_MPLS / KSP2 prefixes, drained nodes
    and parallel links: nexthops with PUSH / SWAP / PHP actions."""
    dbs = random_topology(5000 + seed, n=20, extra=30)
    rng = random.Random(seed)
    pfx = []
    for i in range(40):
        for db in rng.sample(dbs, rng.randint(1, 3)):
            e = create_prefix_entry(IpPrefix.of(f"fc00:{seed}::{i:x}/128"))
            if rng.random() < 0.4:
                e.forwardingType = PrefixForwardingType.SR_MPLS
                if rng.random() < 0.5:
                    e.forwardingAlgorithm = PrefixForwardingAlgorithm.KSP2_ED_ECMP
            pfx.append((db.thisNodeName, K_TESTING_AREA, e))
    als, ps = load_topology(oracle, dbs, pfx)
    me = sorted(db.thisNodeName for db in dbs)[seed]
    wire = oracle.spf_solver(me, True)._impl.build_route_db(me, als._impl, ps._impl)
    _check_db_bytes(mod, wire, me)


def test_route_delta_bytes(mod, oracle):
    """calculateUpdate between two builds, as thrift::RouteDatabaseDelta."""
    dbs, pfx = bench_grid(6, 1)
    als, ps = load_topology(oracle, dbs, pfx)
    solver = oracle.spf_solver("1", True)._impl
    old = solver.build_route_db("1", als._impl, ps._impl)
    victim = next(d for d in dbs if d.thisNodeName == "7")
    victim.adjacencies = victim.adjacencies[1:]
    als[K_TESTING_AREA].update_adjacency_database(victim)
    ps.delete_prefix("20", K_TESTING_AREA, pfx[20][2].prefix)
    new = solver.build_route_db("1", als._impl, ps._impl)
    delta = mod.calculate_update(old, new)
    got = decode(mod.route_delta_thrift(old, new))
    uu, ud, mu, md = delta
    assert sorted((g[1][1][1], g[1][2]) for g in got[2]) == sorted((u[0], u[1]) for u in uu)
    assert sorted((g[1][1], g[2]) for g in got[3]) == sorted((a, l) for a, l in ud)
    assert [m[1] for m in got[4]] == sorted(m[0] for m in mu)
    assert got[5] == sorted(md)
    assert len(ud) == 1 and len(uu) > 0


def test_adjacency_database_round_trip(mod):
    dbs, _ = bench_grid(4, 0)
    for db in dbs:
        w = db.to_wire()
        data = mod.adj_db_to_compact(w)
        assert mod.adj_db_from_compact(data) == w
        d = decode(data)
        assert d[1] == db.thisNodeName.encode() and len(d[3]) == len(db.adjacencies)
        assert [a[4] for a in d[3]] == [a.metric for a in db.adjacencies]


def test_prefix_database_round_trip(mod):
    rng = random.Random(3)
    for i in range(20):
        e = create_prefix_entry(IpPrefix.of(f"fd00:{i:x}::/64" if i % 2 else f"10.{i}.0.0/16"))
        e.metrics = PrefixMetrics(1, rng.randrange(1000), rng.randrange(1000), rng.randrange(10))
        w = e.to_wire()
        stacks = [["A", "B"]] if i % 3 == 0 else []
        data = mod.prefix_db_to_compact(f"n{i}", "A", [w], i % 4 == 0, stacks)
        node, area, entries, delete, got_stacks = mod.prefix_db_from_compact(data)
        assert (node, area, delete) == (f"n{i}", "A", i % 4 == 0)
        assert entries == [w] and got_stacks == (stacks or [[]])
    with pytest.raises(ValueError):
        mod.prefix_db_from_compact(b"\x18\x05ab")  # truncated


# ---- hostile input (the decoders run on peer-supplied publication bytes) ----

def _insert_before_stop(data, extra):
    assert data[-1:] == b"\x00"
    return data[:-1] + extra + b"\x00"


def test_oversized_counts_rejected_before_allocation(mod):
    """A list / map count beyond the remaining bytes is a decode error, not a
    multi-GB container reservation (fbthrift rejects it the same way)."""
    huge = b"\xff\xff\xff\xff\x0f"  # varint 2^32 - 1
    with pytest.raises(ValueError, match="beyond the input"):
        mod.prefix_db_from_compact(b"\x18\x01a" + b"\x29\xfc" + huge)  # prefixEntries: list<struct>
    with pytest.raises(ValueError, match="beyond the input"):
        mod.adj_db_from_compact(b"\x18\x01a" + b"\x29\xfc" + huge)  # adjacencies
    db = bench_grid(2, 0)[0][0]
    data = mod.adj_db_to_compact(db.to_wire())
    with pytest.raises(ValueError, match="beyond the input"):  # unknown map field, huge count
        mod.adj_db_from_compact(_insert_before_stop(data, b"\xeb" + huge + b"\x51"))
    pub = mod.publication_to_compact("A", {"k": (1, "o", b"v", 10, 1)}, ["x"])
    assert mod.publication_from_compact(pub) == ("A", {"k": (1, "o", b"v", 10, 1)}, ["x"])
    with pytest.raises(ValueError):
        mod.publication_from_compact(b"\x2b" + huge + b"\x8c")  # keyVals map<string, Value>


def test_nesting_depth_limited(mod):
    db = bench_grid(2, 0)[0][0]
    data = mod.adj_db_to_compact(db.to_wire())
    deep = b"\xec" + b"\x1c" * 200 + b"\x00" * 201  # unknown field 20: 201 nested structs
    with pytest.raises(ValueError, match="nesting"):
        mod.adj_db_from_compact(_insert_before_stop(data, deep))
    shallow = b"\xec" + b"\x1c" * 8 + b"\x00" * 9
    assert mod.adj_db_from_compact(_insert_before_stop(data, shallow)) == db.to_wire()


@pytest.mark.parametrize("kind", ["list", "map"])
def test_container_nesting_depth_limited(mod, kind):
    """Unknown fields of nested lists (one byte per level) or maps (three
    bytes per level) are bounded like nested structs: a peer cannot drive
    skip() into unbounded recursion."""
    db = bench_grid(2, 0)[0][0]
    data = mod.adj_db_to_compact(db.to_wire())

    def nested(levels):
        if kind == "list":  # field 20 list<list<...<list<>>>>: one element per level
            return b"\xe9" + b"\x19" * levels + b"\x09"
        return b"\xeb" + b"\x01\x5b\x02" * levels + b"\x00"  # map<i32, map<...>>: {1: ...}

    with pytest.raises(ValueError, match="nesting"):
        mod.adj_db_from_compact(_insert_before_stop(data, nested(1_000_000)))
    assert mod.adj_db_from_compact(_insert_before_stop(data, nested(8))) == db.to_wire()


def test_skip_map_of_bools(mod):
    """An unknown map<i32, bool> field: each bool is a one-byte value, so the
    fields after it must still decode."""
    db = bench_grid(2, 0)[0][0]
    w = db.to_wire()
    data = mod.adj_db_to_compact(w)
    m = b"\xeb" + b"\x02\x51" + b"\x02\x01" + b"\x04\x02"  # field 20 map<i32,bool>{1: true, 2: false}
    assert mod.adj_db_from_compact(_insert_before_stop(data, m)) == w
    # an unknown scalar field after the map
    assert mod.adj_db_from_compact(_insert_before_stop(data, b"\xe5\x06")) == w  # field 20 i32 3


def test_malformed_prefix_rejected(mod):
    """toIPNetwork throws on an address that is neither 4 nor 16 bytes or a
    length outside [0, 8 * size]; the entry is a decode error."""
    for addr, length in ((bytes(16), 129), (bytes(4), 33), (bytes(16), -1), (bytes(5), 8)):
        e = create_prefix_entry(IpPrefix.of("fd00::/64"))
        e.prefix = IpPrefix(BinaryAddress(addr), length)
        data = mod.prefix_db_to_compact("n", "A", [e.to_wire()])
        with pytest.raises(ValueError, match="malformed prefix"):
            mod.prefix_db_from_compact(data)
