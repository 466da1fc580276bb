"""Known-answer tests transcribed from openr/decision/tests/LinkStateTest.cpp.

Each test runs against the CPU oracle (``-m "not gpu"``) and against the HIP
product (``-m gpu``) through the same facade.
"""
import pytest

from openr_amd.topology import int_topology
from openr_amd.types import K_TESTING_AREA, create_adj_db, create_adjacency


def _ls(backend):
    return backend.area_link_states(K_TESTING_AREA)[K_TESTING_AREA]


def _feed(ls, dbs):
    for db in dbs:
        ls.update_adjacency_database(db)
    return ls


def _link_set(ls, node):
    return {(l.n1, l.if1, l.n2, l.if2) for l in ls.links_from_node(node)}


def test_link_state_basic_operation(backend):
    """LinkStateTest.BasicOperation (LinkStateTest.cpp:137-198)."""
    n1, n2, n3 = "node1", "node2", "node3"
    adj12 = create_adjacency(n2, "if2", "if1", "fe80::2", "10.0.0.2", 1, 1, 1)
    adj13 = create_adjacency(n3, "if3", "if1", "fe80::3", "10.0.0.3", 1, 1, 1)
    adj21 = create_adjacency(n1, "if1", "if2", "fe80::1", "10.0.0.1", 1, 1, 1)
    adj23 = create_adjacency(n3, "if3", "if2", "fe80::3", "10.0.0.3", 1, 1, 1)
    adj31 = create_adjacency(n1, "if1", "if3", "fe80::1", "10.0.0.1", 1, 1, 1)
    adj32 = create_adjacency(n2, "if2", "if3", "fe80::2", "10.0.0.2", 1, 1, 1)
    l1 = (n1, "if2", n2, "if1")
    l2 = (n2, "if3", n3, "if2")
    l3 = (n1, "if3", n3, "if1")
    db1 = create_adj_db(n1, [adj12, adj13], 1)
    db2 = create_adj_db(n2, [adj21, adj23], 2)
    db3 = create_adj_db(n3, [adj31, adj32], 3)
    ls = _ls(backend)
    assert not ls.update_adjacency_database(db1).topologyChanged
    assert ls.update_adjacency_database(db2).topologyChanged
    assert ls.update_adjacency_database(db3).topologyChanged
    assert _link_set(ls, n1) == {l1, l3}
    assert _link_set(ls, n2) == {l1, l2}
    assert _link_set(ls, n3) == {l2, l3}
    assert _link_set(ls, "node4") == set()

    assert not ls.is_node_overloaded(n1)
    db1.isOverloaded = True
    assert ls.update_adjacency_database(db1).topologyChanged
    assert ls.is_node_overloaded(n1)
    assert not ls.update_adjacency_database(db1).topologyChanged
    db1.isOverloaded = False
    assert ls.update_adjacency_database(db1).topologyChanged
    assert not ls.is_node_overloaded(n1)

    db1 = create_adj_db(n1, [adj13], 1)
    assert ls.update_adjacency_database(db1).topologyChanged
    assert _link_set(ls, n1) == {l3}
    assert _link_set(ls, n2) == {l2}
    assert _link_set(ls, n3) == {l2, l3}

    assert ls.delete_adjacency_database(n1).topologyChanged
    assert _link_set(ls, n1) == set()
    assert _link_set(ls, n2) == {l2}
    assert _link_set(ls, n3) == {l2}


def test_path_a_in_path_b(oracle_mod):
    """LinkStateTest.pathAInPathB (LinkStateTest.cpp:200-243)."""
    l1 = ("1", "1/2", "2", "2/1")
    l2 = ("2", "2/3", "3", "3/2")
    l3 = ("1", "1/3", "3", "3/1")
    f = oracle_mod.path_a_in_path_b
    p1, p2 = [], []
    assert f(p1, p2) and f(p2, p1)
    p1.append(l1)
    assert not f(p1, p2) and f(p2, p1)
    p2.append(l1)
    assert f(p1, p2) and f(p2, p1)
    p1.append(l2)
    assert not f(p1, p2) and f(p2, p1)
    p1.append(l3)
    p2.append(l2)
    assert not f(p1, p2) and f(p2, p1)
    p1, p2 = [l3, l2], [l1]
    assert not f(p1, p2) and not f(p2, p1)


def _path_cost(ls, path, start):
    node, cost = start, 0
    for link in path:
        cost += ls.metric_from_node(link, node)
        node = link.n2 if link.n1 == node else link.n1
    return cost


def test_get_kth_paths_weighted_box(backend, oracle_mod):
    """LinkStateTest.getKthPaths, first block (LinkStateTest.cpp:246-279)."""
    adj_map = {1: [(2, 10), (3, 5)], 2: [(1, 10), (4, 15), (4, 35)],
               3: [(1, 5), (4, 20)], 4: [(2, 15), (3, 20), (2, 35)]}
    order = oracle_mod.unordered_int_order(list(adj_map))
    ls = _feed(_ls(backend), int_topology(adj_map, order=order))
    first = ls.get_kth_paths("2", "4", 1)
    assert len(first) == 1 and len(first[0]) == 1
    assert ls.metric_from_node(first[0][0], "2") == 15
    second = ls.get_kth_paths("2", "4", 2)
    assert sorted(len(p) for p in second) == [1, 3]
    for p in second:
        assert _path_cost(ls, p, "2") == 35


def test_get_kth_paths_parallel_mesh(backend, oracle_mod):
    """LinkStateTest.getKthPaths, second block (LinkStateTest.cpp:281-316)."""
    adj_map = {1: [2, 2, 3, 3, 4, 4], 2: [1, 1, 3, 3, 4, 4],
               3: [1, 1, 2, 2, 4, 4], 4: [1, 1, 2, 2, 3, 3]}
    order = oracle_mod.unordered_int_order(list(adj_map))
    ls = _feed(_ls(backend), int_topology(adj_map, order=order))
    first = ls.get_kth_paths("2", "4", 1)
    assert len(first) == 2 and all(len(p) == 1 for p in first)
    second = ls.get_kth_paths("2", "4", 2)
    assert len(second) == 4 and all(len(p) == 2 for p in second)
    seen = set()
    for p in first + second:
        for link in p:
            assert link not in seen  # edge-disjoint across all paths
            seen.add(link)


@pytest.mark.parametrize("case", ["box", "line", "disconnected"])
def test_get_hop_counts(backend, oracle_mod, case):
    """LinkStateTest.getHopCounts (LinkStateTest.cpp:319-378)."""
    maps = {
        "box": {1: [2, 3], 2: [1, 4], 3: [1, 4], 4: [2, 3]},
        "line": {1: [2], 2: [1, 3], 3: [2, 4], 4: [3, 5], 5: [4]},
        "disconnected": {1: [2], 2: [1, 3], 3: [2, 4], 4: [3], 5: []},
    }
    adj_map = maps[case]
    order = oracle_mod.unordered_int_order(list(adj_map))
    ls = _feed(_ls(backend), int_topology(adj_map, order=order))
    if case == "box":
        assert ls.get_hops_from_a_to_b("1", "2") == 1
        assert ls.get_hops_from_a_to_b("1", "4") == 2
        assert ls.get_max_hops_to_node("1") == 2
    elif case == "line":
        assert ls.get_hops_from_a_to_b("1", "2") == 1
        assert ls.get_hops_from_a_to_b("1", "4") == 3
        assert ls.get_hops_from_a_to_b("2", "3") == 1
        assert ls.get_max_hops_to_node("1") == 4
        assert ls.get_max_hops_to_node("2") == 3
        assert ls.get_max_hops_to_node("3") == 2
    else:
        assert ls.get_hops_from_a_to_b("1", "5") is None
        assert ls.get_hops_from_a_to_b("2", "3") == 1
        assert ls.get_max_hops_to_node("1") == 3
        assert ls.get_max_hops_to_node("5") == 0
