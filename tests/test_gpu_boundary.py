"""The drop-in boundary's reference-shaped SPF result (``-m gpu``).

``openr_amd::LinkState::getSpfResult(node, useLinkMetric)`` returns the
reference's ``SpfResult`` shape (LinkState.h:203-272): reachable node name ->
NodeSpfResult{metric, nextHops, pathLinks in the reference's order}, memoized
until a topology change. It must equal the oracle's runSpf result and the row
form the route build reads (getSpfRow), before and after mutations.
"""
import copy

import pytest

from openr_amd.facade import NodeSpfResult, load_topology
from openr_amd.types import K_TESTING_AREA

from test_gpu_parity import random_topology

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA


def _oracle_view(ls, node, metric):
    return {k: (v.metric, v.nextHops, list(v.pathLinks))
            for k, v in ls.get_spf_result(node, metric).items()}


def _ref_view(ls, node, metric):
    raw = ls._impl.get_spf_result_ref(node, metric)
    return {k: (r.metric, r.nextHops, r.pathLinks)
            for k, r in ((k, NodeSpfResult(*v)) for k, v in raw.items())}


@pytest.mark.parametrize("seed", range(4))
def test_spf_result_reference_shape(hip, oracle, seed):
    dbs = random_topology(4000 + seed, parallel=0.3)
    als_h, _ = load_topology(hip, dbs, [])
    als_o, _ = load_topology(oracle, dbs, [])
    names = sorted(db.thisNodeName for db in dbs)
    for step in range(2):
        for nm in names + ["unknown-node"]:
            for metric in (True, False):
                ref = _ref_view(als_h[A], nm, metric)
                assert ref == _oracle_view(als_o[A], nm, metric), (seed, step, nm, metric)
                assert ref == _oracle_view(als_h[A], nm, metric), (seed, step, nm, metric)
        # a topology change invalidates the memo: drop a node's adjacencies
        db = copy.deepcopy(next(d for d in dbs if d.thisNodeName == names[step]))
        db.adjacencies = db.adjacencies[1:]
        for ls in (als_h[A], als_o[A]):
            ls.update_adjacency_database(copy.deepcopy(db))
