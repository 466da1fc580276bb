"""Parity at the configs' full sizes against the independent fast checker
(oracle/src/oracle_fast.h, validated against the faithful oracle in
tests/test_oracle_fast.py), where the faithful oracle (~1 SPF/s on the 50k
WAN) can only pin samples:

  C4 KSP2     all 1,024 benched (src, dst) pairs: getKthPaths k = 1 and 2,
              link by link, in order (LinkState.cpp:762-791, :398-419)
  C4 what-if  the benched 262,144-request job as the bench runs it
              (copy-on-write): every request's row digest (orh_row_digest) from
              the device, and >= 4,096 of them - every request of tiers 2-4 plus
              a seeded sample of tiers 0 and 1 - recomputed by the checker
              (runSpf(src, true, {link}), LinkState.cpp:808-882)
  C3 sweep    all 2,472 all-sources rows of the Clos fabric, dist and first hops
"""
import random

import numpy as np
import pytest

from openr_amd.facade import LinkDesc, load_topology
from openr_amd.types import K_TESTING_AREA

pytestmark = pytest.mark.gpu
A = K_TESTING_AREA
THREADS = 16


def _c4(hip, oracle):
    from openr_amd.workloads import c4_wan
    adj, _ = c4_wan()
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    names = ls.node_names()
    als_o, _ = load_topology(oracle, adj, [])
    fc = oracle.module.FastChecker(als_o[A]._impl, names)
    return adj, ls, names, fc


@pytest.fixture(scope="module")
def c4(hip, oracle):
    return _c4(hip, oracle)


def test_c4_ksp2_all_benched_pairs(c4):
    from openr_amd.workloads import C4_KSP2_PAIRS, c4_ksp2_pairs
    adj, ls, names, fc = c4
    kp = c4_ksp2_pairs(names, C4_KSP2_PAIRS)
    ls.prefetch_kth_paths(kp)  # the bench's call: one device batch
    dev, host = ls.ksp_stats()
    assert dev >= 0.9 * len(kp)
    ids = {n: i for i, n in enumerate(names)}
    want = fc.kth_paths([(ids[s], ids[d]) for s, d in kp], THREADS)
    bad = []
    for (s, d), (k1, k2) in zip(kp, want):
        for k, paths in ((1, k1), (2, k2)):
            got = [[LinkDesc(*l) for l in p] for p in ls.get_kth_paths(s, d, k)]
            if got != [[LinkDesc(*l) for l in p] for p in paths]:
                bad.append((s, d, k))
    assert not bad, f"{len(bad)} of {2 * len(kp)} path lists differ, first {bad[:3]}"
    # non-trivial: every pair has a first path and most have a second
    assert all(k1 for k1, _ in want) and sum(1 for _, k2 in want if k2) > 0.8 * len(kp)


def test_c4_what_if_job_vs_checker(c4):
    from openr_amd.workloads import C4_WHATIF_CHUNK, c4_what_if_job
    adj, ls, names, fc = c4
    links = dict(ls.link_ids())
    srcs, idx, sets = c4_what_if_job(list(links), names)
    job = ls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=True)
    job.set_digests()
    job.run()
    job.sync()
    info, dig = job.info(), job.digests()
    del job
    tier = info & 7
    rng = random.Random(505)
    heavy = [int(i) for i in np.nonzero(tier >= 2)[0]]
    light = [int(i) for i in np.nonzero(tier <= 1)[0]]
    pick = sorted(set(heavy + rng.sample(light, max(0, 4096 - len(heavy)))))
    assert len(pick) >= 4096
    ids = {n: i for i, n in enumerate(names)}
    q_src = [ids[srcs[idx[i]]] for i in pick]
    q_ign = []
    for i in pick:
        n1, if1, n2 = links[sets[i][0]][:3]
        li = fc.link_index(n1, if1, n2)
        assert li >= 0
        q_ign.append([li])
    want = fc.row_digests(q_src, q_ign, THREADS)
    bad = [pick[k] for k in range(len(pick)) if int(want[k]) != int(dig[pick[k]])]
    assert not bad, f"{len(bad)} of {len(pick)} what-if rows differ, first {bad[:5]} tiers {tier[bad[:5]]}"
    # the source rows themselves (the base of every tier-0 request)
    base = fc.row_digests([ids[s] for s in srcs], [], THREADS)
    t0 = [i for i in light if tier[i] == 0][:64]
    assert all(int(dig[i]) == int(base[idx[i]]) for i in t0)


def test_c3_sweep_all_rows_vs_checker(hip, oracle):
    from openr_amd.workloads import c3_fabric
    adj, _ = c3_fabric(num_prefixes=0)
    als_h, _ = load_topology(hip, adj, [])
    ls = als_h[A]._impl
    names = ls.node_names()
    srcs = [db.thisNodeName for db in adj]
    sw = ls.sweep(srcs, True)
    sw.run()
    sw.sync()
    als_o, _ = load_topology(oracle, adj, [])
    fc = oracle.module.FastChecker(als_o[A]._impl, names)
    ids = {n: i for i, n in enumerate(names)}
    dist, nh = fc.spf_rows([ids[s] for s in srcs], [], THREADS)
    W = nh.shape[2]
    assert W >= 2  # spines: more than 32 distinct neighbours
    for i, s in enumerate(srcs):
        d, m = sw.fetch(i)
        m = m.reshape(len(names), sw.words)
        assert np.array_equal(d, dist[i]), s
        assert np.array_equal(m[:, :W], nh[i]), s
        assert not m[:, W:].any(), s
    nb = ls.neighbors(srcs[0])
    assert [names[v] for v in fc.neighbours(ids[srcs[0]])] == nb
