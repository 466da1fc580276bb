"""The N-rank bench legs (bench.py --gpus N: rank r runs block r of C3's
prefix-sharded buildRouteDb and of C4's what-if job / KSP2 batch on its own
GPU, bench_legs.rank_c3 / rank_c4): the union of the ranks' outputs equals
the single job's, at N = 2, 4 and 8. On this one-GPU box the ranks run one
after another in this process, each block exactly as its rank builds it."""
import numpy as np
import pytest

import bench_legs

pytestmark = pytest.mark.gpu


def _hashes(digest):
    n_uc, n_mp, raw = digest
    h = np.frombuffer(raw, dtype=np.uint64)
    assert len(h) == n_uc + n_mp
    return np.sort(h[:n_uc]), np.sort(h[n_uc:])


@pytest.fixture(scope="module")
def c3_state(hip):
    return bench_legs.c3_rank_state(hip)


@pytest.fixture(scope="module")
def c4_state(hip):
    return bench_legs.c4_rank_state(hip)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rank_c3_union_equals_whole_build(hip, c3_state, world):
    als, ps = c3_state
    me = "2-0-0"
    uc1, mp1 = _hashes(hip.spf_solver(me, True)._impl.build_route_db_digest(me, als._impl, ps._impl))
    ucs, mps = [], []
    for r in range(world):
        out = bench_legs.rank_c3(hip, r, world, state=c3_state, reps=1, digest=True)
        uc, mp = _hashes(out["digest"])
        ucs.append(uc)
        if r:
            assert len(mp) == 0  # shard 0 builds the MPLS routes
        else:
            mps.append(mp)
        assert len(uc) < len(uc1)  # a real block, not the whole build
    assert np.array_equal(np.sort(np.concatenate(ucs)), uc1)
    assert np.array_equal(mps[0], mp1)


def test_rank_c4_union_equals_single_job(hip, c4_state):
    from helpers import assert_tiers_match
    from openr_amd.workloads import C4_WHATIF_CHUNK
    als, ls, srcs, idx, sets, pairs = c4_state
    one = ls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=True)
    one.set_digests()
    one.run()
    one.sync()
    info1, dig1 = one.info(), one.digests()
    one.release()
    del one
    ls.prefetch_kth_paths(pairs)
    want = [(ls.get_kth_path_ids(s, d, 1), ls.get_kth_path_ids(s, d, 2)) for s, d in pairs]
    for world in (2, 4, 8):
        info = np.full(len(idx), 0xFFFFFFFF, dtype=np.uint64)
        dig = np.zeros(len(idx), dtype=np.uint64)
        seen = np.zeros(len(idx), dtype=bool)
        kseen = [None] * len(pairs)
        for r in range(world):
            out = bench_legs.rank_c4(hip, r, world, state=c4_state, reps=1, digest=True)
            reqs = np.array(out["what_if_reqs"], dtype=np.int64)
            assert not seen[reqs].any()
            seen[reqs] = True
            info[reqs] = out["what_if_info"]
            dig[reqs] = out["what_if_digests"]
            for i, p in zip(out["ksp2_idx"], out["ksp2_paths"]):
                assert kseen[i] is None
                kseen[i] = p
            assert out["what_if_requests"] <= len(idx) // world + 4096
        assert seen.all() and all(k is not None for k in kseen)
        assert_tiers_match(info, info1, world >= bench_legs.SEARCH_LARGE_BLOCKS)
        bad = np.nonzero(dig != dig1)[0]
        assert len(bad) == 0, f"world {world}: {len(bad)} what-if rows differ, first {bad[:5]}"
        bad = [i for i in range(len(pairs)) if [list(x) for x in kseen[i]] != [list(x) for x in want[i]]]
        assert not bad, f"world {world}: {len(bad)} KSP2 pairs differ, first {bad[:3]}"

