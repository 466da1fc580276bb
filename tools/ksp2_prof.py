"""The benched C4 KSP2 batch (1,024 pairs, prefetchKthPaths) broken down by
ORH_KSP_PROF (host and device time per stage, on stderr), next to the same
batch through MultiDeviceKthPaths on one context (orh_ksp2_batch + path
parsing, no memo): python tools/ksp2_prof.py"""
import os
import sys
import time

os.environ.setdefault("ORH_KSP_PROF", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.types import K_TESTING_AREA as A  # noqa: E402
from openr_amd.workloads import C4_KSP2_PAIRS, C4_SEED, c4_ksp2_pairs, c4_wan  # noqa: E402

hip = host_backend()
adj, _ = c4_wan()
als, _ = load_topology(hip, adj, [])
ls = als[A]._impl
names = ls.node_names()
kp = c4_ksp2_pairs(names, C4_KSP2_PAIRS)
ls.prefetch_kth_paths(c4_ksp2_pairs(names, 64, seed=C4_SEED + 99))
print("--- benched batch", flush=True)
sys.stderr.flush()
t0 = time.perf_counter()
ls.prefetch_kth_paths(kp)
print(f"prefetch_kth_paths: {1e3 * (time.perf_counter() - t0):.3f} ms wall", flush=True)
rls = hip.module.ReplicatedLinkState(A, [0])
for db in adj:
    rls.update_adjacency_database(db.to_wire())
mk = rls.kth_paths_batch(kp)
for _ in range(3):
    mk.run()
    print(f"MultiDeviceKthPaths (1 context): {mk.last_ms(0):.3f} ms wall", flush=True)
