"""KSP2 device batch (1,024 C4 pairs) wall time for several ORH_KSP_CHUNK
values, each on a fresh LinkState (no memo): python tools/ksp2_chunk_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.types import K_TESTING_AREA as A  # noqa: E402
from openr_amd.workloads import C4_KSP2_PAIRS, C4_SEED, c4_ksp2_pairs, c4_wan  # noqa: E402

hip = host_backend()
adj, _ = c4_wan()
for chunk in ("2048", "512", "256", "2048"):
    os.environ["ORH_KSP_CHUNK"] = chunk
    als, _ = load_topology(hip, adj, [])
    ls = als[A]._impl
    names = ls.node_names()
    ls.prefetch_kth_paths(c4_ksp2_pairs(names, 64, seed=C4_SEED + 99))
    kp = c4_ksp2_pairs(names, C4_KSP2_PAIRS)
    t0 = time.perf_counter()
    ls.prefetch_kth_paths(kp)
    dt = time.perf_counter() - t0
    print(f"chunk {chunk}: {len(kp)} pairs in {dt * 1e3:.1f} ms = {len(kp) / dt:.0f} pairs/s", flush=True)
    del ls, als
