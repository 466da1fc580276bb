"""C4 KSP2 batch stages (ORH_KSP_PROF=1 lines on stderr) with the k = 1 / k = 2
searches in LDS (u16 distances, spf_lds16_kernel) and in HBM
(ORH_KSP_LDS=0): 1,024 pairs, three batches per mode (the first warms up),
plus the wall time of each prefetch.
usage: python tools/ksp2_stage_ab.py [modes...]   (modes: 1 0)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.types import K_TESTING_AREA as A
from openr_amd.workloads import C4_KSP2_PAIRS, c4_wan, c4_ksp2_pairs

hip = host_backend()
adj, _ = c4_wan()
os.environ["ORH_KSP_PROF"] = "1"
for mode in (sys.argv[1:] or ["1", "0"]):
    os.environ["ORH_KSP_LDS"] = mode
    for rep in range(3):
        als, _ = load_topology(hip, adj, [])
        ls = als[A]._impl
        pairs = c4_ksp2_pairs(ls.node_names(), C4_KSP2_PAIRS)
        print(f"== ORH_KSP_LDS={mode} rep {rep}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        ls.prefetch_kth_paths(pairs)
        t1 = time.perf_counter()
        print(f"ORH_KSP_LDS={mode} rep {rep}: prefetch {1e3 * (t1 - t0):.2f} ms = "
              f"{len(pairs) / (t1 - t0):.0f} pairs/s", file=sys.stderr, flush=True)
