"""C4 KSP2 batch broken down: plain SPFs of the sources (k = 1 rows), the
k = 1 traces, and the k = 2 re-runs + traces (prefetch_kth_paths)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.types import K_TESTING_AREA as A
from openr_amd.workloads import c4_wan, c4_ksp2_pairs

hip = host_backend()
adj, _ = c4_wan()
for rep in range(2):
    als, _ = load_topology(hip, adj, [])
    ls = als[A]._impl
    kp = c4_ksp2_pairs(ls.node_names(), 256)
    t0 = time.perf_counter()
    ls.prefetch_spf_results([a for a, _ in kp])
    t1 = time.perf_counter()
    for a, b in kp:
        ls.get_kth_paths(a, b, 1)
    t2 = time.perf_counter()
    ls.prefetch_kth_paths(kp)
    t3 = time.perf_counter()
    print(f"rep {rep}: k=1 SPFs {1e3*(t1-t0):.2f} ms, k=1 traces {1e3*(t2-t1):.2f} ms, "
          f"k=2 SPFs + traces {1e3*(t3-t2):.2f} ms, total {1e3*(t3-t0):.2f} ms", flush=True)

# device time alone for the k = 1 batch (plain rows of the same sources, no host copies)
sw = ls.what_if_sweep([a for a, _ in kp], [[] for _ in kp])
sw.run(); sw.sync()
sw.run(); sw.sync()
print(f"k=1 batch device only: {sw.last_ms():.3f} ms ({len(kp)} rows)", flush=True)
