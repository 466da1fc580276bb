"""MS-BFS load balance probe: distance-phase time vs number of 32-source
batches (workgroups) on the 100x100 grid."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import K_TESTING_AREA as A
hip = host_backend()
adj, _ = bench_grid(100, 1)
als, _ = load_topology(hip, adj, [])
ls = als[A]._impl
for n in (1024, 4096, 8000, 8192, 9000, 10000):
    sw = ls.sweep([str(i) for i in range(n)], True)
    for _ in range(2):
        sw.run(); sw.last_ms()
    ph = []
    for _ in range(5):
        sw.run(); sw.last_ms(); ph.append(sw.phase_ms())
    d = statistics.mean(p[0] for p in ph); h = statistics.mean(p[1] for p in ph)
    print(f"sources {n}: dist {d:.3f} ms hop {h:.3f} ms", flush=True)
