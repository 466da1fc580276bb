"""Step time of T what-if sweeps of the C2 grid dealt over L stream lanes
(one context + HIP stream per lane): does overlapping independent sweeps pay?"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import K_TESTING_AREA
import bench

hip = host_backend()
n = 100
names = [str(i) for i in range(n * n)]
T = int(os.environ.get("T", "16"))
lss = {}
for L in [int(x) for x in os.environ.get("LANES", "1,2,4,8").split(",")]:
    sweeps = []
    for t in range(T):
        adj, pfx = bench_grid(n, 1)
        if t:
            bench.drain_what_if_link(adj, n, t)
        als, _ = load_topology(hip, adj, pfx, lane=t % L)
        ls = als[K_TESTING_AREA]
        sweeps.append((als, ls._impl.sweep(names, True)))
    for _ in range(2):
        for _, sw in sweeps: sw.run()
        for _, sw in sweeps: sw.sync()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        for _, sw in sweeps: sw.run()
    for _, sw in sweeps: sw.sync()
    dt = (time.perf_counter() - t0) / reps
    print(f"T={T} lanes={L}: {dt*1e3:.2f} ms/step = {dt*1e3/T:.3f} ms/sweep = {T*n*n/dt/1e6:.2f} M SPF-sources/s", flush=True)
    del sweeps
