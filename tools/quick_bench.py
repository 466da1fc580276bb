import sys, time, statistics
sys.path.insert(0, '/root/repo')
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.topology import bench_grid
from openr_amd.types import K_TESTING_AREA
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
adj, pfx = bench_grid(n, 1)
hip = host_backend()
als, ps = load_topology(hip, adj, pfx)
ls = als[K_TESTING_AREA]
sw = ls._impl.sweep([str(i) for i in range(n*n)], True)
for _ in range(3): sw.run(); sw.last_ms()
ts=[]; ph=[]
t0=time.perf_counter()
for _ in range(10):
    sw.run(); ts.append(sw.last_ms()); ph.append(sw.phase_ms())
el=time.perf_counter()-t0
print("kernel ms", statistics.mean(ts), "phases", [round(statistics.mean(x),3) for x in zip(*ph)], "wall/step ms", el*100)
