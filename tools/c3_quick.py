"""C3 Clos all-sources sweep: device time per phase (A/B of kernel variants)."""
import os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.types import K_TESTING_AREA as A
from openr_amd.workloads import c3_fabric
hip = host_backend()
adj, _ = c3_fabric()
als, _ = load_topology(hip, adj, [])
sw = als[A]._impl.sweep([db.thisNodeName for db in adj], True)
for _ in range(3):
    sw.run(); sw.last_ms()
ts, ph = [], []
for _ in range(10):
    sw.run(); ts.append(sw.last_ms()); ph.append(sw.phase_ms())
print("C3 kernel ms", round(statistics.mean(ts), 4), "phases", [round(statistics.mean(x), 4) for x in zip(*ph)])
