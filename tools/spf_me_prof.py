"""Time the pieces of a route build's own SPF on C2 (GPU box): getSpfResult
of one source after a metric flip (memo cleared, mirror patched), split into
the mirror flush, the device SPF and the host row fill.

  python tools/spf_me_prof.py
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.topology import bench_grid  # noqa: E402
from openr_amd.types import K_TESTING_AREA  # noqa: E402

hip = host_backend()
n = 100
adj_dbs, _ = bench_grid(n)
als, _ = load_topology(hip, adj_dbs, [])
ls = als[K_TESTING_AREA]
db = adj_dbs[n * n // 2]
t_upd, t_spf = [], []
for i in range(15):
    db.adjacencies[0].metric = 1 + (i & 1)
    t0 = time.perf_counter()
    ls.update_adjacency_database(db)
    t1 = time.perf_counter()
    ls._impl.get_spf_result("1", True)
    t2 = time.perf_counter()
    t_upd.append((t1 - t0) * 1e3)
    t_spf.append((t2 - t1) * 1e3)
print({"update_adjacency_database_ms": round(statistics.median(t_upd), 3),
       "get_spf_result_cold_ms": round(statistics.median(t_spf), 3)})
