"""C4 what-if batch device time vs the HBM kernel's near/far width
(ORH_DELTA_PCT, read at context creation): python tools/c4_delta.py PCT"""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.types import K_TESTING_AREA as A
from openr_amd.workloads import c4_wan, c4_what_if_pairs

hip = host_backend()
adj, _ = c4_wan()
als, _ = load_topology(hip, adj, [])
ls = als[A]._impl
names = ls.node_names()
lids = [lid for lid, _ in ls.link_ids()]
pairs = c4_what_if_pairs(lids, names, 64, 16)
sw = ls.what_if_sweep([s for s, _ in pairs], [[l] for _, l in pairs])
sw.run(); sw.sync()
ts = []
for _ in range(5):
    sw.run(); sw.sync(); ts.append(sw.last_ms())
print(f"delta_pct {os.environ.get('ORH_DELTA_PCT', '100')}: what-if {len(pairs)} device "
      f"{statistics.median(ts):.3f} ms", flush=True)
