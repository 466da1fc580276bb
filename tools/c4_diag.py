"""C4 what-if diagnostics: device phase split of the what-if batch and of a
plain (no ignore set) batch on the 50k-node WAN."""
import os, sys, time
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
for nl, ns in ((64, 16), (16, 16)):
    pairs = c4_what_if_pairs(lids, names, nl, ns)
    sw = ls.what_if_sweep([s for s, _ in pairs], [[l] for _, l in pairs])
    sw.run(); sw.sync()
    t0 = time.perf_counter()
    for _ in range(3):
        sw.run()
    sw.sync()
    dt = (time.perf_counter() - t0) / 3
    sw.run()
    print(f"what-if {len(pairs)}: wall {dt*1e3:.2f} ms, device {sw.last_ms():.2f} ms, phases {sw.phase_ms()}", flush=True)
    plain = ls.sweep(sorted({s for s, _ in pairs}) * 1, True)
    plain.run(); plain.sync(); plain.run()
    print(f"plain {plain.sources}: device {plain.last_ms():.2f} ms phases {plain.phase_ms()}", flush=True)
big = ls.sweep(names[:1024], True)
big.run(); big.sync(); big.run()
print(f"plain 1024 contiguous: device {big.last_ms():.2f} ms phases {big.phase_ms()}", flush=True)
