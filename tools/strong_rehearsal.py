"""Strong scaling of ONE topology's all-sources sweep, rehearsed on one GPU
(verdict r03 item 9): the C2 grid mirrored on N device contexts
(ReplicatedLinkState), its 10,000 sources cut into N equal-work blocks
(MultiDeviceSweep); each block is swept ALONE on the GPU, as it would run on
its own device, and the per-device time is the slowest block's. Reports the
speedup over N = 1 against the 1/N^0.7 bar.
usage: python tools/strong_rehearsal.py [grid_n] [Ns...]"""
import statistics
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.topology import bench_grid
from openr_amd.types import K_TESTING_AREA

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
Ns = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
hip = host_backend()
adj, _ = bench_grid(n)
names = [str(i) for i in range(n * n)]
base = None
for N in Ns:
    rls = hip.module.ReplicatedLinkState(K_TESTING_AREA, [0] * N)
    for db in adj:
        rls.update_adjacency_database(db.to_wire())
    sw = rls.sweep(names, True)
    per_block = []
    for r in range(N):
        for _ in range(2):  # warm
            sw.run_block(r)
            sw.sync()
        ts = []
        for _ in range(5):
            sw.run_block(r)
            sw.sync()
            ts.append(sw.last_ms(r))
        per_block.append(statistics.median(ts))
    t = max(per_block)
    base = base or t
    lo, hi = sw.block(0)
    print(f"N={N}: per-device sweep {t:.3f} ms (blocks {[round(x, 3) for x in per_block]}, "
          f"{hi - lo} sources in block 0); speedup {base / t:.2f}x, bar N^0.7 = {N ** 0.7:.2f}x", flush=True)
    del sw, rls
