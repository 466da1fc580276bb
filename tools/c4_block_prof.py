"""One source block of the C4 what-if job run alone (what a device runs when
the job is split over N devices), for kernel traces: python
tools/c4_block_prof.py N r [reps]. Block r = sources [r*64/N, (r+1)*64/N)
and their requests, copy-on-write (the bench's mode)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.types import K_TESTING_AREA as A  # noqa: E402
from openr_amd.workloads import C4_WHATIF_CHUNK, c4_wan, c4_what_if_job  # noqa: E402

N, r = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
hip = host_backend()
adj, _ = c4_wan()
als, _ = load_topology(hip, adj, [])
ls = als[A]._impl
srcs, idx, sets = c4_what_if_job([lid for lid, _ in ls.link_ids()], ls.node_names())
lo, hi = r * len(srcs) // N, (r + 1) * len(srcs) // N
pick = [i for i in range(len(idx)) if lo <= idx[i] < hi]
b = ls.what_if_batch(srcs[lo:hi], [idx[i] - lo for i in pick], [sets[i] for i in pick], C4_WHATIF_CHUNK,
                     share_base=True)
for k in range(reps):
    t0 = time.perf_counter()
    b.run()
    b.sync()
    print(f"block {r}/{N}: {len(pick)} requests, {(time.perf_counter() - t0) * 1e3:.3f} ms wall, "
          f"{b.last_ms():.3f} ms device", flush=True)
info = b.info()
tiers = [int(((info & 7) == t).sum()) for t in range(5)]
print("tiers", tiers, "max affected", int((info >> 3).max()), flush=True)
