"""One block of the C4 what-if job split N ways (MultiDeviceWhatIf), run
alone REPS times on one GPU: the command to put under rocprofv3
--kernel-trace --stats to see where a block's time goes.
usage: python tools/md_block_prof.py [N] [block] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.types import K_TESTING_AREA as A  # noqa: E402
from openr_amd.workloads import C4_WHATIF_CHUNK, c4_wan, c4_what_if_job  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
R = int(sys.argv[2]) if len(sys.argv) > 2 else 0
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 5
hip = host_backend()
adj, _ = c4_wan()
als, _ = load_topology(hip, adj, [])
ls = als[A]._impl
names = ls.node_names()
srcs, idx, sets = c4_what_if_job([lid for lid, _ in ls.link_ids()], names)
rls = hip.module.ReplicatedLinkState(A, [0] * N)
for db in adj:
    rls.update_adjacency_database(db.to_wire())
md = rls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=True)
for i in range(REPS + 1):
    t0 = time.perf_counter()
    md.run_block(R)
    md.sync()
    print(f"block {R} of {N}: {(time.perf_counter() - t0) * 1e3:.3f} ms{' (warm-up)' if i == 0 else ''}", flush=True)
