"""C4 what-if job and KSP2 batch split over N devices, rehearsed on one GPU
(verdict r04 item 1): the 50k WAN mirrored on N device contexts
(ReplicatedLinkState); MultiDeviceWhatIf cuts the job's 64 sources into N
blocks of equal request counts, MultiDeviceKthPaths the 1,024 pairs into N
source blocks. Each block runs ALONE on the GPU, as it would on its own
device, and the per-device time is the slowest block's; the whole job on one
context is the N = 1 line. Bar: slowest block <= 1.3 / N of the whole job.
usage: python tools/c4_multi_device_rehearsal.py [Ns...]  (default 2 4 8)"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.types import K_TESTING_AREA as A  # noqa: E402
from openr_amd.workloads import (C4_KSP2_PAIRS, C4_WHATIF_CHUNK, c4_ksp2_pairs, c4_wan,  # noqa: E402
                                 c4_what_if_job)

Ns = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
REPS = 3
hip = host_backend()
adj, _ = c4_wan()
als, _ = load_topology(hip, adj, [])
ls = als[A]._impl
names = ls.node_names()
srcs, idx, sets = c4_what_if_job([lid for lid, _ in ls.link_ids()], names)
kp = c4_ksp2_pairs(names, C4_KSP2_PAIRS)
out = {"workload": f"C4 WAN N={len(names)}: {len(idx)} what-if requests ({len(srcs)} sources), "
                   f"{len(kp)} KSP2 pairs", "chunk": C4_WHATIF_CHUNK, "reps": REPS, "lines": []}


def timed(fn, sync):
    fn()
    sync()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts)


# N = 1: the whole job on one context (copy-on-write, the bench's mode)
one = ls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=True)
w1 = timed(one.run, one.sync)
one.release()
del one
rls1 = hip.module.ReplicatedLinkState(A, [0])
for db in adj:
    rls1.update_adjacency_database(db.to_wire())
k1 = rls1.kth_paths_batch(kp)
kt1 = timed(k1.run, lambda: None)
del k1, rls1
out["lines"].append({"N": 1, "what_if_ms": round(w1, 3), "ksp2_ms": round(kt1, 3)})
print(json.dumps(out["lines"][-1]), flush=True)
for N in Ns:
    rls = hip.module.ReplicatedLinkState(A, [0] * N)
    for db in adj:
        rls.update_adjacency_database(db.to_wire())
    md = rls.what_if_batch(srcs, idx, sets, C4_WHATIF_CHUNK, share_base=True)
    wb = []
    for r in range(N):
        wb.append(timed(lambda: md.run_block(r), md.sync))
        md.release(r)
    mk = rls.kth_paths_batch(kp)
    kb = []
    for r in range(N):
        kb.append(timed(lambda: mk.run_block(r), lambda: None))
    line = {"N": N, "what_if_blocks_ms": [round(x, 3) for x in wb], "what_if_ms": round(max(wb), 3),
            "what_if_frac_of_whole": round(max(wb) / w1, 4), "what_if_bar": round(1.3 / N, 4),
            "what_if_speedup": round(w1 / max(wb), 2),
            "block_requests": [md.block_requests(r) for r in range(N)],
            "ksp2_blocks_ms": [round(x, 3) for x in kb], "ksp2_ms": round(max(kb), 3),
            "ksp2_frac_of_whole": round(max(kb) / kt1, 4), "ksp2_speedup": round(kt1 / max(kb), 2),
            "block_pairs": [mk.block_pairs(r) for r in range(N)]}
    out["lines"].append(line)
    print(json.dumps(line), flush=True)
    del md, mk, rls
print(json.dumps(out), flush=True)
