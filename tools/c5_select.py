"""C5 route builds (4 areas, 1M prefixes, best-route selection) for kernel
profiling of route_select_kernel: python tools/c5_select.py [builds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend  # noqa: E402
from openr_amd.facade import load_topology  # noqa: E402
from openr_amd.workloads import C5_AREAS, c5_multi_area  # noqa: E402

hip = host_backend()
areas, pfx = c5_multi_area()
als, ps = load_topology(hip, [db for a in C5_AREAS for db in areas[a]], pfx)
solver = hip.spf_solver("me", True, enable_best_route_selection=True)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    sec, n = solver._impl.time_build_route_db("me", als._impl, ps._impl)
    print(f"build {sec * 1e3:.2f} ms, select kernel {solver._impl.last_select_ms:.4f} ms", flush=True)
