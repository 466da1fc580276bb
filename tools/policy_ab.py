"""C5 RibPolicy application time (1M routes, UCMP weights by area), three
builds: python tools/policy_ab.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import host_backend
from openr_amd.facade import load_topology
from openr_amd.rib_policy import RibPolicy, RibPolicyStatement, RibRouteActionWeight
from openr_amd.workloads import C5_AREAS, C5_TAG, c5_multi_area

hip = host_backend()
areas, pfx = c5_multi_area()
als, ps = load_topology(hip, [db for a in C5_AREAS for db in areas[a]], pfx)
solver = hip.spf_solver("me", True, enable_best_route_selection=True)
policy = RibPolicy([RibPolicyStatement("ucmp", None, [C5_TAG], RibRouteActionWeight(
    0, {"A": 1, "B": 2, "C": 3, "D": 4}, {}))], 3600)
for rep in range(3):
    b, p, n, u = solver._impl.time_build_route_db_with_policy("me", als._impl, ps._impl, policy._impl)
    print(f"{os.environ.get('ORH_POLICY_COPY') and 'copy' or 'move'} rep {rep}: build {b*1e3:.1f} ms "
          f"policy {p*1e3:.1f} ms ({u} of {n} routes)", flush=True)
