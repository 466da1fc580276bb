"""Run bench_legs.leg_c4 alone (C4 what-if job + KSP2 at BASELINE shape) and
print its JSON: python tools/c4_leg.py [--cpu]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs  # noqa: E402
from openr_amd import host_backend  # noqa: E402

print(json.dumps(bench_legs.leg_c4(host_backend(), "--cpu" in sys.argv)), flush=True)
