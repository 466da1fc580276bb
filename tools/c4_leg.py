"""Run bench_legs.leg_c4 alone (C4 what-if job + KSP2 at BASELINE shape) and
print its JSON: python tools/c4_leg.py [--cpu] [--chunk=N]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_legs  # noqa: E402
from openr_amd import host_backend  # noqa: E402

chunk = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--chunk=")), None)
print(json.dumps(bench_legs.leg_c4(host_backend(), "--cpu" in sys.argv, chunk=chunk)), flush=True)
