#!/bin/bash
# C2 buildRouteDb("1") with the product's allocator tuning and with glibc
# defaults, twice each (bench: cold = after a topology change, warm)
set -e
ONE='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("cold", d["build_route_db_ms"], "warm", d["build_route_db_warm_ms"])'
for T in 1 0 1 0; do
  echo "ORH_MALLOC_TUNE=$T: $(ORH_MALLOC_TUNE=$T timeout -k 10 200 python bench.py --steps 2 --warmup 1 --legs '' --no-cpu-baseline --topologies 1 --lanes 1 | python -c "$ONE")"
done
