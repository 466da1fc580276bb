#!/bin/bash
# glibc malloc tuning A/B on the route-build legs (C3, C5): the product default
# (WorkerPool::tuneAllocator), then glibc defaults (ORH_MALLOC_TUNE=0)
set -e
ONE='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c3=d["legs"]["c3"]; c5=d["legs"]["c5"]; print("c3 build", c3["build_route_db_ms"], "best", c3.get("build_route_db_best_route_ms"), "| c5 build", c5["build_route_db_ms"], "policy", c5["rib_policy_ms"], "first", c5["incremental"]["first_full_rebuild_ms"], "delta", c5["incremental"]["rebuild_ms"], "whole", c5["incremental"]["whole_build_route_db_ms"], "prefix-only", c5["incremental_prefix_only"]["rebuild_ms"])'
echo "product default: $(timeout -k 10 300 python bench.py --steps 2 --warmup 1 --legs c3,c5 --no-cpu-baseline | python -c "$ONE")"
echo "glibc defaults (ORH_MALLOC_TUNE=0): $(ORH_MALLOC_TUNE=0 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --legs c3,c5 --no-cpu-baseline | python -c "$ONE")"
