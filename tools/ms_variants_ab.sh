#!/bin/bash
# MS-BFS variant A/B: for each configuration (space-separated VAR=value
# settings, one configuration per argument) one sweep alone (quick_bench) and
# the bench step (32 sweeps over 4 lanes).
# usage: tools/ms_variants_ab.sh "ORH_MS_BLOCK=768" "ORH_MS_BLOCK=512 ORH_MS_SKIP=1" ...
set -e
for CFG in "$@"; do
  echo "[$CFG] sweep: $(env $CFG timeout -k 10 120 python tools/quick_bench.py)"
  echo "[$CFG] step: $(env $CFG timeout -k 10 200 python bench.py --steps 10 --warmup 2 --legs '' --no-route-db --no-cpu-baseline | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
