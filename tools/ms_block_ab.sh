#!/bin/bash
# MS-BFS workgroup size A/B (ORH_MS_BLOCK): one sweep alone (quick_bench) and
# the bench step (32 sweeps over 4 lanes), per setting
set -e
for B in ${MS_BLOCKS:-768 512 640 768}; do
  echo "ORH_MS_BLOCK=$B sweep: $(ORH_MS_BLOCK=$B timeout -k 10 120 python tools/quick_bench.py)"
  echo "ORH_MS_BLOCK=$B step: $(ORH_MS_BLOCK=$B timeout -k 10 200 python bench.py --steps 10 --warmup 2 --legs '' --no-route-db --no-cpu-baseline | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
