#!/bin/bash
# bench step (32 C2 sweeps) at several stream-lane counts
set -e
for L in 4 2 6 8 4; do
  echo "lanes $L: $(timeout -k 10 200 python bench.py --steps 10 --warmup 2 --legs '' --no-route-db --no-cpu-baseline --lanes $L | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
done
