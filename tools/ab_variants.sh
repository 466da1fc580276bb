#!/bin/bash
# A/B of compile-time variants of libopenr_hip on the GPU box (scratch copy):
#   tools/ab_variants.sh "-DFOO" "" "-DBAR"  -> phase ms + value per variant
set -e
for V in "$@"; do
  bash tools/diag_build.sh $V
  timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-route-db > gpurun_out/ab.json 2>&1
  echo "[$V]: $(python3 -c "import json;d=json.loads(open('gpurun_out/ab.json').read().splitlines()[-1]);print(d['roofline']['phase_ms'], d['value'])")"
done
