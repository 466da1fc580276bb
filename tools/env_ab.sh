#!/bin/bash
# Runtime A/B of environment knobs on the GPU box (timing only): per spec,
# one isolated C2 sweep (tools/quick_bench.py) and the 4-lane 32-variant step
# (tools/lanes_probe.py), alternating the specs REPS times.
#   tools/env_ab.sh "ORH_MS_ONE=0" "ORH_MS_ONE=1"
set -e
REPS=${REPS:-2}
for r in $(seq 1 "$REPS"); do
  for V in "$@"; do
    echo "[$V] step: $(env $V T=32 LANES=${LANES:-2} timeout -k 10 300 python tools/lanes_probe.py) | isolated: $(env $V timeout -k 10 120 python tools/quick_bench.py)"
  done
done
