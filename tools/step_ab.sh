#!/bin/bash
# Step-time A/B of compile-time variants (GPU box scratch copy; timing only):
# T what-if sweeps over 4 lanes and one isolated sweep per variant.
#   tools/step_ab.sh "" "-DORH_EXP_MSBFS_ONLY" ...
set -e
for V in "$@"; do
  bash tools/diag_build.sh $V
  echo "[$V] $(T=32 LANES=4 timeout -k 10 300 python tools/lanes_probe.py) | isolated: $(timeout -k 10 120 python tools/quick_bench.py)"
done
