#!/bin/bash
# A/B of compile-time variants on the GPU box (scratch copy), timing only
# (no correctness check: diagnostic variants may be wrong on purpose):
#   tools/ab_quick.sh "" "-DORH_EXP_NO_LVL_STORE"
set -e
for V in "$@"; do
  bash tools/diag_build.sh $V
  echo "[$V]: $(timeout -k 10 120 python tools/quick_bench.py)"
done
