#!/bin/bash
# SQ-counter pass of the bench (one pass = one rocprofv3 run; <= 8 SQ counters)
set -e
TAG=${1:-sq}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR \
  --output-format csv -d "$OUT/pmc_SQ" -o run -- python3 "$REPO/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-route-db > "$OUT/pmc_SQ.log" 2>&1
