#!/bin/bash
# Kernel-trace stats + one SQ counter pass of the bench (GPU box).
# usage: tools/prof_round.sh TAG   -> gpurun_out/prof_TAG/{trace,pmc_SQ}
set -e
TAG=${1:-cur}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-route-db > "$OUT/trace.log" 2>&1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VALU \
  --output-format csv -d "$OUT/pmc_SQ" -o run -- python3 "$REPO/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-route-db > "$OUT/pmc_SQ.log" 2>&1
