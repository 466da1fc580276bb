#!/bin/bash
# Kernel trace + one PMC pass per counter group over one python tool run
# (rocprofv3 does not split counters over passes; FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950). Output: gpurun_out/prof_<tag>/
#   tools/profile_cmd.sh TAG tools/c4_leg.py [args]
set -e
TAG=$1
shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
SCRIPT=$1
shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$REPO/$SCRIPT" "$@" > "$OUT/trace.log" 2>&1
for CTR in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
    "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"; do
  NAME=$(echo "$CTR" | cut -d' ' -f1)
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $CTR --output-format csv -d "$OUT/pmc_$NAME" -o run \
    -- python3 "$REPO/$SCRIPT" "$@" > "$OUT/pmc_$NAME.log" 2>&1
done
echo "profile_cmd $TAG done"
