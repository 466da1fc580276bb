#!/bin/bash
# One LDS/VALU counter pass of one isolated C2 sweep (tools/quick_bench.py)
# per prebuilt libopenr_hip variant (build_var/NAME); pmc_summary.py reads them.
#   tools/pmc_lds_ab.sh TAG NAME ...
set -o pipefail
TAG=$1
shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  OUT=$REPO/gpurun_out/pmc_${TAG}_$V
  mkdir -p "$OUT"
  LD_LIBRARY_PATH=$REPO/build_var/$V timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT" -o run \
    -- python3 "$REPO/tools/quick_bench.py" > "$OUT/run.log" 2>&1 || { echo "pmc $V failed"; exit 1; }
done
echo "pmc_lds_ab $TAG done"
