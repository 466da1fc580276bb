#!/bin/bash
# One LDS/VALU counter pass of one isolated C2 sweep (tools/quick_bench.py)
# per environment spec ("VAR=a VAR2=b"); output gpurun_out/pmc_<tag>_<i>/.
#   tools/pmc_lds_env.sh TAG "ORH_MS_ORDER=cm" "ORH_MS_ORDER=host"
set -o pipefail
TAG=$1
shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
for SPEC in "$@"; do
  OUT=$REPO/gpurun_out/pmc_${TAG}_$i
  mkdir -p "$OUT"
  echo "$SPEC" > "$OUT/spec.txt"
  for kv in $SPEC; do export "$kv"; done
  timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d "$OUT" -o run \
    -- python3 "$REPO/tools/quick_bench.py" > "$OUT/run.log" 2>&1 || { echo "pmc $SPEC failed"; exit 1; }
  for kv in $SPEC; do unset "${kv%%=*}"; done
  i=$((i + 1))
done
echo "pmc_lds_env $TAG done"
