#!/bin/bash
# C4 what-if job under rocprofv3 --kernel-trace, then the kernel timeline of
# the last job run (tools/timeline.py) into gpurun_out/$1/timeline.txt
set -e
TAG=${1:-c4tl}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/tools/c4_leg.py" > "$OUT/c4_leg.out" 2> "$OUT/c4_leg.err"
cd "$REPO"
python tools/timeline.py "$OUT/trace" --from=whatif_seed --nth=-4 --window=45 > "$OUT/timeline.txt"
echo "c4_timeline $TAG done"
