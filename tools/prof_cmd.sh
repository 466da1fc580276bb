#!/bin/bash
# Kernel trace + stats of one python tool run: tools/prof_cmd.sh TAG script.py [args]
set -e
TAG=$1
shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/$@" > "$OUT/trace.out" 2> "$OUT/trace.err"
echo "prof_cmd $TAG done"
