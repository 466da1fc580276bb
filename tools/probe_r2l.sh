#!/bin/bash
# MS-BFS dispatch-order A/B (GPU box): gpurun_out/$1/*.txt
set -e
O=gpurun_out/${1:-probe}
mkdir -p "$O"
export ORH_MS_WIDE=0
P="python -u tools/msbfs_probe.py --cases all"
timeout -k 10 120 $P > "$O/skip.txt" 2>&1
ORH_MS_SKIP=0 timeout -k 10 120 $P > "$O/noskip.txt" 2>&1
ORH_MS_PERM=mid timeout -k 10 120 $P > "$O/mid_skip.txt" 2>&1
ORH_MS_PERM=mid ORH_MS_SKIP=0 timeout -k 10 120 $P > "$O/mid_noskip.txt" 2>&1
