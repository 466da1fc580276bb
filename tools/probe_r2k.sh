#!/bin/bash
# MS-BFS A/B on the GPU box: batch order (balls / cm), level stores on / off
# (build_var/nostore), skip on / off, u32 masks. Results in gpurun_out/$1/.
set -e
O=gpurun_out/${1:-probe}
mkdir -p "$O"
export ORH_MS_WIDE=0
P="python -u tools/msbfs_probe.py"
timeout -k 10 120 $P --cases all,corner32,center32 > "$O/balls.txt" 2>&1
ORH_MS_ORDER=cm timeout -k 10 120 $P --cases all > "$O/cm.txt" 2>&1
LD_LIBRARY_PATH=build_var/nostore timeout -k 10 120 $P --cases all,corner32 > "$O/nostore_balls.txt" 2>&1
ORH_MS_ORDER=cm LD_LIBRARY_PATH=build_var/nostore timeout -k 10 120 $P --cases all > "$O/nostore_cm.txt" 2>&1
ORH_MS_SKIP=0 timeout -k 10 120 $P --cases all > "$O/balls_noskip.txt" 2>&1
LD_LIBRARY_PATH=build_var/diag timeout -k 10 120 $P --cases all --reps 1 > "$O/diag_balls.txt" 2>&1
