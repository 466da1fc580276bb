#!/bin/bash
# A/B of the MS-BFS level-scratch fill (GPU box scratch copy): the built
# library (unreached bytes written at the end of the search) against
# build_var/lvlinit (-DORH_MS_LVL_INIT: a fill pass before the search),
# alternating, default bench (C2 sweeps, no route DB / CPU baseline)
set -e
OUT=gpurun_out/${1:-lvl_ab}
mkdir -p "$OUT"
cp openr_amd/lib/libopenr_hip.so "$OUT/../new_lib.so"
for R in 1 2 3; do
  for V in new lvlinit; do
    if [ "$V" = new ]; then cp "$OUT/../new_lib.so" openr_amd/lib/libopenr_hip.so; else cp build_var/lvlinit/libopenr_hip.so openr_amd/lib/libopenr_hip.so; fi
    timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-route-db --legs '' > "$OUT/$V$R.json" 2>"$OUT/$V$R.err"
    echo "[$V $R]: $(python3 -c "import json;d=json.loads(open('$OUT/$V$R.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'].get('phase_ms'))")" | tee -a "$OUT/summary.txt"
  done
done
cp "$OUT/../new_lib.so" openr_amd/lib/libopenr_hip.so
rm -f "$OUT/../new_lib.so"
