#!/bin/bash
# Round-6 MS-BFS A/B on one box (timing only): the 32-sweep step at 2 lanes
# (tools/lanes_probe.py) and one isolated sweep (tools/quick_bench.py) for the
# shipped library, prebuilt variants in build_var/NAME, or env settings
# (an argument with '=': space-free K=V pairs joined by ','), alternating.
#   tools/ms_ab_r06.sh OUTDIR "" msold ORH_MS_DIRECT=0 ORH_MS_ORDER=cm,ORH_MS_DIRECT=0
OUT=$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for V in "$@"; do
    LP=""; ENVS=""; TAG=${V:-shipped}
    if [[ "$V" == *=* ]]; then ENVS=${V//,/ }; elif [ -n "$V" ]; then LP="build_var/$V"; fi
    R=$(env $ENVS LD_LIBRARY_PATH=$LP T=32 LANES=2 timeout -k 10 200 python tools/lanes_probe.py) || exit 1
    Q=$(env $ENVS LD_LIBRARY_PATH=$LP timeout -k 10 120 python tools/quick_bench.py) || exit 1
    echo "[$TAG rep$rep] step: $R | isolated: $Q" | tee -a "$OUT/ms_ab.txt"
  done
done
