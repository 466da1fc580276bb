#!/bin/bash
# Round-6 MS-BFS A/B on one box (timing only): the 32-sweep step at 2 lanes
# (tools/lanes_probe.py) and one isolated sweep (tools/quick_bench.py) for the
# shipped library and prebuilt variants in build_var/NAME, alternating.
#   tools/ms_ab_r06.sh OUTDIR "" msold mszeros ...   ("" = the shipped library)
OUT=$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for V in "$@"; do
    if [ -z "$V" ]; then LP=""; TAG=shipped; else LP="build_var/$V"; TAG=$V; fi
    R=$(LD_LIBRARY_PATH=$LP T=32 LANES=2 timeout -k 10 200 python tools/lanes_probe.py) || exit 1
    Q=$(LD_LIBRARY_PATH=$LP timeout -k 10 120 python tools/quick_bench.py) || exit 1
    echo "[$TAG rep$rep] step: $R | isolated: $Q" | tee -a "$OUT/ms_ab.txt"
  done
done
