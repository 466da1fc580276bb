#!/bin/bash
# Round-6 KSP2 search A/B on one box: per spec, the benched C4 batch's stage
# times (tools/ksp2_prof.py: k = 1 / k = 2 search device ms) and the wall time
# of prefetchKthPaths, alternating the specs twice. A spec is "" (shipped),
# a prebuilt variant name (build_var/NAME) or space-free K=V pairs joined by ','.
#   tools/ksp2_ab_r06.sh OUTDIR "" ORH_LDS16_OWN=1 sleep4
OUT=$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for V in "$@"; do
    LP=""; ENVS=""; TAG=${V:-shipped}
    if [[ "$V" == *=* ]]; then ENVS=${V//,/ }; elif [ -n "$V" ]; then LP="build_var/$V"; fi
    env $ENVS LD_LIBRARY_PATH=$LP timeout -k 10 200 python tools/ksp2_prof.py > "$OUT/ksp2_${TAG//[^A-Za-z0-9]/_}_$rep.log" 2>&1 || exit 1
    echo "[$TAG rep$rep] $(grep -A7 'benched batch' "$OUT/ksp2_${TAG//[^A-Za-z0-9]/_}_$rep.log" | grep -E 'search|prefetch_kth' | tr -s ' ' | tr '\n' '|')" | tee -a "$OUT/ksp2_ab.txt"
  done
done
