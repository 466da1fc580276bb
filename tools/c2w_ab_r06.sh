#!/bin/bash
# C2w (weighted all-sources) A/B on one box: tools/c2w_probe.py per variant,
# alternating, twice. A variant is "" (shipped), build_var/NAME, or space-free
# K=V pairs joined by ',' (optionally NAME+K=V,...).
#   tools/c2w_ab_r06.sh OUTDIR "" ORH_WMS_SKIP=0 wmsocc2 wmsocc2+ORH_WMS_SKIP=0
OUT=$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for V in "$@"; do
    LIB=${V%%+*}; ENVS=""
    [[ "$V" == *+* ]] && ENVS=${V#*+}
    [[ "$LIB" == *=* ]] && { ENVS=$LIB; LIB=""; }
    LP=${LIB:+build_var/$LIB}
    R=$(env ${ENVS//,/ } LD_LIBRARY_PATH=$LP timeout -k 10 120 python tools/c2w_probe.py) || exit 1
    echo "[${V:-shipped} rep$rep] $R" | tee -a "$OUT/c2w_ab.txt"
  done
done
