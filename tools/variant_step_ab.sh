#!/bin/bash
# Step-time A/B of prebuilt libopenr_hip variants (tools/build_variant.sh NAME
# ...; timing only, diagnostic variants may compute garbage on purpose): per
# variant, T what-if sweeps over LANES (default 2) lanes (tools/lanes_probe.py) and one sweep
# alone (tools/quick_bench.py).
# usage (repo root, via gpurun): tools/variant_step_ab.sh base msbfs_only ...
set -o pipefail
OUT=gpurun_out/variant_ab
mkdir -p "$OUT"
for V in "$@"; do
  export LD_LIBRARY_PATH=$PWD/build_var/$V
  S=$(T=32 LANES=${LANES:-2} timeout -k 10 300 python tools/lanes_probe.py 2>&1 | tail -1); rc=$?
  [ $rc -ne 0 ] && { echo "[$V] step failed rc=$rc" | tee -a "$OUT/ab.txt"; exit $rc; }
  Q=$(timeout -k 10 120 python tools/quick_bench.py 2>&1 | tail -1); rc=$?
  [ $rc -ne 0 ] && { echo "[$V] sweep failed rc=$rc" | tee -a "$OUT/ab.txt"; exit $rc; }
  echo "[$V] $S | alone: $Q" | tee -a "$OUT/ab.txt"
done
