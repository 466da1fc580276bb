#!/bin/bash
# Round-4 GPU pass i: padded log assembly (sweep parity); the 4-lane step and
# one sweep alone with: base, ORH_HOP_NARROW=1 (4 nodes per first-hop
# thread), the hop_w4 build (first-hop VGPRs capped for 4 waves per SIMD),
# ORH_MS_BLOCK=768 / 1024; then the SQ counters of the isolated sweep.
TAG=${1:-r04i}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step LOG CMD...
  local log=$1; shift
  "$@" > "$log" 2>&1
  local rc=$?
  echo "step rc=$rc: $*" >> "$OUT/steps.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step "$OUT/sweep_tests.log" timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v -k "sweep_all or first_hops_exact or latency or u16 or ladder" --timeout 300 --timeout-method thread
run() {  # run NAME ENV...
  local n=$1; shift
  step "$OUT/sweep_$n.log" env "$@" timeout -k 10 120 python -u tools/quick_bench.py
  step "$OUT/step_$n.log" env "$@" T=32 LANES=4 timeout -k 10 300 python -u tools/lanes_probe.py
}
run base ORH_NOP=1
run narrow ORH_HOP_NARROW=1
run w4 LD_LIBRARY_PATH=$ROOT/build_var/hop_w4
run b768 ORH_MS_BLOCK=768
run b1024 ORH_MS_BLOCK=1024
cd /tmp && export TMPDIR=/tmp
step "$OUT/pmc_sq.log" timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/pmc_sq" -o run -- python3 "$ROOT/bench.py" --topologies 1 --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-route-db --legs=
echo "r04i $TAG done"
