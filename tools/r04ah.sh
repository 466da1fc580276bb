#!/bin/bash
# Round-4 final check: the whole GPU suite and smoke on the committed tree.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04ah}
mkdir -p "$OUT"
timeout -k 10 780 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests rc=$?" >> "$OUT/steps.txt"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
echo "smoke rc=$?" >> "$OUT/steps.txt"
