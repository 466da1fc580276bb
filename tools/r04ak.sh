#!/bin/bash
# Round-4 closing pass: the whole GPU suite and smoke on the committed tree,
# then the default bench line when both pass.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04ak}
bash "$ROOT/tools/r04ah.sh" "$TAG" || exit $?
grep -q "tests rc=0" "$ROOT/gpurun_out/$TAG/steps.txt" && grep -q "smoke rc=0" "$ROOT/gpurun_out/$TAG/steps.txt" || exit 1
bash "$ROOT/tools/r04n.sh" "$TAG"
echo "r04ak done"
