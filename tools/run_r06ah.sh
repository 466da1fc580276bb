set -e
mkdir -p gpurun_out/r06ah
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_weighted.py tests/test_gpu_parity.py > gpurun_out/r06ah/tests.log 2>&1
bash tools/c2w_ab_r06.sh gpurun_out/r06ah "" ORH_HOP_XCD=0
