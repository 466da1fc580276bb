set -e
mkdir -p gpurun_out/r06u
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_weighted.py > gpurun_out/r06u/tests.log 2>&1
bash tools/c2w_ab_r06.sh gpurun_out/r06u "" ORH_WMS_BAND=0
