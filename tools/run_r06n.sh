set -e
mkdir -p gpurun_out/r06n
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_multi_device.py tests/test_gpu_rank_legs.py > gpurun_out/r06n/tests.log 2>&1
bash tools/ms_ab_r06.sh gpurun_out/r06n "" ORH_MS_DEFER=0
T=32 LANES=1,3,4 timeout -k 10 300 python tools/lanes_probe.py > gpurun_out/r06n/lanes_defer.txt 2>&1
