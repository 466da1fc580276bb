set -e
mkdir -p gpurun_out/r06k
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_policy.py > gpurun_out/r06k/tests.log 2>&1
bash tools/ksp2_ab_r06.sh gpurun_out/r06k "" g8 g2
timeout -k 10 600 python -u bench.py > gpurun_out/r06k/bench.json 2> gpurun_out/r06k/bench.err
