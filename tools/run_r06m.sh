set -e
mkdir -p gpurun_out/r06m
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ksp2_abi.py tests/test_gpu_at_scale.py::test_c4_ksp2_all_benched_pairs > gpurun_out/r06m/ksp2_tests.log 2>&1
bash tools/ksp2_ab_r06.sh gpurun_out/r06m "" wc0
bash tools/run_r06l.sh
