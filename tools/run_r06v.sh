set -e
mkdir -p gpurun_out/r06v
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ksp2_abi.py tests/test_gpu_at_scale.py::test_c4_ksp2_all_benched_pairs > gpurun_out/r06v/tests.log 2>&1
bash tools/ksp2_ab_r06.sh gpurun_out/r06v "" ORH_KSP_ORDER=0
bash tools/c2w_ab_r06.sh gpurun_out/r06v "" ORH_WMS_SKIP=0
