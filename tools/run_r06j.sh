set -e
mkdir -p gpurun_out/r06j
ORH_LDS16_OWN=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ksp2_abi.py tests/test_gpu_at_scale.py::test_c4_ksp2_all_benched_pairs > gpurun_out/r06j/own_tests.log 2>&1
bash tools/ms_ab_r06.sh gpurun_out/r06j "" ORH_MS_DIRECT=0 ORH_MS_ORDER=cm,ORH_MS_DIRECT=0
bash tools/ksp2_ab_r06.sh gpurun_out/r06j "" ORH_LDS16_OWN=1 sleep4 ORH_LDS16_BLOCK=512
