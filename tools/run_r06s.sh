set -e
mkdir -p gpurun_out/r06s
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_multi_device.py tests/test_gpu_rank_legs.py tests/test_gpu_ksp2_abi.py tests/test_gpu_at_scale.py::test_c4_ksp2_all_benched_pairs > gpurun_out/r06s/tests.log 2>&1
bash tools/ksp2_ab_r06.sh gpurun_out/r06s "" ignglob
timeout -k 10 300 python tools/c4_multi_device_rehearsal.py 2 4 8 > gpurun_out/r06s/rehearsal.jsonl 2>&1
