set -e
mkdir -p gpurun_out/r06aq
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multi_device.py tests/test_gpu_rank_legs.py tests/test_gpu_whatif_repair.py tests/test_gpu_at_scale.py > gpurun_out/r06aq/tests.log 2>&1
timeout -k 10 400 python -u tools/c4_multi_device_rehearsal.py 2 4 8 > gpurun_out/r06aq/rehearsal.jsonl 2>&1
