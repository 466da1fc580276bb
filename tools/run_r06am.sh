set -e
mkdir -p gpurun_out/r06am
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ksp2_abi.py tests/test_gpu_at_scale.py::test_c4_ksp2_all_benched_pairs tests/test_ka_decision_more.py tests/test_ka_decision.py > gpurun_out/r06am/tests.log 2>&1
bash tools/ksp2_ab_r06.sh gpurun_out/r06am ""
grep -h "ksp-prof paths\|prefetch_kth" gpurun_out/r06am/ksp2_shipped_*.log > gpurun_out/r06am/paths.txt
timeout -k 10 900 python tools/route_ab_r06.py "" "ORH_FILL_CHUNKS=1" > gpurun_out/r06am/route_ab.txt 2>&1
