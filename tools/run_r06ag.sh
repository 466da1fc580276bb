set -e
mkdir -p gpurun_out/r06ag
LD_LIBRARY_PATH=build_var/wsplit timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_weighted.py > gpurun_out/r06ag/tests_split.log 2>&1
bash tools/c2w_ab_r06.sh gpurun_out/r06ag "" wsplit
