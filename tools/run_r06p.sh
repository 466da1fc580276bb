set -e
mkdir -p gpurun_out/r06p
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_whatif_repair.py tests/test_gpu_at_scale.py tests/test_gpu_ksp2_abi.py tests/test_gpu_multi_device.py > gpurun_out/r06p/tests.log 2>&1
for rep in 1 2; do
  for V in "" awc0; do
    LD_LIBRARY_PATH=${V:+build_var/$V} timeout -k 10 300 python tools/c4_multi_device_rehearsal.py 8 > gpurun_out/r06p/rehearsal_${V:-shipped}_$rep.jsonl 2>&1
  done
done
