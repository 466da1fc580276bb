set -e
mkdir -p gpurun_out/r06au
timeout -k 10 600 python -u tools/c5_rebuild_ab.py "ORH_UPD_COPY=1" "ORH_UPD_COPY=0" > gpurun_out/r06au/c5_upd_copy_ab.txt 2>&1
bash tools/gpu_round.sh r06au
