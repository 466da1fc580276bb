set -e
mkdir -p gpurun_out/r06at
timeout -k 10 600 python -u tools/c5_rebuild_ab.py "ORH_NH_ALIAS=1" "ORH_NH_ALIAS=0" > gpurun_out/r06at/c5_alias_ab.txt 2>&1
bash tools/gpu_round.sh r06at
