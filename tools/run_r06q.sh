set -e
mkdir -p gpurun_out/r06q
bash tools/ms_ab_r06.sh gpurun_out/r06q "" ORH_HOP_NODES=4
