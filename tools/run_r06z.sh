set -e
mkdir -p gpurun_out/r06z
bash tools/ms_ab_r06.sh gpurun_out/r06z "" ORH_HOP_NARROW=1 hw6
