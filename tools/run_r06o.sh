set -e
mkdir -p gpurun_out/r06o
bash tools/ms_ab_r06.sh gpurun_out/r06o "" ORH_MS_BLOCK=768 ORH_MS_BLOCK=1024
