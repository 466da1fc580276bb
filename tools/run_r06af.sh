set -e
mkdir -p gpurun_out/r06af
bash tools/c2w_ab_r06.sh gpurun_out/r06af "" ORH_MS_ORDER=host
