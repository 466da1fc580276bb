set -e
mkdir -p gpurun_out/r06x
bash tools/c2w_ab_r06.sh gpurun_out/r06x "" ownlds fb2
