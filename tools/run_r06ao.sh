set -e
mkdir -p gpurun_out/r06ao
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/r06ao/trace -o run -- python3 $REPO/tools/md_block_prof.py 8 0 5 > $REPO/gpurun_out/r06ao/block.log 2>&1
