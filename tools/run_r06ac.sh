set -e
mkdir -p gpurun_out/r06ac
timeout -k 10 900 python tools/route_ab_r06.py "" "ORH_POOL_PIN=1" > gpurun_out/r06ac/route_ab.txt 2>&1
