set -e
mkdir -p gpurun_out/r06ap
for v in "" "ORH_WHATIF_SKIP_T2=1" "ORH_WHATIF_SKIP_T2=1 ORH_WHATIF_SEARCH_CAP=128" "ORH_WHATIF_SKIP_T2=1 ORH_WHATIF_SEARCH_CAP=256"; do
  tag=$(echo "${v:-default}" | tr ' =' '__')
  env $v timeout -k 10 400 python -u tools/c4_multi_device_rehearsal.py 4 8 > gpurun_out/r06ap/md_$tag.jsonl 2>&1
done
