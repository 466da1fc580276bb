set -e
mkdir -p gpurun_out/r06an
for v in 1 2 4; do
  ORH_MD_CHUNKS=$v timeout -k 10 400 python -u tools/c4_multi_device_rehearsal.py 4 8 > gpurun_out/r06an/md_chunks_$v.jsonl 2>&1
done
for v in 1 2 4; do
  ORH_MD_CHUNKS=$v timeout -k 10 400 python -u tools/c4_multi_device_rehearsal.py 8 > gpurun_out/r06an/md_chunks_${v}_rep2.jsonl 2>&1
done
