set -e
OUT=gpurun_out/probe_e
mkdir -p $OUT
for e in 1 2 3 4; do
  for shape in "10 4 4096 1048576" "16 4 4096 1048576" "10 4 1048576 4096"; do
    timeout -k 10 60 python tools/rebuild_probe.py $shape $e >> $OUT/probe.jsonl
  done
done
echo done
