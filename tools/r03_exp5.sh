#!/bin/bash
# C5 sweep with the per-point CPU baseline, then rows-vs-fused rebuild probes
# around the fused path's default bound (64 MiB of survivors per call):
# 4 KiB blocks of RS(16,4) / RS(10,4) and 1 MiB blocks of RS(10,4), from
# 16 MiB to 1 GiB of survivors, two interleaved rounds.  Each GPU step has
# its own time limit; the first failure ends the call.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-exp5}
mkdir -p $OUT
timeout -k 10 700 python bench.py --no-e2e --no-small --no-pmc --sweep > $OUT/sweep.json 2> $OUT/sweep.err
for i in 1 2; do
  for shape in "16 4 4096 4096" "16 4 4096 16384" "16 4 4096 65536" "16 4 4096 262144" \
               "10 4 4096 6144" "10 4 4096 24576" "10 4 4096 98304" \
               "10 4 1048576 16" "10 4 1048576 64" "10 4 1048576 256"; do
    for f in 0 1; do
      MEMO_EC_REBUILD_FUSED=$f timeout -k 10 90 python tools/rebuild_probe.py $shape | sed "s/^{/{\"fused\": $f, /" >> $OUT/probe.jsonl
    done
  done
done
echo done
