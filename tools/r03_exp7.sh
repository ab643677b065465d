#!/bin/bash
# Exact-k decode with an m bound of 4 (fewer registers: RS(16,4) 93 -> 68
# VGPRs) against the previous library (abtmp/old): parity + segments tests of
# the new library, interleaved 4 KiB rebuild probes and a kernel trace of
# each (tools/ab_r03.sh); then rows-vs-fused probes around the fused path's
# default bound (64 MiB of survivors per call).
set -e
export TMPDIR=/tmp
TAG=${1:-exp7}
OUT=gpurun_out/$TAG
SHAPES="16_4_4096_1048576 10_4_4096_1048576" bash tools/ab_r03.sh $TAG
for shape in "16 4 4096 4096" "16 4 4096 16384" "16 4 4096 65536" "16 4 4096 262144" \
             "10 4 4096 6144" "10 4 4096 24576" "10 4 4096 98304" \
             "10 4 1048576 16" "10 4 1048576 64" "10 4 1048576 256"; do
  for f in 0 1; do
    MEMO_EC_REBUILD_FUSED=$f timeout -k 10 90 python tools/rebuild_probe.py $shape | sed "s/^{/{\"fused\": $f, /" >> $OUT/fused_probe.jsonl
  done
done
echo done
