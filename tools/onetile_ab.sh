#!/bin/bash
# One-tile shards: the rebuild paths side by side (images through HBM, the
# fused kernel, tables built in LDS), three interleaved rounds of
# tools/rebuild_probe.py per shape.  Run from the repo root on the GPU box.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r06_fused1t
mkdir -p $OUT
for i in 1 2 3; do
  for v in images fused lds; do
    for shape in "16 4 65536 65536" "10 4 40960 102400" "4 2 16384 262144"; do
      case $v in
        images) E="MEMO_EC_REBUILD_FUSED=0" ;;
        fused) E="MEMO_EC_REBUILD_FUSED=1" ;;
        lds) E="MEMO_EC_REBUILD_FUSED=0 MEMO_EC_IMAGE_MIN_TILES=1000000" ;;
      esac
      env $E timeout -k 10 90 python tools/rebuild_probe.py $shape | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/probe.jsonl
    done
  done
done
echo done
