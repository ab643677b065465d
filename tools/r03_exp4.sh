#!/bin/bash
# ASan/UBSan run of the host plugin tests (tools/host_asan.sh run), then
# interleaved rows-vs-fused rebuild probes on the 4 KiB shapes and C3.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-exp4}
mkdir -p $OUT
bash tools/host_asan.sh run && cp gpurun_out/asan/out.log $OUT/asan.log
for i in 1 2 3; do
  for f in 0 1; do
    for shape in 16_4_4096_1048576 10_4_4096_1048576 10_4_1048576_4096; do
      MEMO_EC_REBUILD_FUSED=$f timeout -k 10 90 python tools/rebuild_probe.py ${shape//_/ } | sed "s/^{/{\"fused\": $f, /" >> $OUT/probe.jsonl
    done
  done
done
echo done
