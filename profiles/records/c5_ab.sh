#!/bin/bash
# Library A/B on one box for the C5 mixed call and the C3 / 4 KiB rebuild
# shapes: this tree's libmemo_ec.so against another build (OLD), interleaved
# processes (tools/seg_probe.py, tools/rebuild_probe.py), 3 rounds.
set -e
OUT=gpurun_out/${1:-c5_ab}
OLD=${OLD:-abtmp/r04/memo_amd/_lib/libmemo_ec.so}
mkdir -p $OUT
for i in 1 2 3; do
  for v in new old; do
    L=""; [ $v = old ] && L=$OLD
    timeout -k 10 120 python3 tools/seg_probe.py 10 4 $L >> $OUT/seg_$v.jsonl 2>> $OUT/err.log
    for shape in "10 4 1048576 4096" "16 4 1048576 4096" "16 4 4096 1048576"; do
      MEMO_EC_PROBE_LIB=$L timeout -k 10 120 python3 tools/rebuild_probe.py $shape >> $OUT/probe_$v.jsonl 2>> $OUT/err.log
    done
  done
done
echo done
