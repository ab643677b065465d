#!/bin/bash
# A/B of MEMO_EC_DECODE_OVERLAP on the C5 mixed call (tools/seg_probe.py):
# interleaved processes, later decodes on the side stream (1) or all decodes
# first on the call's stream (0), ROUNDS rounds.
set -e
OUT=gpurun_out/${1:-overlap_ab}
mkdir -p $OUT
for i in $(seq ${ROUNDS:-4}); do
  for v in 1 0; do
    MEMO_EC_DECODE_OVERLAP=$v timeout -k 10 120 python3 tools/seg_probe.py 20 >> $OUT/seg_$v.jsonl 2>> $OUT/err.log
  done
done
echo done
