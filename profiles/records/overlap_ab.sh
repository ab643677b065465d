#!/bin/bash
# A/B of the mixed call's stream use on the C5 mix (tools/seg_probe.py,
# clocks settled by 150 untimed calls): VARIANTS of
# decode_overlap:class_streams (MEMO_EC_DECODE_OVERLAP, and
# MEMO_EC_CLASS_STREAMS for the library that had it: see
# profiles/HISTORY.md), interleaved processes, ROUNDS rounds.
set -e
OUT=gpurun_out/${1:-overlap_ab}
mkdir -p $OUT
for i in $(seq ${ROUNDS:-4}); do
  for v in ${VARIANTS:-1:0 0:0}; do
    SEG_PROBE_WARMUP=150 MEMO_EC_DECODE_OVERLAP=${v%%:*} MEMO_EC_CLASS_STREAMS=${v##*:} timeout -k 10 120 \
      python3 tools/seg_probe.py 20 >> $OUT/seg_${v/:/_}.jsonl 2>> $OUT/err.log
  done
done
echo done
