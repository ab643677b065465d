#!/bin/bash
# (Measured late round 2 and NOT kept: the MEMO_EC_DECODE_CHUNKS knob it sets
# existed only in that experiment; DESIGN.md section 9 has the numbers.)
# GPU call: decode/MAC overlap of the two-kernel rebuild (MEMO_EC_DECODE_CHUNKS
# = 1: off, 2/4/8 chunks), interleaved per round on 4 KiB random-pattern
# rebuilds of 1M blocks (RS(16,4), RS(10,4)) and C3; every run checks its
# rebuilt shards against the gather of the encoded parity (bit_exact).
set -e
OUT=gpurun_out/${1:-decode_overlap}
mkdir -p $OUT
for r in 1 2 3; do
  for shape in "16 4 4096 1048576" "10 4 4096 1048576" "10 4 1048576 4096"; do
    for c in 1 2 4 8; do
      MEMO_EC_DECODE_CHUNKS=$c timeout -k 10 90 python tools/rebuild_probe.py $shape 4 20 >> $OUT/ab.jsonl
    done
  done
done
echo done
