#!/bin/bash
# (Measured late round 2 and NOT kept: MEMO_EC_DECODE_TABLE and the row table
# existed only in that experiment; DESIGN.md section 9 has the numbers.)
# GPU call: parity tests of the decode row table, then the two-kernel
# rebuild with the table on / off (MEMO_EC_DECODE_TABLE=1/0), interleaved per
# round on 4 KiB random-pattern rebuilds of 1M blocks and on C3; every run
# checks its rebuilt shards (bit_exact).  Then one rocprofv3 kernel trace of
# each setting on the RS(16,4) shape (decode kernel time apart from the MAC).
set -e
OUT=gpurun_out/${1:-decode_table}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "decode_row or invalid or headline or small_blocks or singular or every_erasure or random_geometries" > $OUT/gputest.log 2>&1
for r in 1 2 3; do
  for shape in "16 4 4096 1048576" "10 4 4096 1048576" "10 4 1048576 4096"; do
    for t in 1 0; do
      MEMO_EC_DECODE_TABLE=$t timeout -k 10 90 python tools/rebuild_probe.py $shape 4 20 >> $OUT/ab.jsonl
    done
  done
done
for t in 1 0; do
  MEMO_EC_DECODE_TABLE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_t$t -o run -f csv -- python tools/rebuild_probe.py 16 4 4096 1048576 4 20 > $OUT/prof_t$t.log 2>&1
done
echo done
