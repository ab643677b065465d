#!/bin/bash
# (Measured late round 2 and NOT kept: MEMO_EC_MAC_WAVE_IMG and the wave-local
# build existed only in that experiment; DESIGN.md section 4.1 has the numbers.)
# GPU call: rows-MAC tests, then the two-kernel rebuild with wave-local table
# sets (MEMO_EC_MAC_WAVE_IMG=1, default) against the workgroup-wide build
# (=0), interleaved per round, on 4 KiB random-pattern rebuilds of 1M blocks
# and on C3; every run checks its rebuilt shards (bit_exact).
set -e
OUT=gpurun_out/${1:-wave_img}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_soak.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rows or soak or headline or small_blocks or every_erasure or random_geometries or split or singular or invalid" > $OUT/gputest.log 2>&1
for r in 1 2 3; do
  for shape in "16 4 4096 1048576" "10 4 4096 1048576" "4 2 4096 1048576" "10 4 1048576 4096"; do
    for w in 1 0; do
      MEMO_EC_MAC_WAVE_IMG=$w timeout -k 10 90 python tools/rebuild_probe.py $shape 4 20 | sed "s/^{/{\"wave_img\": $w, /" >> $OUT/ab.jsonl
    done
  done
done
echo done
