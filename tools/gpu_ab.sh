#!/bin/bash
# GPU call: rebuild parity tests, then interleaved bench runs of the fused
# and the two-kernel rebuild (MEMO_EC_REBUILD_FUSED=1 / 0).
set -e
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rebuild or fused or golden or erasure or singular or small_blocks or full_size or split" > $OUT/gputest.log 2>&1
for i in 1 2; do
  for f in 1 0; do
    MEMO_EC_REBUILD_FUSED=$f timeout -k 10 240 python bench.py --no-cpu --no-e2e > $OUT/bench_f${f}_$i.json 2> $OUT/bench_f${f}_$i.err
  done
done
echo done
