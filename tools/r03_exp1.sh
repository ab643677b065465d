#!/bin/bash
# GPU tests (whole-batch parity included), host plugin tests, rows vs fused
# rebuild probes on the 4 KiB shapes, and the C5 sweep (mixed rebuild with
# batched decode launches).  Each step has its own limit.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-exp1}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
for i in 1 2; do
  for f in 0 1; do
    for shape in 16_4_4096_1048576 10_4_4096_1048576; do
      MEMO_EC_REBUILD_FUSED=$f timeout -k 10 90 python tools/rebuild_probe.py ${shape//_/ } | sed "s/^{/{\"fused\": $f, /" >> $OUT/probe.jsonl
    done
  done
done
timeout -k 10 500 python bench.py --no-cpu --no-e2e --no-small --no-pmc --sweep > $OUT/sweep.json 2> $OUT/sweep.err
echo done
