#!/bin/bash
# GPU tests on the in-tree library, host plugin tests, then interleaved
# rebuild_probe runs of compile-time variants (tools/build_variants.sh) and
# the in-tree library ("new"), then the C5 sweep of the in-tree library.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-exp2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
SHAPES=${SHAPES:-"16_4_4096_1048576 10_4_4096_1048576 10_4_1048576_4096"}
for i in 1 2 3; do
  for v in new $VARIANTS; do
    for shape in $SHAPES; do
      if [ $v = new ]; then unset MEMO_EC_LIB; else export MEMO_EC_LIB=memo_amd/_lib/variants/lib_$v.so; fi
      timeout -k 10 90 python tools/rebuild_probe.py ${shape//_/ } | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/probe.jsonl
    done
  done
done
unset MEMO_EC_LIB
[ -n "$NOSWEEP" ] || timeout -k 10 500 python bench.py --no-cpu --no-e2e --no-small --no-pmc --sweep > $OUT/sweep.json 2> $OUT/sweep.err
echo done
