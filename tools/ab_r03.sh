#!/bin/bash
# Library A/B on one box: the in-tree libmemo_ec.so (new) against another
# build (OLD, default abtmp/old/libmemo_ec.so) -- correctness of the new one
# first (parity + segments tests), then interleaved rebuild_probe runs on
# SHAPES, then one kernel-trace pass of each on the first shape.  Run from
# the repo root on the GPU box.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_r03}
OLD=${OLD:-abtmp/old/libmemo_ec.so}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segments.py -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} > $OUT/gputest.log 2>&1
SHAPES=${SHAPES:-"16_4_4096_1048576 10_4_4096_1048576 10_4_1048576_4096"}
for i in 1 2 3; do
  for v in new old; do
    for shape in $SHAPES; do
      if [ $v = old ]; then export MEMO_EC_LIB=$OLD; else unset MEMO_EC_LIB; fi
      timeout -k 10 90 python tools/rebuild_probe.py ${shape//_/ } | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT/probe.jsonl
    done
  done
done
unset MEMO_EC_LIB
FIRST=${SHAPES%% *}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace_new -o t -f csv -- python3 tools/rebuild_probe.py ${FIRST//_/ } > $OUT/trace_new.log 2>&1
export MEMO_EC_LIB=$OLD
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace_old -o t -f csv -- python3 tools/rebuild_probe.py ${FIRST//_/ } > $OUT/trace_old.log 2>&1
echo done
