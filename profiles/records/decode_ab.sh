#!/bin/bash
# Decode kernel A/B: decode-row tests, then interleaved rebuild_probe runs
# with $VAR=1 and $VAR=0 (default MEMO_EC_DECODE_EXACT: exact-k kernel vs
# the generic one; MEMO_EC_DECODE_STAGE: LDS-staged vs register-direct row
# stores), and one kernel-trace pass of each for the decode kernels' times.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-decode_ab}
VAR=${VAR:-MEMO_EC_DECODE_EXACT}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode_rows or invalid_sets or golden or encode_rebuild or small_blocks or full_size" > $OUT/gputest.log 2>&1
for i in 1 2 3; do
  for x in 1 0; do
    for shape in "16 4 4096 1048576" "10 4 4096 1048576" "10 4 1048576 4096"; do
      env $VAR=$x timeout -k 10 60 python tools/rebuild_probe.py $shape >> $OUT/probe_x$x.jsonl
    done
  done
done
for x in 1 0; do
  env $VAR=$x timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace_x$x -o t -f csv -- python3 tools/rebuild_probe.py 16 4 4096 1048576 > $OUT/trace_x$x.log 2>&1
done
echo done
