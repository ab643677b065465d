#!/bin/bash
# One GPU call: parity tests, then the bench with the fused rebuild and with
# the two-kernel rebuild (A/B), then a rocprofv3 kernel-stats pass of the
# bench.  Every GPU step has its own time limit; the first failure ends it.
set -e
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 240 python bench.py --no-cpu --no-e2e > $OUT/bench_fused.json 2> $OUT/bench_fused.err
MEMO_EC_REBUILD_FUSED=0 timeout -k 10 240 python bench.py --no-cpu --no-e2e > $OUT/bench_rows.json 2> $OUT/bench_rows.err
timeout -k 10 240 python bench.py --no-cpu --no-e2e > $OUT/bench_fused2.json 2> $OUT/bench_fused2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --no-cpu --no-e2e > $OUT/bench_prof.json 2> $OUT/bench_prof.err
echo done
