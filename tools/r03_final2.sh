#!/bin/bash
# Final evidence on the final library (no sanitizer step: its builds stay
# off the pushed tree): the GPU test suite, the host plugin tests, smoke(),
# the bench line with the driver's arguments, the rocprofv3 kernel trace +
# counter passes of the bench (tools/profile.sh), and the C5 sweep with the
# per-point CPU baseline.  Each GPU step has its own time limit; the first
# failure ends the call.
set -e
TAG=${1:-r03_final2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
OUT=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
timeout -k 10 600 python bench.py --no-e2e --no-small --no-pmc --sweep > $OUT/sweep.json 2> $OUT/sweep.err
echo done
