#!/bin/bash
# One GPU call: the GPU test suite, the host plugin tests, smoke(), the
# default bench line (counter passes included) and the C5 sweep.  Each GPU
# step has its own time limit; the first failure ends the call.
set -e
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 500 python bench.py --no-cpu --no-e2e --no-small --no-pmc --sweep > $OUT/sweep.json 2> $OUT/sweep.err
echo done
