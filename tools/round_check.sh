#!/bin/bash
# Round-end evidence in one GPU call: the full GPU test suite, smoke(), the
# host plugin tests, the default bench line (with the CPU baseline) and the
# rocprofv3 profile (tools/profile.sh).  Each GPU step has its own limit;
# the first failure ends the call.
set -e
TAG=${1:-r02_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
OUT=$OUT/prof bash tools/profile.sh
echo done
