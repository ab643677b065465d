#!/bin/bash
# Final evidence of the round in one GPU call: host plugin tests under
# ASan/UBSan (host code only), the GPU test suite, the plain host plugin
# tests, smoke(), the bench line with the driver's arguments (its own
# counter passes included) and the rocprofv3 kernel trace + stats and
# FETCH_SIZE / WRITE_SIZE passes of the bench (tools/profile.sh).  Each GPU
# step has its own time limit; the first failure ends the call.
set -e
TAG=${1:-r03_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/host_asan.sh run && cp gpurun_out/asan/out.log $OUT/asan.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
OUT=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
echo done
