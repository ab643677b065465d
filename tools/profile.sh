#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box from
# the repo root).  Kernel trace + stats in one pass; FETCH_SIZE and
# WRITE_SIZE in separate counter passes (MI355X_MICROARCH.md: they cannot
# share a pass; no --pmc with trace domains).  Output under gpurun_out/prof.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
ARGS=${ARGS:---no-cpu --no-e2e}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o trace -f csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o fetch -f csv -- python3 bench.py $ARGS --no-rebuild > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o write -f csv -- python3 bench.py $ARGS --no-rebuild > $OUT/write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50
