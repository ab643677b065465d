#!/bin/bash
# rocprofv3 evidence for bench.py's kernels (run on the GPU box from the repo
# root): kernel trace + stats in one pass; FETCH_SIZE and WRITE_SIZE in
# separate counter passes (MI355X_MICROARCH.md: they cannot share a pass; no
# --pmc with trace domains).  Output under gpurun_out/prof.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
ARGS=${ARGS:---no-cpu --no-e2e --no-small --no-pmc --no-verify --no-c5 --no-plugin --no-sha}
PMC_ARGS=${PMC_ARGS:---no-cpu --no-e2e --no-small --no-pmc --no-verify --no-c5 --no-plugin --no-sha --steps 4 --warmup 2 --settle-ms 0}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace -f csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch -f csv -- python3 bench.py $PMC_ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write -f csv -- python3 bench.py $PMC_ARGS > $OUT/write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50
