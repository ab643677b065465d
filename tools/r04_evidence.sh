#!/bin/bash
# Evidence on the current library: the bench line with the driver's
# arguments, the rocprofv3 kernel trace + counter passes of the bench
# (tools/profile.sh), and the 4 KiB counter set (tools/pmc_4k.sh).  Each GPU
# step has its own time limit; the first failure ends the call.
set -e
TAG=${1:-r04_evidence}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "default_line or stream_probe" > $OUT/gputest.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
OUT=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
OUT=$OUT/pmc_4k bash tools/pmc_4k.sh > $OUT/pmc.log 2>&1
echo done
