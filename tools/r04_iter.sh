#!/bin/bash
# One GPU call of this round's iteration: the selected GPU tests, the host
# plugin tests, the bench line with the driver's arguments, then the 4 KiB
# rebuild counter passes.  Each GPU step has its own time limit; the first
# failure ends the call.
set -e
TAG=${1:-r04_iter}
SEL=${SEL-n2_line}  # SEL= (empty): every GPU test
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  ${SEL:+-k "$SEL"} > $OUT/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
if [ -z "$NO_PMC" ]; then OUT=$OUT/pmc_4k bash tools/pmc_4k.sh > $OUT/pmc.log 2>&1; fi
echo done
