#!/bin/bash
# Decode with the survivor x non-survivor logs kept (m <= 4) against the
# previous library (abtmp/old): parity + segments tests of the new library,
# interleaved 4 KiB rebuild probes of both and a kernel trace of each
# (tools/ab_r03.sh), then the C5 sweep with the per-point CPU baseline.
set -e
export TMPDIR=/tmp
TAG=${1:-exp6}
SHAPES="16_4_4096_1048576 10_4_4096_1048576" bash tools/ab_r03.sh $TAG
timeout -k 10 700 python bench.py --no-e2e --no-small --no-pmc --sweep > gpurun_out/$TAG/sweep.json 2> gpurun_out/$TAG/sweep.err
echo done
