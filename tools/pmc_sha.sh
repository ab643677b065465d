#!/bin/bash
# Counters of sha256_kernel (tools/sha_probe.py, 1M x 4 KiB): a kernel trace
# pass, then one SQ counter pass (8 SQ counters + GRBM_GUI_ACTIVE).
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_sha}
mkdir -p $OUT
timeout -k 10 120 python3 tools/sha_probe.py > $OUT/probe.json 2> $OUT/probe.err
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace -f csv -- python3 tools/sha_probe.py --reps 5 > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/sq -o sq -f csv -- python3 tools/sha_probe.py --reps 3 > $OUT/sq.log 2>&1
echo done
