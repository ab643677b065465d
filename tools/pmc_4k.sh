#!/bin/bash
# Counter set of the 4 KiB per-block-pattern rebuild against the encode of
# the same blocks: a kernel trace and two
# SQ counter passes (+ GRBM_GUI_ACTIVE for the clock) of
# tools/rebuild_probe.py on 1M x 4 KiB blocks, RS(16,4) and RS(10,4), rows
# path.  Each pass under its own time limit; the first failure ends it.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_4k}
mkdir -p $OUT
SQ1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_COUNT"
# SHAPES: k_m_B_n shapes (default: the two 4 KiB shapes)
for tag in ${SHAPES:-16_4_4096_1048576 10_4_4096_1048576}; do
  shape=${tag//_/ }
  d=$OUT/${tag}_f0
  mkdir -p $d
  MEMO_EC_REBUILD_FUSED=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/trace -o trace -f csv -- python3 tools/rebuild_probe.py $shape > $d/trace.log 2>&1
  MEMO_EC_REBUILD_FUSED=0 timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $d/sq1 -o sq1 -f csv -- python3 tools/rebuild_probe.py $shape 4 6 > $d/sq1.log 2>&1
  MEMO_EC_REBUILD_FUSED=0 timeout -s KILL 120 rocprofv3 --pmc $SQ2 -d $d/sq2 -o sq2 -f csv -- python3 tools/rebuild_probe.py $shape 4 6 > $d/sq2.log 2>&1
done
echo done
