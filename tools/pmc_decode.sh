#!/bin/bash
# Counters of the decode kernels on 1M x 4 KiB RS(16,4) / RS(10,4) blocks
# (tools/rebuild_probe.py), one counter pass each.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_decode}
mkdir -p $OUT
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
SQ2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for shape in "16 4 4096 1048576" "10 4 4096 1048576"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/${tag}_sq1 -o sq1 -f csv -- python3 tools/rebuild_probe.py $shape 4 4 > $OUT/${tag}_sq1.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 -d $OUT/${tag}_sq2 -o sq2 -f csv -- python3 tools/rebuild_probe.py $shape 4 4 > $OUT/${tag}_sq2.log 2>&1
done
echo done
