#!/bin/bash
# Attribute the rebuild MAC's gap to encode: for each
# shape and rebuild path, one kernel-trace pass and separate counter passes
# (SQ stall/issue counters; FETCH_SIZE; WRITE_SIZE) of tools/rebuild_probe.py.
# Each pass under its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_rebuild}
mkdir -p $OUT
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS"
for shape in "16 4 4096 1048576" "10 4 4096 1048576" "10 4 1048576 4096"; do
  tag=$(echo $shape | tr ' ' '_')
  for path in 0 1; do
    d=$OUT/${tag}_f$path
    mkdir -p $d
    MEMO_EC_REBUILD_FUSED=$path timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/trace -o trace -f csv -- python3 tools/rebuild_probe.py $shape > $d/trace.log 2>&1
    MEMO_EC_REBUILD_FUSED=$path timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $d/sq1 -o sq1 -f csv -- python3 tools/rebuild_probe.py $shape 4 6 > $d/sq1.log 2>&1
    MEMO_EC_REBUILD_FUSED=$path timeout -s KILL 120 rocprofv3 --pmc $SQ2 -d $d/sq2 -o sq2 -f csv -- python3 tools/rebuild_probe.py $shape 4 6 > $d/sq2.log 2>&1
    MEMO_EC_REBUILD_FUSED=$path timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o fetch -f csv -- python3 tools/rebuild_probe.py $shape 4 6 > $d/fetch.log 2>&1
    MEMO_EC_REBUILD_FUSED=$path timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $d/write -o write -f csv -- python3 tools/rebuild_probe.py $shape 4 6 > $d/write.log 2>&1
  done
done
echo done
