#!/bin/bash
# Counter passes of the rebuild MAC at one-tile shards:
# 65,536 x 64 KiB RS(16,4) blocks (one 4 KiB tile per shard), rows path, with
# the per-block table images through HBM (image_min_tiles 1, the default)
# and with tables built in LDS (images off), beside the encode MAC of the
# same blocks (tools/rebuild_probe.py runs both).  Per variant: a kernel
# trace, two SQ passes and the FETCH_SIZE / WRITE_SIZE passes, each its own
# run under its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_onetile}
mkdir -p $OUT
SQ1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_COUNT"
SHAPE=${SHAPE:-16 4 65536 65536}
for v in ${VARIANTS:-images lds}; do
  case $v in
    images) MIN=1 ;;
    lds) MIN=1000000 ;;
  esac
  d=$OUT/$v
  mkdir -p $d
  export MEMO_EC_REBUILD_FUSED=0 MEMO_EC_IMAGE_MIN_TILES=$MIN
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $d/trace -o trace -f csv -- python3 tools/rebuild_probe.py $SHAPE > $d/trace.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc $SQ1 -d $d/sq1 -o sq1 -f csv -- python3 tools/rebuild_probe.py $SHAPE 4 6 > $d/sq1.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc $SQ2 -d $d/sq2 -o sq2 -f csv -- python3 tools/rebuild_probe.py $SHAPE 4 6 > $d/sq2.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $d/fetch -o fetch -f csv -- python3 tools/rebuild_probe.py $SHAPE 4 6 > $d/fetch.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $d/write -o write -f csv -- python3 tools/rebuild_probe.py $SHAPE 4 6 > $d/write.log 2>&1
done
echo done
