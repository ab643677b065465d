#!/bin/bash
# Library A/B on one box: the in-tree libmemo_ec.so (new) against a build of
# an older revision in abtmp/old (MEMO_EC_LIB), interleaved rebuild_probe
# runs on the 4 KiB / 1 MiB shapes, one kernel-trace pass of each, and the
# decode counters of the new library.  Run from the repo root on the GPU box.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lib_ab}
OLD=${OLD:-abtmp/old/libmemo_ec.so}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTS:-decode_rows or invalid_sets or golden or encode_rebuild or small_blocks or full_size}" > $OUT/gputest.log 2>&1
SHAPES=${SHAPES:-"16_4_4096_1048576 10_4_4096_1048576 10_4_1048576_4096"}
for i in 1 2 3; do
  for v in new old; do
    for shape in $SHAPES; do
      if [ $v = old ]; then export MEMO_EC_LIB=$OLD; else unset MEMO_EC_LIB; fi
      timeout -k 10 60 python tools/rebuild_probe.py ${shape//_/ } >> $OUT/probe_$v.jsonl
    done
  done
done
unset MEMO_EC_LIB
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace_new -o t -f csv -- python3 tools/rebuild_probe.py 16 4 4096 1048576 > $OUT/trace_new.log 2>&1
export MEMO_EC_LIB=$OLD
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace_old -o t -f csv -- python3 tools/rebuild_probe.py 16 4 4096 1048576 > $OUT/trace_old.log 2>&1
unset MEMO_EC_LIB
if [ -n "$PMC" ]; then
  SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  SQ2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  timeout -s KILL 120 rocprofv3 --pmc $SQ1 -d $OUT/pmc1 -o sq1 -f csv -- python3 tools/rebuild_probe.py 16 4 4096 1048576 4 4 > $OUT/pmc1.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ2 -d $OUT/pmc2 -o sq2 -f csv -- python3 tools/rebuild_probe.py 16 4 4096 1048576 4 4 > $OUT/pmc2.log 2>&1
fi
echo done
