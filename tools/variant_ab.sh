#!/bin/bash
# Interleaved rebuild_probe runs of the in-tree library against tuning
# variants (tools/build_variants.sh; MEMO_EC_LIB selects one), on the given
# shapes; each run checks its rebuilt shards (bit_exact).
#   usage: VARIANTS="w4 w4np" SHAPES="16_4_4096_1048576" tools/variant_ab.sh tag
set -e
OUT=gpurun_out/${1:-variant_ab}
mkdir -p $OUT
SHAPES=${SHAPES:-"16_4_4096_1048576 16_4_1048576_4096"}
for i in 1 2 3; do
  for v in base $VARIANTS; do
    for shape in $SHAPES; do
      if [ $v = base ]; then unset MEMO_EC_LIB; else export MEMO_EC_LIB=memo_amd/_lib/variants/lib_$v.so; fi
      timeout -k 10 90 python tools/rebuild_probe.py ${shape//_/ } | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/ab.jsonl
    done
  done
done
echo done
