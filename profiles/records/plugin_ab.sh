#!/bin/bash
# Plugin-level A/B on one box: this tree's bench_plugin against another
# build of it (OLD, e.g. an earlier revision's host/ built into abtmp/),
# interleaved, 1 MiB and 4 KiB blocks, one JSON line per run.
set -e
OUT=gpurun_out/${1:-plugin_ab}
OLD=${OLD:-abtmp/old_host/host/_build/bench_plugin}
mkdir -p $OUT
export LD_LIBRARY_PATH=$PWD/memo_amd/_lib
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then B=$OLD; else B=host/_build/bench_plugin; fi
    timeout -k 10 240 $B 512 1048576 >> $OUT/${v}_1m.jsonl 2>> $OUT/${v}.err
    timeout -k 10 240 $B 16384 4096 >> $OUT/${v}_4k.jsonl 2>> $OUT/${v}.err
  done
done
echo done
