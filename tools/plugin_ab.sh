#!/bin/bash
# Same-box A/B of the host plugin: abtmp/hold/bench_plugin (an older build)
# against host/_build/bench_plugin, alternating, 4 KiB and 1 MiB blocks.
set -e
OUT=gpurun_out/${1:-plugin_ab}
mkdir -p $OUT
export LD_LIBRARY_PATH=$PWD/memo_amd/_lib
for i in 1 2 3; do
  for v in new old; do
    B=host/_build/bench_plugin; [ $v = old ] && B=abtmp/hold/bench_plugin
    timeout -k 10 300 $B 16384 4096 2>/dev/null | sed "s/^{/{\"build\": \"$v\", /" >> $OUT/b4k.jsonl
    timeout -k 10 300 $B 512 1048576 2>/dev/null | sed "s/^{/{\"build\": \"$v\", /" >> $OUT/b1m.jsonl
  done
done
echo done
