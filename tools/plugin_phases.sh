#!/bin/bash
# Host-side phase times of the plugin bench (MEMO_EC_PLUGIN_TIMING=1) at
# 4 KiB blocks, for several pool sizes: where the plugin's store, fetch and
# repair time goes.  Run on the GPU box from the repo root.
set -e
OUT=${OUT:-gpurun_out/plugin_phases}
mkdir -p $OUT
for t in ${THREADS:-4 16}; do
  MEMO_EC_PLUGIN_THREADS=$t MEMO_EC_PLUGIN_TIMING=1 timeout -k 10 120 host/_build/bench_plugin 16384 4096 \
    > $OUT/t$t.json 2> $OUT/t$t.err
done
echo done
