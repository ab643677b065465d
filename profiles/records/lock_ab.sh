set -e
mkdir -p gpurun_out/r06_lockab
for r in 1 2 3; do
 for b in bench_plugin_old bench_plugin; do
  MEMO_EC_PLUGIN_TIMING=1 timeout -k 10 240 host/_build/$b 16384 4096 1 > gpurun_out/r06_lockab/$b.$r.json 2> gpurun_out/r06_lockab/$b.$r.timing
 done
done
timeout -k 10 300 host/_build/test_erasure > gpurun_out/r06_lockab/test_erasure.log 2>&1
tail -1 gpurun_out/r06_lockab/test_erasure.log
