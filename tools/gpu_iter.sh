#!/bin/bash
# One GPU iteration call: the GPU tests (SEL selects with -k; empty: all),
# smoke, then optional probes named in PROBES ("image_ab", "host", "bench",
# "sweep", "profile": tools/profile.sh, "pmc4k": tools/pmc_4k.sh, "pmc1t":
# tools/pmc_onetile.sh, "plugin": host/_build/bench_plugin at 4 KiB and 1 MiB).
# Every GPU step has its own time limit; the first failure ends the call.
set -e
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${SEL:+-k "$SEL"} > $OUT/gputest.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
fi
for p in $PROBES; do
  case $p in
    image_ab) timeout -k 10 600 python -u tools/image_ab.py ${AB_ROUNDS:-3} 10 $AB_SHAPES > $OUT/image_ab.jsonl 2> $OUT/image_ab.err ;;
    host) timeout -k 10 300 host/_build/test_erasure > $OUT/host_tests.log 2>&1 ;;
    bench) timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err ;;
    sweep) timeout -k 10 900 python bench.py --sweep --no-pmc --no-plugin --no-sha > $OUT/sweep.json 2> $OUT/sweep.err ;;
    profile) OUT=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1 ;;
    pmc4k) OUT=$OUT/pmc_4k bash tools/pmc_4k.sh > $OUT/pmc_4k.log 2>&1 ;;
    pmc1t) OUT=$OUT/pmc_onetile bash tools/pmc_onetile.sh > $OUT/pmc_onetile.log 2>&1 ;;
    plugin) timeout -k 10 300 host/_build/bench_plugin 16384 4096 ${PLUGIN_REPS:-5} > $OUT/plugin_4k.json 2> $OUT/plugin_4k.err
            timeout -k 10 300 host/_build/bench_plugin 512 1048576 ${PLUGIN_REPS:-5} > $OUT/plugin_1m.json 2> $OUT/plugin_1m.err ;;
  esac
done
echo done
