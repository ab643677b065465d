#!/bin/bash
# Host-side sanitizers for the plugin (the GPU code is not instrumented):
# builds host/tests/test_erasure with AddressSanitizer + UBSan against the
# in-tree libmemo_ec.so, then (on the GPU box) runs it.
#   tools/host_asan.sh build    (here)    tools/host_asan.sh run   (GPU box)
set -e
cd "$(dirname "$0")/../host"
if [ "$1" = build ]; then
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fPIC -Wall -msse4.2 \
    -I../include tests/test_erasure.cc model.cc erasure_consensus.cc -L../memo_amd/_lib -lmemo_ec \
    -Wl,-rpath,'$ORIGIN/../../memo_amd/_lib' -lcrypto -lpthread -o _build/test_erasure_asan
else
  mkdir -p ../gpurun_out/asan
  ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    timeout -k 10 500 _build/test_erasure_asan > ../gpurun_out/asan/out.log 2>&1
fi
