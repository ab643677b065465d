#!/bin/bash
# Host-side sanitizers (the GPU code is not instrumented): builds
# host/tests/test_erasure with AddressSanitizer + UBSan, and the host side of
# libmemo_ec.so (memo_ec.cpp: launch planning, pipelines, caches) the same
# way into memo_amd/_lib/asan/ next to the in-tree kernels object; then (on
# the GPU box) runs the plugin tests against that library.
#   tools/host_asan.sh build    (here)    tools/host_asan.sh run   (GPU box)
# The two sanitizer builds are listed in .gpurunignore (they are large and
# no round-end run loads them): drop those two lines for a call that runs it.
set -e
cd "$(dirname "$0")/../host"
if [ "$1" = build ]; then
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fPIC -Wall -msse4.2 \
    -I../include tests/test_erasure.cc model.cc erasure_consensus.cc -L../memo_amd/_lib -lmemo_ec \
    -Wl,-rpath,'$ORIGIN/../../memo_amd/_lib' -lcrypto -lpthread -o _build/test_erasure_asan
  mkdir -p ../memo_amd/_lib/asan
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fPIC -Wall \
    -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c ../memo_amd/csrc/memo_ec.cpp -o ../memo_amd/_lib/asan/memo_ec.o
  g++ -shared -fsanitize=address,undefined -o ../memo_amd/_lib/asan/libmemo_ec.so \
    ../memo_amd/_lib/asan/memo_ec.o ../memo_amd/_lib/ec_kernels.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
else
  mkdir -p ../gpurun_out/asan
  ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 LD_LIBRARY_PATH=$PWD/../memo_amd/_lib/asan \
    timeout -k 10 500 _build/test_erasure_asan > ../gpurun_out/asan/out.log 2>&1
fi
