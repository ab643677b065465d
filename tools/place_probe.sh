#!/bin/bash
# Builds tools/place_probe.cc against the plugin's objects (host/_build) and
# runs it: full placement, framing only, stores only.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_bin
g++ -std=c++17 -O2 -g -msse4.2 -Iinclude tools/place_probe.cc host/_build/model.o host/_build/erasure_consensus.o \
  -Lmemo_amd/_lib -lmemo_ec -Wl,-rpath,"$PWD/memo_amd/_lib" -lcrypto -lpthread -o tools/_bin/place_probe
for mode in ${MODES:-0 1 2 3 4}; do tools/_bin/place_probe ${1:-65536} $mode; done
