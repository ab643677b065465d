#!/bin/bash
# Diagnostic builds of libmemo_ec.so for attributing the 4 KiB rebuild MAC's
# time (wrong results by design; never shipped): a copy of the kernels is
# patched by sed in a temp dir and linked into memo_amd/_lib/variants/.
#   oneset : every lane reads the table set of its tile's first block
#   noimg  : coefficients loaded, product-table images not built/stored
#   nocoef : no coefficient loads (images built from lane indices)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/memo_amd/_lib/variants
mkdir -p $OUT
TMP=$(mktemp -d)
cp $ROOT/memo_amd/csrc/*.hip $ROOT/memo_amd/csrc/*.h $ROOT/memo_amd/csrc/*.cpp $TMP/
mkdir -p $TMP/../include 2>/dev/null || true
build() {  # name, sed script
  local d=$TMP/$1; mkdir -p $d; cp $TMP/*.hip $TMP/*.h $TMP/*.cpp $d/
  sed -i "$2" $d/ec_kernels.hip
  sed -i 's|"../../include/memo_ec.h"|"'$ROOT'/include/memo_ec.h"|' $d/ec_kernels.h $d/memo_ec.cpp
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $d/ec_kernels.hip -o $d/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $d/memo_ec.cpp -o $d/h.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/lib_$1.so $d/k.o $d/h.o
}
build oneset 's|const uint32_t x0 = sg.coef_bstride ? u.set \* (R \* kpad + 1) : 0u;|const uint32_t x0 = 0u;|' &
build noimg 's|if (t < total) {  // waves past the tile|if (false) {  // waves past the tile|; s|if (t + 1024u < total) {|if (false) {|' &
build nocoef 's|cv\[q\] = base\[ci < total ? ci : total - 1u\];|cv[q] = ci * 7u + 3u;|' &
wait
rm -rf $TMP
ls $OUT
