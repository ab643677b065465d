#!/bin/bash
# Build tuning variants of libmemo_ec.so (compile-time knobs of the MAC
# kernel) into memo_amd/_lib/variants/.  Tuning only; the product library is
# memo_amd/_lib/libmemo_ec.so built by memo_amd/csrc/Makefile.
set -e
cd "$(dirname "$0")/../memo_amd/csrc"
OUT=../_lib/variants
mkdir -p $OUT
build() {  # name, extra flags
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c ec_kernels.hip -o $OUT/$name.k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -x hip -c memo_ec.cpp -o $OUT/$name.h.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/lib_$name.so $OUT/$name.k.o $OUT/$name.h.o
  rm -f $OUT/$name.k.o $OUT/$name.h.o
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build $name $flags &
done
wait
ls $OUT
