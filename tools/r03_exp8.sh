#!/bin/bash
# k = 16 bodies with per-block tables without shard pairing (124 VGPRs, 4
# waves per SIMD; abtmp/p0, built with -DMEMO_EC_MAC_PAIR16_COEF=0) against
# the in-tree library (paired, 153 VGPRs): parity + segments tests of the
# in-tree library, then interleaved probes of both on the rows path (1M x
# 4 KiB, 4096 x 1 MiB) and the fused path (65,536 x 4 KiB = 256 MiB).
set -e
export TMPDIR=/tmp
TAG=${1:-exp8}
OLD=abtmp/p0/libmemo_ec.so SHAPES="16_4_4096_1048576 16_4_1048576_4096 16_4_4096_65536 10_4_4096_1048576" bash tools/ab_r03.sh $TAG
echo done
