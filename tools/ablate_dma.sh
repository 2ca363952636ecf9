#!/bin/bash
# LDS-DMA fp16x3 kernel: full vs no in-kernel split (pure fp16 GEMM upper bound).
set -e
cd "$GRAFT_REPO_ROOT"
SH=${1:-"16 76 128 256 3 1 30"}
for T in ${2:-46 50 51 52}; do
  MICRO_PREC=1 MICRO_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/tile $T full    /"
  MICRO_PREC=1 MICRO_TILE=$T MICRO_LIB=tools/bin/libadvpatch_nosplit.so timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/tile $T nosplit /"
done
