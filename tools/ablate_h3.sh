#!/bin/bash
# fp16x3 conv ablations on one shape: full / no staging loads / no LDS stores.
set -e
cd "$GRAFT_REPO_ROOT"
SH=${1:-"16 76 128 256 3 1 30"}
for T in ${2:-34 29 41}; do
  MICRO_PREC=1 MICRO_TILE=$T timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/tile $T full    /"
  MICRO_PREC=1 MICRO_TILE=$T MICRO_LIB=tools/bin/libadvpatch_noload.so timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/tile $T noload  /"
  MICRO_PREC=1 MICRO_TILE=$T MICRO_LIB=tools/bin/libadvpatch_nostore.so timeout -k 10 60 python tools/conv_micro.py $SH | grep -v amdgpu.ids | sed "s/^/tile $T nostore /"
done
