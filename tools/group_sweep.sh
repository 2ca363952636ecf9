#!/bin/bash
# Workgroup-order sweep (PO_CONV_GROUP) over the headline's large launches (GPU box).
set -o pipefail
for G in 0 8 16 32 64; do
  for SPEC in "65:16 19 512 1024 3 1" "65:16 38 256 512 3 1" "65:16 76 128 256 3 1" "65:16 152 64 128 3 1" \
              "15:16 608 32 64 3 2" "13:16 304 64 128 3 2" "11:16 152 128 256 3 2" "11:16 76 256 512 3 2" \
              "27:16 38 512 1024 3 2" "18:16 19 1024 512 1 1"; do
    T=${SPEC%%:*}; SH=${SPEC#*:}
    PO_CONV_GROUP=$G MICRO_TILE=$T timeout -k 10 60 python3 tools/conv_micro.py $SH 30 2>/dev/null | sed "s/^/G=$G tile=$T /" || exit 1
  done
done
