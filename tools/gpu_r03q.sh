#!/bin/bash
# Tile 68 epilogue: HEAD vs compute-then-store + hoisted pass-1 loads (tools/abl libs), plain and with
# the fused shortcut + sign bits (MICRO_RES=1), interleaved.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-r03q}
mkdir -p $OUT
for rnd in 1 2; do
for res in 0 1; do
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 19 512 1024" "16 19 1024 512"; do
  for lib in ${LIBS:-head hoist}; do
    echo -n "r$rnd res$res $lib $shp: " >> $OUT/micro.txt
    MICRO_RES=$res MICRO_LIB=tools/abl/libadvpatch_$lib.so MICRO_TILE=68 timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 30 2>&1 | tail -1 >> $OUT/micro.txt || exit 1
  done
done
done
done
cat $OUT/micro.txt
