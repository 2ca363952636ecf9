#!/bin/bash
# Tile 68 ablations: scalar transform adds (PO_WINO_SCALAR) and s_setprio 1 on
# waves 4-7 (PO_WINO_PRIO), timed with tools/conv_micro.py, interleaved rounds.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03k
mkdir -p $OUT
for rnd in 1 2; do
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 19 512 1024" "16 19 1024 512"; do
  for lib in base scal prio both; do
    echo -n "r$rnd $lib $shp: " >> $OUT/micro.txt
    MICRO_LIB=tools/abl/libadvpatch_$lib.so MICRO_TILE=68 timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 30 2>&1 | tail -1 >> $OUT/micro.txt || exit 1
  done
done
done
cat $OUT/micro.txt
