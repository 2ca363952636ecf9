#!/bin/bash
# Tile 69 occupancy variants (2/3/4 workgroups per CU) on the tiny 208^2 pooled conv.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03t
mkdir -p $OUT
for rnd in 1 2; do
for lib in occ2 default occ4; do
  L=tools/abl/libadvpatch_$lib.so; [ $lib = default ] && L=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/libadvpatch_hip.so
  echo -n "r$rnd $lib: " >> $OUT/micro.txt
  MICRO_LIB=$L MICRO_POOL=1 MICRO_TILE=69 timeout -k 5 60 python3 tools/conv_micro.py 256 208 16 32 3 1 20 2>&1 | tail -1 >> $OUT/micro.txt || exit 1
done; done
cat $OUT/micro.txt
