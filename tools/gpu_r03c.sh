#!/bin/bash
# Winograd tile 67: parity tests, per-shape timings against tiles 65/66, then
# a re-tune of the boxed and Winograd cache entries and the bench line.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03c
mkdir -p $OUT/tiles
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wino.py \
    > $OUT/wino_tests.log 2>&1 || { echo "wino tests rc=$?"; tail -30 $OUT/wino_tests.log; exit 1; }
tail -3 $OUT/wino_tests.log
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 76 256 128" "16 38 256 512" "16 38 512 256" \
           "16 19 512 1024" "16 19 1024 512" "256 104 32 64" "256 52 64 128" "256 26 128 256"; do
  for t in 65 66 67; do
    echo -n "$shp tile $t: " >> $OUT/wino_cmp.txt
    MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1 >> $OUT/wino_cmp.txt || exit 1
  done
done
cat $OUT/wino_cmp.txt
T=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles
python tools/retune_boxed.py --wino $T/conv_tiles_yolov3_b16.json $T/conv_tiles_tiny_b256.json > $OUT/retune.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench_tune.json 2> $OUT/bench_tune.err || exit $?
cp $T/*.json $OUT/tiles/
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
