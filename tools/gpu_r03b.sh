#!/bin/bash
# Re-time the boxed launches of both committed tile caches (training-like
# tuning footprints, live-tile-aware split-K candidates), then bench.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03b
mkdir -p $OUT/tiles
T=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles
python tools/retune_boxed.py $T/conv_tiles_yolov3_b16.json $T/conv_tiles_tiny_b256.json > $OUT/retune.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench_tune.json 2> $OUT/bench_tune.err || exit $?
cp $T/*.json $OUT/tiles/
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
