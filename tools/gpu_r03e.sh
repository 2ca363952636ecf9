#!/bin/bash
# PMC of Winograd tiles 67 vs 66 at a long-K shape; the conv / train / eval
# tests; direct conv_k old vs new (two-step register prefetch); re-tune
# (boxed + Winograd entries) and bench.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03e
mkdir -p $OUT/tiles
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_darknet.py tests/test_gpu_patch_ops.py tests/test_gpu_step.py \
    tests/test_gpu_cones.py tests/test_gpu_first_conv.py tests/test_gpu_eval_folder.py \
    "tests/test_gpu_train.py::test_nonfinite_guard_and_flags" tests/test_gpu_train.py::test_empty_shard_adds_only_its_patch_terms \
    tests/test_gpu_placement.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -5 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OUT=$OUT/direct_cmp.txt bash tools/direct_cmp.sh || exit 1
grep -c ImportError $OUT/direct_cmp.txt && exit 1
for shp in "16 304 32 64" "16 152 64 128" "16 76 128 256" "16 38 256 512" "16 38 512 256" "16 19 512 1024" \
           "16 19 1024 512" "256 52 64 128" "256 26 128 256"; do
  for t in 66 67 68; do
    echo -n "$shp tile $t: " >> $OUT/wino_cmp.txt
    MICRO_TILE=$t timeout -k 5 60 python3 tools/conv_micro.py $shp 3 1 20 2>&1 | tail -1 >> $OUT/wino_cmp.txt || exit 1
  done
done
[ $rc -eq 0 ] || exit 1
T=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles
python tools/retune_boxed.py --wino $T/conv_tiles_yolov3_b16.json $T/conv_tiles_tiny_b256.json > $OUT/retune.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench_tune.json 2> $OUT/bench_tune.err || exit $?
cp $T/*.json $OUT/tiles/
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
