#!/bin/bash
# Restored conv_k main loop: conv / eval tests; re-tune (boxed + Winograd
# entries, tiles 67/68 competing) and bench with the CPU baseline.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03f
mkdir -p $OUT/tiles
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eval_folder.py tests/test_gpu_wino.py \
    tests/test_gpu_darknet.py tests/test_gpu_first_conv.py tests/test_gpu_view_move.py tests/test_gpu_patch_ops.py > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/torch_ops_profile.py > $OUT/torch_ops.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/warp_micro.py > $OUT/warp_micro.txt 2>&1 || exit 1
T=adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd/tiles
python tools/retune_boxed.py --wino $T/conv_tiles_yolov3_b16.json $T/conv_tiles_tiny_b256.json > $OUT/retune.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench_tune.json 2> $OUT/bench_tune.err || exit $?
cp $T/*.json $OUT/tiles/
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
