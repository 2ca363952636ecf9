#!/bin/bash
# round 4: phase B table + 32 image groups, Philox 64-bit products;
# tests, bench, launch census
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04j
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_gpu_patch_ops.py tests/test_gpu_placement.py tests/test_gpu_train.py \
    > "$OUT/tests.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" "$OUT/tests.log" | tail -25
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_step.py \
    -k "test_step_tiny_416 or test_step_yolov3_targeted or test_step_yolov3_dota_608 or test_two_adam" > "$OUT/step.log" 2>&1
rc=$?
grep -E "patch grad|PASSED|FAILED|passed|failed|Error" "$OUT/step.log" | tail -30
[ $rc -eq 0 ] || { echo "step pytest rc=$rc"; exit $rc; }
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-300 "$OUT/bench.json"
bash tools/launch_census.sh r04j tiny 256
echo done
