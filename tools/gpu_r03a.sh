#!/bin/bash
# Round 3, first GPU pass: the new parity tests (tiny step, tiny B=256 bench
# plan, headline plan with the fp32-oracle bound), then the bench line.
# A test FAILURE (pytest rc 1) still runs the bench; a timeout, abort or
# fault (any other rc) ends the script.
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
    tests/test_gpu_step.py::test_step_tiny_416 tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 \
    "tests/test_gpu_train.py::test_headline_plan_b16_608[fp32]" "tests/test_gpu_step.py::test_step_yolov3_dota_608[fp32]" \
    tests/test_gpu_step.py::test_step_yolov3_targeted > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
