# end-to-end parity with every tile-70 launch remapped to tile 71 (F(4x4,3x3))
set -o pipefail
mkdir -p gpurun_out/r05c
ADVPATCH_TILE_MAP=70:71 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_gpu_train.py::test_headline_plan_b16_608 tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 \
  "tests/test_gpu_step.py::test_step_yolov3_targeted" > gpurun_out/r05c/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r05c/tests.log
