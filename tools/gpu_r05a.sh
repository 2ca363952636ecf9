set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread \
  tests/test_gpu_wino5.py tests/test_gpu_step.py tests/test_gpu_train.py::test_headline_plan_b16_608 \
  tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 > gpurun_out/r05a/tests.log 2>&1
