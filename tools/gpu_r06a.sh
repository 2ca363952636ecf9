# round 6: the reference fp32 placement geometry (po_patch_params geometry 1/2),
# the flat-list warp box kernels, the first layer's pool-before-activation
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_geometry_ref.py tests/test_gpu_patch_ops.py tests/test_gpu_eval_folder.py tests/test_gpu_first_conv.py \
  > gpurun_out/r06a/tests_geom.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  tests/test_gpu_step.py tests/test_gpu_train.py::test_headline_plan_b16_608 \
  tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 \
  "tests/test_gpu_train.py::test_bench_step_keys_literal_parity[yolov3-0]" \
  "tests/test_gpu_train.py::test_bench_step_keys_literal_parity[tiny-0]" \
  > gpurun_out/r06a/tests_step.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
