set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 120 python -u tools/warp_forms_diag.py > gpurun_out/r06e/forms_flat.txt 2>&1
timeout -k 10 300 python -u tools/geom_box_diag.py > gpurun_out/r06e/diag.txt 2>&1
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_geometry_ref.py tests/test_gpu_patch_ops.py tests/test_gpu_eval_folder.py tests/test_gpu_first_conv.py \
  > gpurun_out/r06e/tests_patch.log 2>&1
timeout -k 10 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread \
  tests/test_gpu_step.py tests/test_gpu_train.py::test_headline_plan_b16_608 \
  tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 \
  "tests/test_gpu_train.py::test_bench_step_keys_literal_parity[yolov3-0]" \
  "tests/test_gpu_train.py::test_bench_step_keys_literal_parity[tiny-0]" \
  > gpurun_out/r06e/tests_step.log 2>&1
true
