set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 1100 python -u -m pytest -v -s --timeout 600 --timeout-method thread \
  tests/test_gpu_step.py tests/test_gpu_train.py \
  > gpurun_out/r06f/tests_step_train.log 2>&1
true
