set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 300 python -u tools/geom_box_diag.py > gpurun_out/r06c/diag.txt 2>&1
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_patch_ops.py tests/test_gpu_eval_folder.py tests/test_gpu_first_conv.py \
  > gpurun_out/r06c/tests_patch.log 2>&1
true
