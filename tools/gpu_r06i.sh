set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06i
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_patch_ops.py \
  tests/test_gpu_eval_folder.py > gpurun_out/r06i/tests_patch.log 2>&1 && \
ADVPATCH_GEOMETRY=ref timeout -k 10 200 python -u bench.py --config tiny --no-cpu-baseline --no-tiny --steps 20 \
    > gpurun_out/r06i/tiny_ref.json 2> gpurun_out/r06i/tiny_ref.err && \
ADVPATCH_GEOMETRY=f64 timeout -k 10 200 python -u bench.py --config tiny --no-cpu-baseline --no-tiny --steps 20 \
    > gpurun_out/r06i/tiny_f64.json 2> gpurun_out/r06i/tiny_f64.err
