set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06h
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_patch_ops.py \
  tests/test_gpu_eval_folder.py > gpurun_out/r06h/tests_patch.log 2>&1 && \
for g in ref f64; do
  ADVPATCH_GEOMETRY=$g timeout -k 10 200 python -u bench.py --config tiny --no-cpu-baseline --no-tiny --steps 20 \
    > gpurun_out/r06h/tiny_$g.json 2> gpurun_out/r06h/tiny_$g.err
done
true
