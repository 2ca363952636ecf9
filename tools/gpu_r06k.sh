set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_patch_ops.py \
  tests/test_gpu_eval_folder.py > $O/tests_patch.log 2>&1 && \
ADVPATCH_GEOMETRY=ref timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ref -o run -- \
  python bench.py --config tiny --no-cpu-baseline --no-tiny --steps 5 --warmup 2 > $O/ref.json 2> $O/ref.err && \
ADVPATCH_GEOMETRY=f64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f64 -o run -- \
  python bench.py --config tiny --no-cpu-baseline --no-tiny --steps 5 --warmup 2 > $O/f64.json 2> $O/f64.err
