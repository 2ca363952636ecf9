set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06q}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_patch_ops.py \
  tests/test_gpu_eval_folder.py > $O/tests_patch.log 2>&1 && \
for g in ref f64; do ADVPATCH_GEOMETRY=$g timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1; done && \
ADVPATCH_GEOMETRY=ref timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ref -o run -- \
  python bench.py --config tiny --no-cpu-baseline --no-tiny --steps 5 --warmup 2 > $O/ref.json 2> $O/ref.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/y3 -o run -- \
  python bench.py --no-cpu-baseline --no-tiny --steps 5 --warmup 2 > $O/y3.json 2> $O/y3.err
