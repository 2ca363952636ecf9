# pooled tile 71 in the tiny bench plan (104^2, 52^2): step parity (the bench plan and its step keys), tiny bench A/B vs tile 70
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06t71p3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_wino6.py \
  tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 "tests/test_gpu_train.py::test_bench_step_keys_literal_parity" -k "fused_pool or tiny" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for m in "" "71:70"; do
    ADVPATCH_TILE_MAP=$m timeout -k 10 200 python -u bench.py --config tiny --no-cpu-baseline --steps 20 \
      > $O/tiny_map${m/:/_}.$rep.json 2> $O/tiny_map${m/:/_}.$rep.err || { tail $O/tiny_map${m/:/_}.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), d['roofline'].get('frac'))" $O/tiny_map${m/:/_}.$rep.json
  done
done
