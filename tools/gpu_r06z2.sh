# tile 73 in the tiny bench plan: step parity (the bench plan and its step keys), tiny bench A/B vs tile 69
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06z2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_wpool.py \
  tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 "tests/test_gpu_train.py::test_bench_step_keys_literal_parity" -k "wpool or tiny" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for m in "" "73:69"; do
    ADVPATCH_TILE_MAP=$m timeout -k 10 200 python -u bench.py --config tiny --no-cpu-baseline --steps 20 \
      > $O/tiny_map${m/:/_}.$rep.json 2> $O/tiny_map${m/:/_}.$rep.err || { tail $O/tiny_map${m/:/_}.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), d['roofline'].get('frac'))" $O/tiny_map${m/:/_}.$rep.json
  done
done
