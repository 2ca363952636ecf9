# in-launch split-K reduction (ABI 28): bit-identity tests, step parity on the
# bench plan, interleaved bench A/B (ADVPATCH_INLAUNCH_REDUCE=1/0), breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06v}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_splitk_inlaunch.py \
  "tests/test_gpu_darknet.py::test_split_k_matches_single_pass" > $O/tests_inl.log 2>&1 || { tail -30 $O/tests_inl.log; exit 1; }
tail -1 $O/tests_inl.log
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_train.py::test_headline_plan_b16_608 tests/test_gpu_train.py::test_tiny_bench_plan_b256_416 \
  > $O/tests_plan.log 2>&1 || { tail -30 $O/tests_plan.log; exit 1; }
tail -1 $O/tests_plan.log
for rep in 1 2; do
  for v in 1 0; do
    ADVPATCH_INLAUNCH_REDUCE=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 \
      > $O/bench_inl$v.$rep.json 2> $O/bench_inl$v.$rep.err || { tail $O/bench_inl$v.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d.get('value_tiny',0)), round(d.get('ms_per_step_tiny',0),3), d['roofline']['conv_launches_per_step'])" $O/bench_inl$v.$rep.json
  done
done
timeout -k 10 300 python -u tools/step_breakdown.py --config yolov3 --steps 5 > $O/step_breakdown_yolov3_b16.txt 2>&1
tail -3 $O/step_breakdown_yolov3_b16.txt
