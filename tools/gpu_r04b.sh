set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino5.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b/tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04b/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/wino5_cmp.sh > gpurun_out/r04b/cmp.txt 2>&1; cat gpurun_out/r04b/cmp.txt
MICRO_RES=1 timeout -k 10 600 bash tools/wino5_cmp.sh > gpurun_out/r04b/cmp_res.txt 2>&1; cat gpurun_out/r04b/cmp_res.txt
