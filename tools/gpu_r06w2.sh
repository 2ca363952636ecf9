# tile 73 A/B: the A fragments requested before the MFMAs (in-tree) vs round-6's first form (tools/var/wp0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06w2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wpool.py > $O/tests_wpool.log 2>&1 || { tail -30 $O/tests_wpool.log; exit 1; }
tail -1 $O/tests_wpool.log
for rep in 1 2; do
  ADVPATCH_LIB=tools/var/wp0/libadvpatch_hip.so timeout -k 10 120 python -u tools/wpool_micro.py 256 208 30 2>&1 | grep tile >> $O/micro_wp0.txt || exit 1
  timeout -k 10 120 python -u tools/wpool_micro.py 256 208 30 2>&1 | grep tile >> $O/micro_cur.txt || exit 1
done
echo "== wp0"; cat $O/micro_wp0.txt; echo "== cur"; cat $O/micro_cur.txt
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_train.py::test_golden_yolov3_608_through_hip > $O/golden.log 2>&1; tail -3 $O/golden.log
