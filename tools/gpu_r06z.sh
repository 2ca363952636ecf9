# tile 73 (conv_wpool_k): bit-identity tests, micro timing against tiles 69/61
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06z}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wpool.py \
  > $O/tests_wpool.log 2>&1 || { tail -40 $O/tests_wpool.log; exit 1; }
tail -1 $O/tests_wpool.log
timeout -k 10 200 python -u tools/wpool_micro.py > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
cat $O/micro.txt
