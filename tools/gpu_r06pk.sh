# tile 73 A/B: epilogue on accumulator pairs with immediate-offset buffer stores
# and the amax work compiled out (in-tree) vs the committed form (tools/var/wp0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06pk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wpool.py > $O/tests_wpool.log 2>&1 || { tail -30 $O/tests_wpool.log; exit 1; }
tail -1 $O/tests_wpool.log
for rep in 1 2; do
  ADVPATCH_LIB=tools/var/wp0/libadvpatch_hip.so timeout -k 10 120 python -u tools/wpool_micro.py 256 208 30 2>&1 | grep tile >> $O/micro_wp0.txt || exit 1
  timeout -k 10 120 python -u tools/wpool_micro.py 256 208 30 2>&1 | grep tile >> $O/micro_cur.txt || exit 1
done
echo "== wp0"; cat $O/micro_wp0.txt; echo "== cur"; cat $O/micro_cur.txt
for rnd in 1 2; do
  ADVPATCH_LIB=tools/var/wp0/libadvpatch_hip.so timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline > $O/t_wp0_$rnd.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline > $O/t_cur_$rnd.json 2>> $O/err.log || exit 1
  for w in wp0 cur; do
    python3 -c "
import json
t=json.loads(open('$O/t_${w}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd $w tiny', round(t['value'],1), round(t['ms_per_step'],3))" | tee -a $O/summary.txt
  done
done
