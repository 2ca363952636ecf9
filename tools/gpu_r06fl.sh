# first layer A/B: the F(2x2) transform's V pairs as one modified v_pk_add each, the bias
# pair as one v_pk_mov, the activation as a template argument (in-tree) vs the committed
# form (tools/var/fp0): first-layer tests, seeded micro with output hashes, tiny bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06fl}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_first_conv.py > $O/tests_first.log 2>&1 || { tail -30 $O/tests_first.log; exit 1; }
tail -1 $O/tests_first.log
for rep in 1 2; do
  ADVPATCH_LIB=tools/var/fp0/libadvpatch_hip.so MICRO_LIB=tools/var/fp0/libadvpatch_hip.so timeout -k 10 120 python -u tools/first_micro.py 50 2>&1 | grep "B=" >> $O/micro_fp0.txt || exit 1
  timeout -k 10 120 python -u tools/first_micro.py 50 2>&1 | grep "B=" >> $O/micro_cur.txt || exit 1
done
echo "== fp0"; cat $O/micro_fp0.txt; echo "== cur"; cat $O/micro_cur.txt
for rnd in 1 2; do
  ADVPATCH_LIB=tools/var/fp0/libadvpatch_hip.so timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline > $O/t_fp0_$rnd.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python -u bench.py --config tiny --no-cpu-baseline > $O/t_cur_$rnd.json 2>> $O/err.log || exit 1
  for w in fp0 cur; do
    python3 -c "
import json
t=json.loads(open('$O/t_${w}_$rnd.json').read().strip().splitlines()[-1])
print('r$rnd $w tiny', round(t['value'],1), round(t['ms_per_step'],3), 'first', round(t['warp_roofline']['first_layer']['us_per_call'],1))" | tee -a $O/summary.txt
  done
done
