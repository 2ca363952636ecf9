# phase B with the chunk-uniform reference-form fp32 path vs the previous kernel (tools/var/oldb): bits + time, then the warp tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06y}; mkdir -p $O
for rep in 1 2; do
  for g in ref f64; do
    ADVPATCH_GEOMETRY=$g ADVPATCH_LIB=tools/var/oldb/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1
    ADVPATCH_GEOMETRY=$g timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1
  done
done
cat $O/micro.txt
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_patch_ops.py tests/test_gpu_eval_folder.py \
  > $O/tests_patch.log 2>&1 || { tail -30 $O/tests_patch.log; exit 1; }
tail -1 $O/tests_patch.log
