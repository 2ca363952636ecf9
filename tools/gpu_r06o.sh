set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o; mkdir -p $O
for v in base form0 form1 eps5 w5 w5f1; do
  for g in ref f64; do
    if [ $v = form0 ] && [ $g = ref ]; then continue; fi
    if [ $g = f64 ] && [ $v != base ] && [ $v != form0 ]; then continue; fi
    ADVPATCH_GEOMETRY=$g ADVPATCH_LIB=tools/var/$v/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py \
      >> $O/micro.txt 2>> $O/micro.err || { echo "variant $v $g failed"; exit 1; }
  done
done
cat $O/micro.txt
