set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06p; mkdir -p $O
(cd _ab_r05 && timeout -k 10 120 python -u tools/warp_bwd_micro.py >> ../$O/micro.txt 2>> ../$O/micro.err) || { echo r05 failed; exit 1; }
for v in p3w5 p3w4; do
  for g in ref f64; do
    ADVPATCH_GEOMETRY=$g ADVPATCH_LIB=tools/var/$v/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py \
      >> $O/micro.txt 2>> $O/micro.err || { echo "variant $v $g failed"; exit 1; }
  done
done
cat $O/micro.txt
