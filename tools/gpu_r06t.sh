set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t; mkdir -p $O
for rep in 1 2; do
for v in oldb uni vA vB vC; do ADVPATCH_GEOMETRY=f64 ADVPATCH_LIB=tools/var/$v/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1; done
done
cat $O/micro.txt
