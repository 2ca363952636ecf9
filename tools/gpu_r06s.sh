set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06s; mkdir -p $O
for rep in 1 2; do
ADVPATCH_GEOMETRY=f64 ADVPATCH_LIB=tools/var/oldb/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1
for v in uni uniw5; do for g in f64 ref; do ADVPATCH_GEOMETRY=$g ADVPATCH_LIB=tools/var/$v/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1; done; done
done
cat $O/micro.txt
