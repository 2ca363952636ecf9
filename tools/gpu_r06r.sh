# same-box A/B of the warp backward's phase B: round-5 tree, the current
# kernel, and the round-5 kernel inside the current library (f64 rows)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06r; mkdir -p $O
for rep in 1 2; do
(cd _ab_r05 && timeout -k 10 120 python -u tools/warp_bwd_micro.py >> ../$O/micro.txt 2>> ../$O/micro.err) || { echo r05 failed; exit 1; }
ADVPATCH_GEOMETRY=f64 ADVPATCH_LIB=tools/var/oldb/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1
for g in f64 ref; do ADVPATCH_GEOMETRY=$g ADVPATCH_LIB=tools/var/cur/libadvpatch_hip.so timeout -k 10 120 python -u tools/warp_bwd_micro.py >> $O/micro.txt 2>> $O/micro.err || exit 1; done
done
cat $O/micro.txt
