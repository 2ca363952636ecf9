set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAGOUT:-r04d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino5.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/wino5_cmp.sh > $OUT/cmp.txt 2>&1; cat $OUT/cmp.txt
AB_ENV="ADVPATCH_TILE_MAP=68:70" TAGOUT= timeout -k 10 900 tools/gpu_ab.sh ${TAGOUT:-r04d}/ab 2
