# conv_k LDS-DMA tiles: all fragment reads of a k-step before the next k-step's DMA (in-tree) vs HEAD (tools/var/ig0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06ig}; mkdir -p $O
(while sleep 30; do date +%T >> $O/heartbeat; done) & HB=$!
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_darknet.py tests/test_gpu_cones.py \
  tests/test_gpu_splitk_inlaunch.py > $O/tests.log 2>&1 || { kill $HB; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for shape in "16 76 256 128 1 1 30:11" "16 608 32 64 3 2 20:16" "16 304 64 128 3 2 20:13" "16 152 128 256 3 2 20:11" "16 76 256 512 3 2 20:11" "16 38 512 1024 3 2 20:14" "16 19 1024 512 1 1 30:18"; do
  sh=${shape%%:*}; t=${shape##*:}
  for v in ig0 cur ig0 cur; do
    if [ $v = cur ]; then L=""; else L=tools/var/$v/libadvpatch_hip.so; fi
    r=$(MICRO_LIB=$L MICRO_TILE=$t timeout -k 10 120 python -u tools/conv_micro.py $sh 2>&1 | grep -v amdgpu.ids | tail -1) || { kill $HB; echo "$sh $v failed $r"; exit 1; }
    echo "$v tile $t $r" | tee -a $O/micro.txt
  done
done
for rep in 1 2; do
  for v in ig0 cur; do
    if [ $v = cur ]; then L=""; else L=tools/var/$v/libadvpatch_hip.so; fi
    ADVPATCH_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { kill $HB; tail $O/bench_$v.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d.get('value_tiny',0)), d['roofline']['families']['direct'])" $O/bench_$v.$rep.json
  done
done
kill $HB
