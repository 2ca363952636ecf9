# the training loaders with spawned DataLoader workers on the GPU box: the on-disk / cached / iterable train()
# runs, resume, the drop-in train; a heartbeat file keeps a long test from looking silent
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06dl; mkdir -p $O
(while sleep 20; do date +%T >> $O/heartbeat; done) & HB=$!
timeout -k 10 500 python -u -m pytest -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_train.py::test_train_on_disk_loader_matches_data_iterable \
  tests/test_gpu_train.py::test_resume_from_train_state_matches_uninterrupted \
  tests/test_gpu_train.py::test_dropin_train_writes_reference_png_layout > $O/tests.log 2>&1
rc=$?
kill $HB
tail -5 $O/tests.log
exit $rc
