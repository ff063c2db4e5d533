# Slow multi-rank / full-size GPU tests (run on the GPU box from the repo root): BASELINE
# configs 4/5 at their multi-rank shape, the 2-rank sharded headline proof and
# the 2^22 x 1024 oracle root check.  A heartbeat file shows progress while the oracle computes.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
(while sleep 30; do date >> gpurun_out/heartbeat.txt; done) &
hb=$!
timeout -k 10 1000 python -u -m pytest tests/test_pcs_sharded.py tests/test_sharded.py \
  -m gpu -x -v --timeout 900 --timeout-method thread --durations=0 \
  -k "configs_4_5 or headline or config5" > gpurun_out/pytest_extra.log 2>&1
rc=$?
kill $hb
echo "exit $rc"
exit $rc
