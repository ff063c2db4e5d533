# Round-5 lane check after the batch hang of gpu_r5_batch2: the opening / lane / batch GPU tests
# with every batch step and proof mark printed live (BFZ_HOST_TRACE=live), so a stall names the
# job, the lane and the step it stopped at.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5lanes
rm -rf $O && mkdir -p $O
BFZ_HOST_TRACE=live timeout -k 10 420 python -u -m pytest tests/test_gpu.py -m gpu -x -v -s --timeout 120 \
  --timeout-method thread -k "open or repeat or batch or chunked or proof_bytes or fibo_x4" > $O/pytest.log 2>&1
rc=$?
echo "exit $rc"; grep -E "PASSED|FAILED|ERROR|Timeout" $O/pytest.log | tail -30
exit $rc
