# Quick GPU check (run on the GPU box from the repo root): selected parity tests, then a short
# bench line.  Each step has its own time limit; the chain stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-divergence or proof_bytes_match or record_from_events}" > gpurun_out/pytest_quick.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 2 ${BENCH_ARGS} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_quick.log
exit $rc
