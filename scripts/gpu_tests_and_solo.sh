# GPU parity tests + smoke, then the bench with the per-rank solo timing of an 8-GPU sharded
# proof (run on the GPU box from the repo root).  Each step has its own time limit.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu-baseline --solo-world 8 ${BENCH_ARGS} > gpurun_out/bench_solo.json 2> gpurun_out/bench_solo.err
rc=$?
echo "exit $rc"
exit $rc
