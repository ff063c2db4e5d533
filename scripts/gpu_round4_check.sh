# Round-4 check on the GPU box (repo root): selected parity tests, the NTT counter passes, a
# short bench and a kernel trace of back-to-back proofs (idle time per proof).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-divergence or proof_bytes_match or coset_lde or record_from or open}" > gpurun_out/pytest_check.log 2>&1 && \
bash scripts/gpu_ntt_counters.sh > gpurun_out/ntt_counters.out 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --sustain-s 2 --solo-world 0 > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > gpurun_out/kt.log 2>&1 && \
python3 scripts/timeline.py gpurun_out/kt/run_kernel_trace.csv > gpurun_out/timeline.txt
rc=$?
echo "exit $rc"
tail -3 gpurun_out/pytest_check.log
exit $rc
