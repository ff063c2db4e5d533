# One round's committed measurements (run on the GPU box from the repo root):
#   bench.json           -- the default bench line (CPU baseline, end-to-end and drop-in figures)
#   prof/                -- rocprofv3 --kernel-trace --stats of a short bench (per-kernel times)
#   kt/ + timeline.txt   -- per-proof GPU busy / idle / under-filled time (scripts/timeline.py)
#   pmc_summary.json     -- FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_pmc.sh)
#   pmc_sq/              -- SQ wave-state counters (scripts/gpu_sq.sh)
#   pcs_c4.json, pcs_c5.json -- BASELINE configs 4 / 5 restated by cell count, on one GPU
# Every step has its own time limit; the chain stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 > gpurun_out/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 > gpurun_out/kt.log 2>&1 && \
python3 scripts/timeline.py gpurun_out/kt/run_kernel_trace.csv > gpurun_out/timeline.txt && \
bash scripts/gpu_pmc.sh > gpurun_out/pmc.out 2>&1 && \
bash scripts/gpu_sq.sh > gpurun_out/sq.out 2>&1 && \
python3 scripts/sq_summary.py gpurun_out > gpurun_out/sq_summary.txt && \
timeout -k 10 300 python bench.py --mode pcs --log-n 22 --cols 256 --steps 3 --warmup 1 > gpurun_out/pcs_c4.json 2> gpurun_out/pcs_c4.err && \
timeout -k 10 300 python bench.py --mode pcs --log-n 22 --cols 1024 --steps 2 --warmup 1 > gpurun_out/pcs_c5.json 2> gpurun_out/pcs_c5.err
rc=$?
echo "exit $rc"
exit $rc
