# One round's committed measurements (run on the GPU box from the repo root).  Raw rocprofv3 CSVs
# go to a scratch directory on the box ($TMPDIR/prof_round); only summaries land in gpurun_out/
# (gpurun copies back at most 64 MiB):
#   bench.json           -- the default bench line (CPU baseline, end-to-end, events, drop-in, solo curve)
#   kernel_stats.csv     -- rocprofv3 --kernel-trace --stats of a short bench (per-kernel times)
#   outliers_stats.txt   -- per-kernel mean / max and the longest launches of that same run
#                           (scripts/kernel_outliers.py: index, grid, phase, neighbours)
#   timeline.txt, outliers_trace.txt -- per-proof busy / idle / under-filled time and outliers of a
#                           separate --kernel-trace run (scripts/timeline.py, kernel_outliers.py)
#   pmc_summary.json     -- FETCH_SIZE / WRITE_SIZE passes with per-kernel mean / max duration
#   sq_summary.txt       -- SQ wave-state counters (scripts/sq_summary.py)
#   pcs_c4.json, pcs_c5.json -- BASELINE configs 4 / 5 restated by cell count, on one GPU
# Every step has its own time limit; the chain stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S=$TMPDIR/prof_round
rm -rf $S && mkdir -p $S
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --no-cold --sustain-s 0 --solo-world 0"
step() { echo "step $1 ($(date +%T))" >> gpurun_out/profile_round.status; }
rm -f gpurun_out/profile_round.status
step bench && timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
step stats && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $S/prof -o run -- $B > $S/prof.log 2>&1 && \
cp $S/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv && \
python3 scripts/kernel_outliers.py $S/prof/run_kernel_trace.csv 16 > gpurun_out/outliers_stats.txt && \
step trace && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $S/kt -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-cold --sustain-s 0 --solo-world 0 > $S/kt.log 2>&1 && \
python3 scripts/timeline.py $S/kt/run_kernel_trace.csv > gpurun_out/timeline.txt && \
python3 scripts/kernel_outliers.py $S/kt/run_kernel_trace.csv 16 > gpurun_out/outliers_trace.txt && \
step fetch && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $S/pmc_FETCH_SIZE -o run -- $B > $S/pmc_f.log 2>&1 && \
step write && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $S/pmc_WRITE_SIZE -o run -- $B > $S/pmc_w.log 2>&1 && \
python3 scripts/pmc_summary.py $S > gpurun_out/pmc_summary.json && \
step sq && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d $S/pmc_sq -o run -- $B > $S/pmc_sq.log 2>&1 && \
python3 scripts/sq_summary.py $S > gpurun_out/sq_summary.txt && \
step pcs4 && timeout -k 10 300 python bench.py --mode pcs --log-n 22 --cols 256 --steps 3 --warmup 1 > gpurun_out/pcs_c4.json 2> gpurun_out/pcs_c4.err && \
step pcs5 && timeout -k 10 300 python bench.py --mode pcs --log-n 22 --cols 1024 --steps 2 --warmup 1 > gpurun_out/pcs_c5.json 2> gpurun_out/pcs_c5.err && \
step done
rc=$?
echo "exit $rc"
cat gpurun_out/profile_round.status
exit $rc
