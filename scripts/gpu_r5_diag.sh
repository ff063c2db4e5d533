# Round-5 first GPU call: smoke, NTT diagnostic variants (scripts/ntt_diag_variant.py) under
# rocprofv3 --stats, a kernel trace of a short bench for per-launch outliers
# (scripts/kernel_outliers.py), then the GPU suite.  Each step has its own time limit.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5diag
O=gpurun_out/r5diag
S=$TMPDIR/r5diag
rm -rf $S && mkdir -p $S
step() { echo "step $1 ($(date +%T))" >> $O/status; }
diag() {  # name [LD_LIBRARY_PATH dir]
  local name=$1 dir=$2
  timeout -k 10 120 env ${dir:+LD_LIBRARY_PATH=$dir} rocprofv3 --kernel-trace --stats --output-format csv -d $S/ntt_$name -o run \
    -- ./scripts/ubench_ntt lde 22 8 5 > $O/ntt_$name.log 2>&1 && \
  cp $S/ntt_$name/run_kernel_stats.csv $O/ntt_${name}_kernel_stats.csv
}
step smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
step ntt && diag base && diag twconst zkvm-brainfuck_amd/variants/twconst && \
  diag noexch zkvm-brainfuck_amd/variants/noexch && diag reps0 zkvm-brainfuck_amd/variants/reps0 && \
step trace && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $S/kt -o run \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > $S/kt.log 2>&1 && \
python3 scripts/kernel_outliers.py $S/kt/run_kernel_trace.csv 16 > $O/outliers.txt && \
python3 scripts/timeline.py $S/kt/run_kernel_trace.csv > $O/timeline.txt && \
step tests && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
step done
rc=$?
echo "exit $rc"; cat $O/status; tail -3 $O/pytest_gpu.log 2>/dev/null
exit $rc
