# NTT A/B on one box: ubench_ntt lde 22 8 against libbfz variants (LD_LIBRARY_PATH overrides the
# RUNPATH), interleaved, each under rocprofv3 --stats for per-kernel averages; then the NTT /
# hand-over GPU tests and the default bench line.  usage: bash scripts/gpu_r5_ab.sh <tag> <variant>...
# ("cur" = the in-tree libbfz.so).  Each step has its own time limit.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
tag=$1; shift
O=gpurun_out/$tag
S=$TMPDIR/$tag
rm -rf $S $O && mkdir -p $S $O
step() { echo "step $1 ($(date +%T))" >> $O/status; }
ab() {  # name rep
  local name=$1 rep=$2 dir=zkvm-brainfuck_amd/variants/$1
  [ "$name" = cur ] && dir=zkvm-brainfuck_amd
  timeout -k 10 120 env LD_LIBRARY_PATH=$dir rocprofv3 --kernel-trace --stats --output-format csv -d $S/${name}_$rep -o run \
    -- ./scripts/ubench_ntt lde 22 8 5 > $O/ntt_${name}_$rep.log 2>&1 && \
  cp $S/${name}_$rep/run_kernel_stats.csv $O/ntt_${name}_${rep}_kernel_stats.csv
}
step ab
for rep in 1 2; do
  for v in "$@"; do ab $v $rep || { echo "ab $v failed"; exit 1; }; done
done
if [ -z "$SKIP_TESTS" ]; then
  if [ -n "$FULL_TESTS" ]; then
    step tests && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
      > $O/pytest.log 2>&1 || exit 1
  else
    step tests && timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "coset_lde or chunked or record_from_cycles or fibo_x4 or commit_root or repeat or batch" > $O/pytest.log 2>&1 || exit 1
  fi
fi
step bench && timeout -k 10 600 python bench.py --no-cpu-baseline $BENCH_ARGS > $O/bench.json 2> $O/bench.err && \
step done
rc=$?
echo "exit $rc"; cat $O/status; tail -2 $O/pytest.log
exit $rc
