# Round-5 checks: the first-proof stall with the pool synchronising before hipMalloc (diagnostic
# library swapped in place, BFZ_AB_VARIANT=1), the opening / lane GPU tests, the default bench line.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5misc
S=$TMPDIR/r5misc
rm -rf $S $O && mkdir -p $S $O
step() { echo "step $1 ($(date +%T))" >> $O/status; }
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0"
cp zkvm-brainfuck_amd/libbfz.so $S/libbfz_orig.so
step syncmalloc && cp zkvm-brainfuck_amd/variants/syncmalloc/libbfz.so zkvm-brainfuck_amd/libbfz.so && \
  BFZ_AB_VARIANT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $S/kt -o run -- $B > $S/kt.log 2>&1
rc=$?
cp $S/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
[ $rc = 0 ] || { echo "syncmalloc run failed"; tail -5 $S/kt.log; exit 1; }
python3 scripts/kernel_outliers.py $S/kt/run_kernel_trace.csv 12 > $O/outliers_syncmalloc.txt && \
python3 scripts/timeline.py $S/kt/run_kernel_trace.csv > $O/timeline_syncmalloc.txt && \
step tests && timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "open or repeat or batch or chunked or proof_bytes or fibo_x4" > $O/pytest.log 2>&1 && \
step bench && timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
step done
rc=$?
echo "exit $rc"; cat $O/status; tail -2 $O/pytest.log
exit $rc
