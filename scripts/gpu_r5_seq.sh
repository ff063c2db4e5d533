# Round-5: a kernel trace of a short bench (the launch sequence of one steady-state proof,
# scripts/proof_sequence.py), then the default bench line.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5seq
S=$TMPDIR/r5seq
rm -rf $O $S && mkdir -p $O $S
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $S/kt -o run \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > $S/kt.log 2>&1 && \
(cd scripts && python3 proof_sequence.py $S/kt/run_kernel_trace.csv 3) > $O/sequence.txt && \
python3 scripts/kernel_outliers.py $S/kt/run_kernel_trace.csv 8 > $O/outliers.txt && \
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?
echo "exit $rc"; tail -25 $O/sequence.txt
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['stages_ms'])"
exit $rc
