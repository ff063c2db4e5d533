# bench + rocprofv3 kernel-trace summary (run on the GPU box from the repo root)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 > gpurun_out/prof.log 2>&1
echo "exit $?"
