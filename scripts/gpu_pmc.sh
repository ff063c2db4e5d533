# HBM traffic counters for the roofline kernel (run on the GPU box from the repo root).
# FETCH_SIZE and WRITE_SIZE need separate passes on gfx950 (TCC slots, MI355X_MICROARCH.md).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$c -o run \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 > gpurun_out/pmc_$c.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.json
echo "exit $?"
