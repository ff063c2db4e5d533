# SQ (wave-state) counters for the hot kernels: where waves spend their cycles
# (run on the GPU box from the repo root; counters only, no trace domains).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run \
  -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 > gpurun_out/pmc_sq.log 2>&1
echo "exit $?"
