# Dynamic counters of the coset-LDE kernels at a known element-stage count:
# scripts/ubench_ntt lde 22 8 3 (one warm + 3 timed coset LDEs of a 2^22 x 8 matrix: DIT tile,
# k_lde_mid<22>, DIF tile) under rocprofv3, one --pmc pass per counter group; then
# scripts/ntt_counters.py turns them into per-kernel instructions per element-stage, VALU issue
# and L2 / traffic figures.  Run on the GPU box from the repo root.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
W="./scripts/ubench_ntt lde 22 8 3"
rm -rf gpurun_out/ntt_pmc_*
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/ntt_pmc_$name -o run \
    -- $W > gpurun_out/ntt_pmc_$name.log 2>&1
}
pass inst SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES && \
pass busy SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE && \
pass l2 TCC_HIT_sum TCC_MISS_sum && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ntt_pmc_stats -o run -- $W > gpurun_out/ntt_pmc_stats.log 2>&1 && \
python3 scripts/ntt_counters.py gpurun_out > gpurun_out/ntt_counters.json
rc=$?
echo "exit $rc"
exit $rc
