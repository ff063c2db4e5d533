# MFMA vs all-VALU 2^14 NTT tiles (run on the GPU box from the repo root): the tile pass alone
# (scripts/ubench_ntt, output hashes must agree; variants in zkvm-brainfuck_amd/variants/<name>/),
# the LDE parity tests, then the bench with each.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 env BFZ_NTT_MFMA=0 ./scripts/ubench_ntt > gpurun_out/ubench_ntt_valu.txt 2>&1 && \
timeout -k 10 120 env BFZ_NTT_MFMA=1 ./scripts/ubench_ntt > gpurun_out/ubench_ntt_mfma.txt 2>&1 && \
for v in ${VARIANTS}; do
  timeout -k 10 120 env LD_LIBRARY_PATH=$PWD/zkvm-brainfuck_amd/variants/$v ./scripts/ubench_ntt > gpurun_out/ubench_ntt_$v.txt 2>&1 || exit 1
done && \
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-coset_lde or proof_bytes_match or commit_root}" > gpurun_out/pytest_ntt.log 2>&1 && \
timeout -k 10 300 env BFZ_NTT_MFMA=0 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > gpurun_out/bench_valu.json 2> gpurun_out/bench_valu.err && \
timeout -k 10 300 env BFZ_NTT_MFMA=1 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > gpurun_out/bench_mfma.json 2> gpurun_out/bench_mfma.err
rc=$?
echo "exit $rc"
grep -h "4096" gpurun_out/ubench_ntt_*.txt
tail -3 gpurun_out/pytest_ntt.log
exit $rc
