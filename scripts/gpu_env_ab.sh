# A/B of an environment switch of the NTT kernels (VAR=0 vs VAR=1, e.g. VAR=BFZ_TILE_WS), run on
# the GPU box from the repo root: tile passes and coset LDEs (output hashes must agree), the LDE
# and proof parity tests with VAR=1, then the bench with each, twice.  Output: gpurun_out/ab_$VAR.txt
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${VAR:?VAR}
O=gpurun_out/ab_$V.txt
: > $O
for i in 1 2; do
  for v in 0 1; do
    echo "== $V=$v tiles" >> $O
    timeout -k 10 120 env $V=$v ./scripts/ubench_ntt >> $O 2>&1 || exit 1
    for L in 22 21; do
      echo "== $V=$v lde $L" >> $O
      timeout -k 10 60 env $V=$v ./scripts/ubench_ntt lde $L 8 10 >> $O 2>&1 || exit 1
    done
  done
done
timeout -k 10 600 env $V=1 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "coset_lde or proof_bytes_match or commit_root" > gpurun_out/pytest_$V.log 2>&1 || exit 1
for r in a b; do
  for v in 0 1; do
    timeout -k 10 300 env $V=$v python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > gpurun_out/bench_${V}_$v$r.json 2> gpurun_out/bench_${V}_$v$r.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/bench_${V}_$v$r.json')); print('bench $V=$v', d['value'], 'ntt_kernel_ms', d['stages_ms']['ntt_kernel_ms'])" >> $O
  done
done
tail -3 gpurun_out/pytest_$V.log >> $O
cat $O
