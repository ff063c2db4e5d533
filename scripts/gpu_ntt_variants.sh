# Same-box NTT A/B of library variants (run on the GPU box from the repo root):
#   VARIANTS="desync1 desync2" REPS=2 bash scripts/gpu_ntt_variants.sh
# Each variant is zkvm-brainfuck_amd/variants/<name>/libbfz.so ("base" = the tree's own library);
# scripts/ubench_ntt lde 22 8 5 (coset LDE of 2^22 x 8) runs under rocprofv3 --kernel-trace --stats
# per variant and rep, interleaved; scripts/ntt_ab_summary.py prints the per-kernel averages.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/ntt_ab
S=$TMPDIR/ntt_ab
rm -rf $O $S && mkdir -p $O $S
for rep in $(seq 1 ${REPS:-2}); do
  for v in base ${VARIANTS}; do
    dir=""
    [ "$v" = base ] || dir=$PWD/zkvm-brainfuck_amd/variants/$v
    timeout -k 10 120 env ${dir:+LD_LIBRARY_PATH=$dir} rocprofv3 --kernel-trace --stats --output-format csv \
      -d $S/${v}_$rep -o run -- ./scripts/ubench_ntt lde 22 8 5 > $O/${v}_$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/${v}_$rep.log; exit 1; }
    cp $S/${v}_$rep/run_kernel_stats.csv $O/${v}_${rep}_kernel_stats.csv
  done
done
python3 scripts/ntt_ab_summary.py $O | tee $O/summary.txt
