# rocprofv3 --kernel-trace --stats of a short bench for each libbfz variant named in $VARIANTS
# (zkvm-brainfuck_amd/variants/libbfz_<name>.so), summaries to gpurun_out/stats_<name>.csv.
export TMPDIR=/tmp BFZ_AB_VARIANT=1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
rc=0
for v in $VARIANTS; do
  cp zkvm-brainfuck_amd/variants/libbfz_$v.so zkvm-brainfuck_amd/libbfz.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/vs_$v -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > gpurun_out/stats_$v.log 2>&1 || { rc=1; break; }
  cp /tmp/vs_$v/run_kernel_stats.csv gpurun_out/stats_$v.csv
done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
exit $rc
