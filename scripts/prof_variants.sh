# Kernel stats (rocprofv3 --kernel-trace --stats) of several libbfz builds, same box:
#   bash scripts/prof_variants.sh zkvm-brainfuck_amd/variants/libbfz_a.so ...
# Writes gpurun_out/kstats_<name>.csv (one per build).
export TMPDIR=/tmp
export BFZ_AB_VARIANT=1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
for so in "$@"; do
  v=$(basename $so .so)
  cp "$so" zkvm-brainfuck_amd/libbfz.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_$v -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 > /tmp/kst_$v.log 2>&1 || { cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so; exit 1; }
  cp $(find /tmp/kst_$v -name 'run_kernel_stats.csv' | head -1) gpurun_out/kstats_$v.csv
done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
