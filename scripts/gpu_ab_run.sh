export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_sharded.py -m gpu > gpurun_out/ab_tests.txt 2>&1 || exit 1
V=zkvm-brainfuck_amd/variants
AB_REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh $V/libbfz_base.so $V/libbfz_qch.so > gpurun_out/ab1.txt 2>&1 || exit 1
export BFZ_AB_VARIANT=1
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
for v in base qch; do
  cp zkvm-brainfuck_amd/variants/libbfz_$v.so zkvm-brainfuck_amd/libbfz.so
  BFZ_HOST_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_$v -o run \
    -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extra --sustain-s 0 > gpurun_out/kt_$v.log 2>&1
  echo "$v rc $?"
done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
echo done
