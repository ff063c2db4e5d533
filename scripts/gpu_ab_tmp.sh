export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true && \
timeout -k 10 900 bash scripts/ab_bench.sh zkvm-brainfuck_amd/variants/libbfz_r8.so zkvm-brainfuck_amd/variants/libbfz_r4.so zkvm-brainfuck_amd/variants/libbfz_r6.so > gpurun_out/ab1.txt 2>&1
echo "exit $?"
