# Parity subset with a libbfz variant in place, then same-box bench pairs against the base build
# (run on the GPU box from the repo root): VARIANT=<name> (zkvm-brainfuck_amd/variants/libbfz_<name>.so),
# PYTEST_K selects the parity tests.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=zkvm-brainfuck_amd/variants
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
cp $V/libbfz_$VARIANT.so zkvm-brainfuck_amd/libbfz.so
BFZ_AB_VARIANT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread -k "${PYTEST_K:-proof_bytes_match or split_commit or open}" > gpurun_out/pytest_$VARIANT.log 2>&1
rc=$?
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
tail -2 gpurun_out/pytest_$VARIANT.log
[ $rc = 0 ] || { tail -30 gpurun_out/pytest_$VARIANT.log; exit 1; }
AB_REPS=${AB_REPS:-3} timeout -k 10 900 bash scripts/ab_bench.sh $V/libbfz_base.so $V/libbfz_$VARIANT.so > gpurun_out/ab_$VARIANT.txt 2>&1
rc=$?
cat gpurun_out/ab_$VARIANT.txt
exit $rc
