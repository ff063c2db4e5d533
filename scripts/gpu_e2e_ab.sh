export TMPDIR=/tmp BFZ_AB_VARIANT=1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
for rep in 1 2; do for v in r05 cur; do
  cp zkvm-brainfuck_amd/variants/libbfz_$v.so zkvm-brainfuck_amd/libbfz.so
  echo "$v $(timeout -k 10 200 python scripts/e2e_probe.py 2>/dev/null)" | tee -a gpurun_out/e2e_ab.txt || break
done; done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
