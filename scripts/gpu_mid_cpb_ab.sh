# k_lde_mid columns-per-block A/B (run on the GPU box from the repo root): coset LDEs of 2^22 x 8
# and 2^21 x 8 with each variant (output hashes must agree), then rocprofv3 FETCH_SIZE of k_lde_mid<22>
# per variant (zkvm-brainfuck_amd/variants/cpb<k>/libbfz.so).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/ab_mid_cpb.txt
: > $O
for rep in 1 2; do for v in ${VARIANTS:-cpb1 cpb2 cpb4}; do
  for L in 22 21; do
    echo "$v $(LD_LIBRARY_PATH=$PWD/zkvm-brainfuck_amd/variants/$v timeout -k 10 60 ./scripts/ubench_ntt lde $L 8 20)" >> $O || exit 1
  done
done; done
for v in ${VARIANTS:-cpb1 cpb2 cpb4}; do
  LD_LIBRARY_PATH=$PWD/zkvm-brainfuck_amd/variants/$v timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_$v -o run -- ./scripts/ubench_ntt lde 22 8 5 > /dev/null 2>&1 || exit 1
  python3 - "$v" >> $O <<'PY'
import csv, glob, sys
f = glob.glob(f"/tmp/pmc_{sys.argv[1]}/**/run_counter_collection.csv", recursive=True)[0]
tot, n = 0.0, 0
for r in csv.DictReader(open(f)):
    if "k_lde_mid" in r["Kernel_Name"]:
        tot += float(r["Counter_Value"]); n += 1
print(sys.argv[1], "k_lde_mid<22> FETCH_SIZE kB per launch", round(tot / max(n, 1), 1), "launches", n)
PY
done
cat $O
