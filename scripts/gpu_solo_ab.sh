# Same-box A/B of a rank's share of an N-GPU sharded proof (bfz_record_prove_shard_solo, wall
# clock, uninstrumented) between library builds in zkvm-brainfuck_amd/variants/libbfz_<v>.so:
#   VARIANTS="base cur" bash scripts/gpu_solo_ab.sh
export TMPDIR=/tmp BFZ_AB_VARIANT=1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
: > gpurun_out/solo_ab.txt
for rep in 1 2; do for v in ${VARIANTS:-base cur}; do
  cp zkvm-brainfuck_amd/variants/libbfz_$v.so zkvm-brainfuck_amd/libbfz.so
  for w in ${WORLDS:-4 8}; do
    r=$(timeout -k 10 120 python3 scripts/solo_trace.py $w 0 4 untimed 2>/dev/null | python3 -c "import sys,ast; print(min(ast.literal_eval(l)['wall_ms'] for l in sys.stdin))")
    echo "$v N=$w rank0 $r ms" | tee -a gpurun_out/solo_ab.txt
  done
done; done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
