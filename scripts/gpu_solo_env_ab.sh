# Same-box A/B of a rank's share of an N-GPU sharded proof (bfz_record_prove_shard_solo, wall
# clock, uninstrumented) between environment switches of one library build:
#   SETTINGS="BFZ_FUSED_RESIDUE=0 BFZ_FUSED_RESIDUE=1" bash scripts/gpu_solo_env_ab.sh
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/solo_env_ab.txt
for rep in 1 2; do for s in ${SETTINGS:-BFZ_FUSED_RESIDUE=0 BFZ_FUSED_RESIDUE=1}; do
  for w in ${WORLDS:-2 4 8}; do
    r=$(env $s timeout -k 10 120 python3 scripts/solo_trace.py $w 0 4 untimed 2>/dev/null | python3 -c "import sys,ast; print(min(ast.literal_eval(l)['wall_ms'] for l in sys.stdin))") || exit 1
    echo "$s N=$w rank0 $r ms" | tee -a gpurun_out/solo_env_ab.txt
  done
done; done
