# Same-box A/B of the FRI shard threshold (BFZ_FRI_SHARD_MIN: rounds with fewer leaves run on every
# rank) on the predicted sharded curve (solo shares + modeled collectives), N = 4 and 8.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/fri_shard_ab.txt
for rep in 1 2; do for s in ${MINS:-262144 1048576 4194304}; do
  BFZ_FRI_SHARD_MIN=$s timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-cold --sustain-s 0 --solo-world ${SOLO:-4,8} > gpurun_out/fri_ab_$s.json 2> gpurun_out/fri_ab_$s.err || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/fri_ab_$s.json')); c=d['shard_solo_curve']
print('min=$s', 'N1', d['value'], 'share', c['ms_per_proof_by_gpus'], 'coll', c['modeled_collective_ms'], 'total', c['ms_per_proof_with_collectives'], 'n_coll', {k: v['collectives'] for k, v in c['collectives_by_gpus'].items()})
" | tee -a gpurun_out/fri_shard_ab.txt
done; done
