# Same-box A/B of the quotient exchange pipeline (BFZ_QUOT_PIPE) on the predicted sharded curve
# (solo shares + the collective model with measured overlap), after the sharded parity tests.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/quot_pipe_ab.txt
: > $O
timeout -k 10 500 python -u -m pytest tests/test_sharded.py tests/test_pcs_sharded.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sharded or proof_bytes_match or x4_2pow22 or (pcs and not c4 and not c5)" > gpurun_out/pytest_quot_pipe.log 2>&1 || { tail -30 gpurun_out/pytest_quot_pipe.log; exit 1; }
tail -1 gpurun_out/pytest_quot_pipe.log >> $O
for rep in 1 2; do for s in BFZ_QUOT_PIPE=0 BFZ_QUOT_PIPE=1; do
  env $s timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-cold --sustain-s 0 --solo-world 2,4,8 > gpurun_out/qp_$s.json 2> gpurun_out/qp_$s.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/qp_$s.json')); c=d['shard_solo_curve']
print('$s', 'N1', d['value'], 'share', c['ms_per_proof_by_gpus'], 'coll', c['modeled_collective_ms'], 'total', c['ms_per_proof_with_collectives'], 'speedup', c['speedup_with_collectives'], 'overlapped', {k: v['overlapped_ms'] for k, v in c['collectives_by_gpus'].items()})
" | tee -a $O
done; done
