# Same-box A/B of a runtime switch with parity first (run on the GPU box from the repo root):
#   NAME=multi PYTEST_K="proof_bytes_match or fibo255" bash scripts/gpu_ab_switch.sh "BFZ_X=0" "BFZ_X=1"
# 1. the GPU parity tests selected by PYTEST_K under the LAST arm (the new default);
# 2. AB_REPS rounds over the arms of bench.py (no cold child, no extras), one summary line each
#    (headline, per-family kernel ms) in gpurun_out/ab_$NAME.txt.  Stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=${NAME:?NAME}
O=gpurun_out/ab_$N.txt
: > $O
last="${@: -1}"
if [ -n "$PYTEST_K" ]; then
  env $last timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_ab_$N.log 2>&1 || { tail -30 gpurun_out/pytest_ab_$N.log; exit 1; }
  tail -2 gpurun_out/pytest_ab_$N.log >> $O
fi
i=0
for rep in $(seq 1 ${AB_REPS:-3}); do
  for arm in "$@"; do
    i=$((i+1))
    env $arm timeout -k 10 300 python bench.py ${AB_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-cold --sustain-s 0 --solo-world 0} > gpurun_out/ab_${N}_$i.json 2>gpurun_out/ab_${N}_$i.err || { tail -20 gpurun_out/ab_${N}_$i.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/ab_${N}_$i.json').read().strip().splitlines()[-1]);s=d['stages_ms']
print('$arm', d['value'], 'ntt', s['ntt_kernel_ms'], 'p2', s['p2_kernel_ms'], 'open', s['open_kernel_ms'], 'reduce', s['reduce_kernel_ms'], 'perm_rows', s.get('perm_rows_ms'), 'stages', [round(s[k],3) for k in ('main_commit_ms','perm_ms','quotient_ms','open_ms','fri_ms')])" | tee -a $O
  done
done
cat $O
