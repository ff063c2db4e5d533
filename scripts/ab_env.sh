# Same-box A/B of runtime switches (run on the GPU box from the repo root):
#   bash scripts/ab_env.sh "BFZ_OVERLAP=0" "BFZ_OVERLAP=1"
# Each argument is an environment assignment list for one arm; AB_REPS rounds over the arms.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for rep in $(seq 1 ${AB_REPS:-3}); do
  for arm in "$@"; do
    i=$((i+1))
    env $arm timeout -k 10 300 python bench.py ${AB_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-extra --sustain-s 4} > gpurun_out/abenv_$i.json 2>gpurun_out/abenv_$i.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abenv_$i.json'));s=d['stages_ms'];print('$arm', d['value'], 'sustained', d.get('sustained',{}).get('ms_per_proof'), 'ntt', s['ntt_kernel_ms'], 'p2', s['p2_kernel_ms'], 'total', s['total_ms'])"
  done
done
