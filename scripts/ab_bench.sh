# Same-box A/B timing of several builds of libbfz (run on the GPU box from the repo root):
#   bash scripts/ab_bench.sh zkvm-brainfuck_amd/variants/libbfz_a.so zkvm-brainfuck_amd/variants/libbfz_b.so ...
# AB_ARGS replaces the bench flags (default: the proof alone, no end-to-end / drop-in extras).
# Two rounds over the builds in order; prints value and the stage times per run.
export TMPDIR=/tmp
export BFZ_AB_VARIANT=1  # the builds come from other source revisions
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
for rep in $(seq 1 ${AB_REPS:-2}); do
  for so in "$@"; do
    v=$(basename $so .so)
    cp "$so" zkvm-brainfuck_amd/libbfz.so
    timeout -k 10 300 python bench.py ${AB_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-extra --sustain-s 0} > gpurun_out/ab_${v}_$rep.json 2>gpurun_out/ab_${v}_$rep.err || { cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${v}_$rep.json'));s=d['stages_ms'];print('$v', d['value'], 'ntt', s['ntt_kernel_ms'], 'open', s['open_ms'], 'fri', s['fri_ms'], 'quot', s['quotient_ms'], 'p2', s['p2_kernel_ms'], 'open_k', s.get('open_kernel_ms'), 'reduce_k', s.get('reduce_kernel_ms'), 'drop_in', d.get('drop_in_path', {}).get('ms'), 'e2e', d.get('end_to_end', {}).get('ms_per_proof'))"
  done
done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
