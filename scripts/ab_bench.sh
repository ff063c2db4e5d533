# A/B timing of two builds of libbfz on the same box (run from the repo root on the GPU box):
#   bash scripts/ab_bench.sh zkvm-brainfuck_amd/variants/libbfz_a.so zkvm-brainfuck_amd/variants/libbfz_b.so
# Alternates a, b, a, b and prints value / NTT kernel ms / FRI stage ms per run.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cp zkvm-brainfuck_amd/libbfz.so /tmp/libbfz_orig.so
for v in a b a b; do
  if [ $v = a ]; then cp "$1" zkvm-brainfuck_amd/libbfz.so; else cp "$2" zkvm-brainfuck_amd/libbfz.so; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));s=d['stages_ms'];print('$v', d['value'], s['ntt_kernel_ms'], s['fri_ms'], s['open_ms'], s['quotient_ms'])"
done
cp /tmp/libbfz_orig.so zkvm-brainfuck_amd/libbfz.so
