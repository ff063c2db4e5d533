# Round-5 batch: misc checks (syncmalloc first-proof stall, opening/lane tests, bench line), the
# NTT counter passes, then an A/B of the openings' rows per thread (bench --no-extra, lib swapped).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r5_misc.sh && bash scripts/gpu_ntt_counters.sh && \
AB_REPS=2 AB_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0" \
  bash scripts/ab_bench.sh zkvm-brainfuck_amd/variants/libbfz_open8.so zkvm-brainfuck_amd/variants/libbfz_open6.so \
  zkvm-brainfuck_amd/variants/libbfz_open4.so > gpurun_out/ab_open_rows_r5.txt 2>&1
rc=$?
cat gpurun_out/ab_open_rows_r5.txt | tail -8
exit $rc
