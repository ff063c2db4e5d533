# Round-5: NTT counter passes (scripts/gpu_ntt_counters.sh), then an A/B of the openings' rows per
# thread (bench --no-extra, library swapped in; builds: bash scripts/build_variant.sh open<R> WORKTREE -DBFZ_OPEN_R=<R>, before the macro was removed).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ntt_counters.sh && \
AB_REPS=2 AB_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0" \
  bash scripts/ab_bench.sh zkvm-brainfuck_amd/variants/libbfz_open8.so zkvm-brainfuck_amd/variants/libbfz_open6.so \
  zkvm-brainfuck_amd/variants/libbfz_open4.so > gpurun_out/ab_open_rows_r5.txt 2>&1
rc=$?
tail -8 gpurun_out/ab_open_rows_r5.txt
exit $rc
