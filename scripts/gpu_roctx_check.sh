export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "coset_lde or proof_bytes_match or commit_root or mfma" > gpurun_out/pytest_ws_default.log 2>&1 && \
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d /tmp/rtx -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --sustain-s 0 --solo-world 0 > gpurun_out/rtx_bench.json 2> gpurun_out/rtx_bench.err && \
find /tmp/rtx -name "*marker*" -o -name "*kernel_stats*" | tee gpurun_out/rtx_files.txt && \
cp $(find /tmp/rtx -name "*marker_api_trace.csv" | head -1) gpurun_out/rtx_marker_api_trace.csv && \
cp $(find /tmp/rtx -name "*kernel_stats.csv" | head -1) gpurun_out/rtx_kernel_stats.csv
rc=$?
tail -3 gpurun_out/pytest_ws_default.log
echo rc=$rc
exit $rc
