export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_pcs_sharded.py tests/test_sharded.py -m gpu -x -q --timeout 600 --timeout-method thread -k "commit_root or proof_bytes_match or root_matches or sharded_proof or split_commit or fri" > gpurun_out/pytest_top1.log 2>&1 || { tail -30 gpurun_out/pytest_top1.log; exit 1; }
tail -2 gpurun_out/pytest_top1.log
V=zkvm-brainfuck_amd/variants
AB_REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh $V/libbfz_base.so $V/libbfz_top1.so > gpurun_out/ab_top1.txt 2>&1
rc=$?
cat gpurun_out/ab_top1.txt
exit $rc
