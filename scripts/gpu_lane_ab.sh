# Signed-lazy lane-mode Poseidon2 (BFZ_P2_LANE_SIGNED) vs the canonical lane form: Poseidon2 and
# proof parity with the new default, then same-box bench pairs of the two builds.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_sharded.py -m gpu -x -q --timeout 600 --timeout-method thread -k "poseidon2 or commit_root or proof_bytes_match or split_commit or sharded_proof or device_transcript or fri" > gpurun_out/pytest_lane.log 2>&1 || { tail -30 gpurun_out/pytest_lane.log; exit 1; }
tail -2 gpurun_out/pytest_lane.log
V=zkvm-brainfuck_amd/variants
AB_REPS=3 timeout -k 10 900 bash scripts/ab_bench.sh $V/libbfz_base.so $V/libbfz_lanes.so > gpurun_out/ab_lane.txt 2>&1
rc=$?
cat gpurun_out/ab_lane.txt
exit $rc
