# Multi-rank rehearsal on a one-GPU box: both bench modes with NPROC (default 2) ranks pinned
# to GPU 0 (timings are not scaling numbers -- the ranks share one GPU).  MODES overrides the
# mode list.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NP=${NPROC:-2}
for mode in ${MODES:-replicas sharded}; do
  BFZ_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $NP --steps 3 --warmup 1 \
    --no-cpu-baseline --mode $mode > gpurun_out/rehearsal_${mode}_$NP.json 2> gpurun_out/rehearsal_${mode}_$NP.err || exit $?
done
echo "exit 0"
