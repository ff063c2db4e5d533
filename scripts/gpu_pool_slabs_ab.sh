# Same-box A/B of the lane pool's slab carving (gpu.h DevicePool, BFZ_POOL_SLABS): the cold
# first proof of a fresh process (scripts/cold_first_proof.py, three fresh processes per
# setting, interleaved), the hipMalloc count of that proof (BFZ_HOST_TRACE), and the warm
# headline (bench.py, no extras).
#   bash scripts/gpu_pool_slabs_ab.sh
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_pool_slabs.txt
: > $out
for s in 0 1; do
  echo "BFZ_POOL_SLABS=$s host trace:" >> $out
  BFZ_POOL_SLABS=$s BFZ_HOST_TRACE=1 timeout -k 10 180 python3 scripts/cold_first_proof.py --warm 1 > gpurun_out/pool_trace_$s.txt 2>&1 || exit 1
  grep -E "pool:" gpurun_out/pool_trace_$s.txt >> $out || true
done
for rep in 1 2 3; do for s in 0 1; do
  r=$(BFZ_POOL_SLABS=$s timeout -k 10 180 python3 scripts/cold_first_proof.py) || exit 1
  echo "BFZ_POOL_SLABS=$s cold: $r" | tee -a $out
done; done
for s in 0 1 0 1; do
  r=$(BFZ_POOL_SLABS=$s timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cold --no-extra --sustain-s 3 --solo-world "" --steps 10 --warmup 3) || exit 1
  echo "BFZ_POOL_SLABS=$s bench: $r" | tee -a $out
done
