# Same-box A/B of kernel preloading at bfz_init (gpu.h PreloadKernels, BFZ_PRELOAD): the cold
# first proof of a fresh process (scripts/cold_first_proof.py, interleaved fresh processes) and
# the host trace of that first proof in either mode.
#   bash scripts/gpu_preload_ab.sh
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/ab_preload.txt
: > $out
for s in 0 1; do
  BFZ_PRELOAD=$s BFZ_HOST_TRACE=1 timeout -k 10 180 python3 scripts/cold_first_proof.py --warm 1 > gpurun_out/preload_trace_$s.txt 2>&1 || exit 1
  echo "BFZ_PRELOAD=$s host trace: $(grep -E '^preload:' gpurun_out/preload_trace_$s.txt)" >> $out
done
for rep in 1 2 3 4; do for s in 0 1; do
  r=$(BFZ_PRELOAD=$s timeout -k 10 180 python3 scripts/cold_first_proof.py) || exit 1
  echo "BFZ_PRELOAD=$s cold: $r" | tee -a $out
done; done
