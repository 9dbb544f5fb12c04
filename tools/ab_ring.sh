# A/B of the ring kernel block size in one box session
set -o pipefail
cd $GRAFT_REPO_ROOT
for W in 8 4; do
  NRT_RING_WAVES=$W timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-check > gpurun_out/ab_w$W.log 2>&1 || exit 1
  echo "W=$W $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_w$W.log) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_w$W.log) $(grep -o '"frac": [0-9.]*' gpurun_out/ab_w$W.log)"
done
