# Time the NRT_EXP variants built by tools/exp_variants.py (one box session).
set -o pipefail
cd $GRAFT_REPO_ROOT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-fp32-check"
for V in 0 "$@"; do
  if [ "$V" = 0 ]; then L=""; else L=build_var/libnrt_hip_e$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python bench.py $ARGS > gpurun_out/exp_e$V.log 2>&1 || { echo "e$V failed"; tail -3 gpurun_out/exp_e$V.log; exit 1; }
  echo "e$V $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp_e$V.log) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/exp_e$V.log)"
done
