# Time the variants built by tools/exp_variants.py (one box session), the shipped build first.
#   bash tools/exp_run.sh e1 d3 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-fp32-check --no-extra-legs $BENCH_EXTRA"
for V in base "$@"; do
  if [ "$V" = base ]; then L=""; else L=build_var/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python bench.py $ARGS > gpurun_out/exp_$V.log 2>&1 || { echo "$V failed"; tail -3 gpurun_out/exp_$V.log; exit 1; }
  echo "$V $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp_$V.log) $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/exp_$V.log)"
done
