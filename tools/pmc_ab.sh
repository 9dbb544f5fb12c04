# Clock + MFMA-busy PMC pass for the shipped build and each variant (one box session).
#   bash tools/pmc_ab.sh e2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
ARGS="--size 800 --steps 1 --warmup 0 --no-cpu-baseline --no-fp32-check"
for V in base "$@"; do
  if [ "$V" = base ]; then L=""; else L=build_var/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex k_march16 -d gpurun_out/pmcab/$V -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmcab/$V.log 2>&1 || { echo "$V failed"; tail -5 gpurun_out/pmcab/$V.log; exit 1; }
  echo "$V ok"
done
