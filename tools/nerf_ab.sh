# NeRFLE schedule A/B (tools/exp_variants.py builds), then PMC passes of k_nerfle16 (shipped build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "nerfle or plain_nerf" -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/nerf_tests.log 2>&1 || { tail -20 gpurun_out/nerf_tests.log; exit 1; }
tail -1 gpurun_out/nerf_tests.log
for V in "$@"; do
  NRT_LIB=build_var/libnrt_hip_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "nerfle" -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/nerf_tests_$V.log 2>&1 || { echo "$V parity failed"; tail -20 gpurun_out/nerf_tests_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/nerf_tests_$V.log)"
done
BENCH_EXTRA="--scene nerfle" bash tools/exp_run.sh "$@" || exit 1
rm -rf gpurun_out/pmc_nerf
mkdir -p gpurun_out/pmc_nerf
A="--scene nerfle --size 800 --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for SET in "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-include-regex k_nerfle16 -d gpurun_out/pmc_nerf/p$i -o run --output-format csv -- python3 bench.py $A > gpurun_out/pmc_nerf/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_nerf/p$i.log; exit 1; }
  echo "nerf pmc pass $i ok"
done
