# Round-3 probe: new tests, a kernel-stats profile of the fp32-split and fp32 frames, and PMC
# passes on k_march3.  Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  NRT_REPORT=gpurun_out/r03_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_split.py "tests/test_gpu_parity.py::test_pathtrace_fused_tiles_match_oracle" tests/test_gpu_dropin.py -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03_tests.log 2>&1
  rc=$?; echo "TESTS EXIT $rc"; tail -4 gpurun_out/r03_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  for PREC in fp32-split fp32; do
    rm -rf /tmp/prof_$PREC
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$PREC -o run --output-format csv -- python3 bench.py --precision $PREC --steps 2 --warmup 1 --no-cpu-baseline --no-extra-legs > gpurun_out/prof_$PREC.log 2>&1
    rc=$?; echo "PROF $PREC EXIT $rc"; [ $rc -eq 0 ] || exit $rc
    mkdir -p gpurun_out/prof_$PREC && find /tmp/prof_$PREC -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$PREC/ \;
  done
fi
if [ "$STEP" = all ] || [ "$STEP" = pmc ]; then
  rm -rf gpurun_out/pmc
  BENCH_ARGS="--precision fp32-split --size 400 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs" bash tools/pmc.sh k_march3 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" || exit 1
fi
