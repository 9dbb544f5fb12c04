# Round-3 probe 2: full GPU suite, training step (fp32, fp32-split), PMC of k_march3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r03c_report.jsonl
NRT_REPORT=gpurun_out/r03c_report.jsonl timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/r03c_tests.log; [ $rc -eq 0 ] || exit $rc
for P in fp32 fp32-split; do
  timeout -k 10 300 python -u bench.py --scene train --precision $P --steps 10 --warmup 2 >> gpurun_out/train_c.jsonl 2> gpurun_out/train_c.err
  rc=$?; echo "TRAIN $P EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_train_c.log 2>&1
rc=$?; echo "PROF TRAIN EXIT $rc"; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/prof_train_c && find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_train_c/ \;
[ -n "$NOPMC" ] && exit 0
rm -rf gpurun_out/pmc
BENCH_ARGS="--precision fp32-split --size 400 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs" bash tools/pmc.sh k_march3 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" || exit 1
