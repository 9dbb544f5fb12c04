# GPU round script: tests, smoke, bench, rocprof, PMC traffic (each step time-limited; stop at
# the first failure).  bash tools/run_gpu_round.sh [all|tests|bench|prof|pmc|scenes|train|trainpmc]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEP=${1:-all}
mkdir -p gpurun_out
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  rm -f gpurun_out/parity_report.jsonl
  NRT_REPORT=gpurun_out/parity_report.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "SMOKE EXIT $rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
  rc=$?; echo "BENCH EXIT $rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32-check --no-extra-legs > gpurun_out/prof.log 2>&1
  rc=$?; echo "PROF EXIT $rc"; tail -1 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = pmc ]; then
  rm -rf gpurun_out/pmc
  SIZE=800 BENCH_ARGS="--size 800 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs" bash tools/pmc.sh k_march32 "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" || exit 1
fi
if [ "$STEP" = all ] || [ "$STEP" = scenes ]; then
  rm -f gpurun_out/scenes.jsonl
  for SC in colocate dtu; do
    for PREC in fp32 fp32-split mixed fp16; do
      timeout -k 10 300 python -u bench.py --scene $SC --precision $PREC --steps 3 --warmup 1 >> gpurun_out/scenes.jsonl 2> gpurun_out/scene_$SC.err
      rc=$?; echo "SCENE $SC $PREC EXIT $rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
  timeout -k 10 300 python -u bench.py --scene nerfle --steps 3 --warmup 1 >> gpurun_out/scenes.jsonl 2> gpurun_out/scene_nerfle.err
  rc=$?; echo "SCENE nerfle EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nerfle -o run --output-format csv -- python3 bench.py --scene nerfle --steps 2 --warmup 1 > gpurun_out/prof_nerfle.log 2>&1
  rc=$?; echo "PROF NERFLE EXIT $rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = train ]; then
  timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 2 > gpurun_out/train.jsonl 2> gpurun_out/train.err
  rc=$?; echo "TRAIN EXIT $rc"; tail -1 gpurun_out/train.jsonl; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --scene train --precision mixed --steps 10 --warmup 2 >> gpurun_out/train.jsonl 2>> gpurun_out/train.err
  rc=$?; echo "TRAIN MIXED EXIT $rc"; tail -1 gpurun_out/train.jsonl; [ $rc -eq 0 ] || exit $rc
  # the kernel trace of a training step is large (every torch op): keep only the stats
  rm -rf /tmp/prof_train
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --precision mixed --steps 5 --warmup 1 > gpurun_out/prof_train.log 2>&1
  rc=$?; echo "PROF TRAIN EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  mkdir -p gpurun_out/prof_train && find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_train/ \;
fi
if [ "$STEP" = trainpmc ]; then
  # the training backward's PMC (column-split vs per-wave kernels) and the option A/B of the step
  bash tools/pmc_train.sh || exit 1
  python tools/pmc_train_summary.py > gpurun_out/pmc_train/summary.json || exit 1
  rm -f gpurun_out/train_ab.jsonl
  for OPT in 0 1 2; do
    timeout -k 10 300 python -u bench.py --scene train --precision mixed --steps 10 --warmup 2 --nrt-option bwd_colsplit=$OPT >> gpurun_out/train_ab.jsonl 2>> gpurun_out/train_ab.err
    rc=$?; echo "TRAIN bwd_colsplit=$OPT EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
