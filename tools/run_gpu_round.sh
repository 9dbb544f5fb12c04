# GPU round script: tests, smoke, bench, rocprof (each step time-limited; stop at first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = tests ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
  rc=$?; echo "BENCH EXIT $rc"; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-check > gpurun_out/prof.log 2>&1
  rc=$?; echo "PROF EXIT $rc"; tail -2 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
  find gpurun_out/prof -name "*stats*" | head
fi
