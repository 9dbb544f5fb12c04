# round 3: training handles + host-sync removal; training bench, sync sites and rocprof of the step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NRT_REPORT=gpurun_out/r03c_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_train_handles.py tests/test_gpu_train_render.py tests/test_gpu_train.py tests/test_gpu_dropin.py -v -x -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03c_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/r03c_tests.log; [ $rc -eq 0 ] || exit $rc
for P in fp32 fp32-split; do
  timeout -k 10 300 python -u bench.py --scene train --precision $P --steps 10 --warmup 2 >> gpurun_out/r03c_train.jsonl 2> gpurun_out/r03c_train.err
  rc=$?; echo "TRAIN $P EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --scene train --steps 2 --warmup 2 --torch-profile gpurun_out/r03c_train_ops.txt > /dev/null 2>> gpurun_out/r03c_train.err
rc=$?; echo "TRAIN PROF EXIT $rc"; [ $rc -eq 0 ] || exit $rc
