# round 3: fused refresh + ring forwards of the training MLPs: tests + training bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NRT_REPORT=gpurun_out/r03e_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_train_handles.py tests/test_gpu_train.py tests/test_gpu_train_render.py tests/test_gpu_split.py tests/test_gpu_ring32.py tests/test_gpu_dropin.py -v -x -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/r03e_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r03e_train.jsonl
for P in fp32 fp32-split; do
  timeout -k 10 300 python -u bench.py --scene train --precision $P --steps 10 --warmup 2 >> gpurun_out/r03e_train.jsonl 2> gpurun_out/r03e_train.err
  rc=$?; echo "TRAIN $P EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --steps 5 --warmup 1 > gpurun_out/r03e_prof_train.log 2>&1
rc=$?; echo "PROF TRAIN EXIT $rc"; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r03e_prof_train && find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/r03e_prof_train/ \;
