# round 3: batched backward of the mixture's NeuralBSDF MLPs (nrt_mlp_backward_multi): tests +
# the training step bench and its rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k
NRT_REPORT=gpurun_out/r03k/report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_render.py -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03k/tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/r03k/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 2 > gpurun_out/r03k/train.jsonl 2> gpurun_out/r03k/train.err
rc=$?; echo "TRAIN EXIT $rc"; tail -c 300 gpurun_out/r03k/train.jsonl; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --steps 5 --warmup 1 > gpurun_out/r03k/prof_train.log 2>&1
rc=$?; echo "PROF EXIT $rc"; [ $rc -eq 0 ] || exit $rc
find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/r03k/train_kernel_stats.csv \;
