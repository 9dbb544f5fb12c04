# training backward A/B on one box: the training tests, PMC of the backward kernels per option,
# then the train bench (mixed and FP32) with its rocprof summary.  bash tools/cs_run.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cs
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_render.py tests/test_gpu_train_handles.py -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/cs/tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/cs/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_train.sh || exit 1
python tools/pmc_train_summary.py > gpurun_out/cs/pmc_summary.json || exit 1
rm -f gpurun_out/cs/train.jsonl
for OPT in 0 1 2; do
  timeout -k 10 300 python -u bench.py --scene train --precision mixed --steps 10 --warmup 2 --nrt-option bwd_colsplit=$OPT >> gpurun_out/cs/train.jsonl 2>> gpurun_out/cs/train.err
  rc=$?; echo "TRAIN $OPT EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 2 >> gpurun_out/cs/train.jsonl 2>> gpurun_out/cs/train.err
rc=$?; echo "TRAIN FP32 EXIT $rc"; [ $rc -eq 0 ] || exit $rc
