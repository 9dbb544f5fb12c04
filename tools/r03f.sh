# round 3: Path under autograd (gradients vs the float64 oracle) + the Path / training suites
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NRT_REPORT=gpurun_out/r03f_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_train_render.py tests/test_gpu_parity.py -k "path or envmap or gradients" -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -4 gpurun_out/r03f_tests.log; [ $rc -eq 0 ] || exit $rc
