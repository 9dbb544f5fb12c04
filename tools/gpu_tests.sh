# Run a subset of the GPU tests on the box: bash tools/gpu_tests.sh <pytest selectors...>
# (one pytest process, per-test thread timeout, log under gpurun_out/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LOG=${LOG:-gpurun_out/gpu_subset.log}
NRT_REPORT=${NRT_REPORT:-gpurun_out/parity_report.jsonl} timeout -k 10 ${TLIMIT:-900} python -u -m pytest "$@" -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > $LOG 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "passed|failed|error" $LOG | tail -3; exit $rc
