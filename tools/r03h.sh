# round 3: SDF callables (warp / displacement / lambda) between the HIP march steps, vs the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
NRT_REPORT=gpurun_out/r03h/report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_callable_sdf.py -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03h/tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -15 gpurun_out/r03h/tests.log; [ $rc -eq 0 ] || exit $rc
