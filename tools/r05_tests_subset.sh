# GPU tests touched this round (each file in one pytest process, time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/parity_report.jsonl
NRT_REPORT=gpurun_out/r05/parity_report.jsonl timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_callable_sdf.py tests/test_gpu_sphere_smoothmin.py tests/test_gpu_ring_occlusion.py tests/test_gpu_parity.py tests/test_gpu_configs.py "$@" > gpurun_out/r05/tests_subset.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -5 gpurun_out/r05/tests_subset.log; exit $rc
