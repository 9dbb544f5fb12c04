# round 3: FP32 / split ring shading + ring normals (tests, bench, rocprof) + NeRFLE VALU cut
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/r03a_report.jsonl
NRT_REPORT=gpurun_out/r03a_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_shade_ring.py tests/test_gpu_ring_normals.py -v -x -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -5 gpurun_out/r03a_tests.log; [ $rc -eq 0 ] || exit $rc
NRT_REPORT=gpurun_out/r03a_report.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -k "nerfle or ring32 or split or render_matches or metric or dtu or colocate" -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03a_more.log 2>&1
rc=$?; echo "MORE TESTS EXIT $rc"; tail -3 gpurun_out/r03a_more.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r03a_bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --scene nerfle --steps 3 --warmup 1 > gpurun_out/r03a_nerfle.jsonl 2> gpurun_out/r03a_nerfle.err
rc=$?; echo "NERFLE EXIT $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03a_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra-legs --steps 3 --warmup 1 > gpurun_out/r03a_prof.log 2>&1
rc=$?; echo "PROF EXIT $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03a_prof_split -o run --output-format csv -- python3 bench.py --precision fp32-split --no-cpu-baseline --no-extra-legs --steps 3 --warmup 1 > gpurun_out/r03a_prof_split.log 2>&1
rc=$?; echo "PROF SPLIT EXIT $rc"; [ $rc -eq 0 ] || exit $rc
