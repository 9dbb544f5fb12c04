# round 6: the whole -m gpu suite and smoke (one pytest process, per-test thread timeout)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r06/tests}
mkdir -p $O
rm -f $O/parity_report.jsonl
NRT_REPORT=$O/parity_report.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "SMOKE EXIT $rc"; tail -2 $O/smoke.log; exit $rc
