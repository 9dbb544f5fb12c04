# quick check after a kernel change: the march / training GPU tests touched, the headline frame
# and the training step lines (each step time-limited; stop at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread ${TESTS:-tests/test_gpu_ring32.py tests/test_gpu_ring_normals.py tests/test_gpu_ring_occlusion.py tests/test_gpu_train.py} > gpurun_out/r05/check_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -2 gpurun_out/r05/check_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra-legs > gpurun_out/r05/check_head.json 2> gpurun_out/r05/check_head.err
rc=$?; echo "HEAD EXIT $rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('gpurun_out/r05/check_head.json').read().strip().splitlines()[-1]); r=d['roofline']; print('head', d['value'], round(d['ms_per_step'],1), round(r['frac'],4), round(r['executed_frac'],4), round(r['avg_kernel_ms'],1))"
rm -f gpurun_out/r05/check_train.jsonl
for P in fp32 mixed; do
  timeout -k 10 300 python -u bench.py --scene train --precision $P --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/r05/check_train.jsonl 2> gpurun_out/r05/check_train_$P.err
  rc=$?; echo "TRAIN $P EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for l in open("gpurun_out/r05/check_train.jsonl"):
    d = json.loads(l)
    r = d["roofline"]
    print(d["config"]["precision"], round(d["ms_per_step"], 2), d["final_loss"], round(d["kernel_ms_per_step"]["k_intersect"], 2),
          {k: (round(v["ms_per_step"], 2), round(v["frac"], 3)) for k, v in r["kernels"].items()})
PY
