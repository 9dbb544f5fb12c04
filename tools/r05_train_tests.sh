# training-path GPU tests + the training step lines (each step time-limited; stop at a failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 180 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_train_handles.py tests/test_gpu_train_render.py tests/test_gpu_callable_sdf.py "$@" > gpurun_out/r05/train_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/r05/train_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r05/train.jsonl
for P in fp32 mixed; do
  timeout -k 10 300 python -u bench.py --scene train --precision $P --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/r05/train.jsonl 2> gpurun_out/r05/train_$P.err
  rc=$?; echo "TRAIN $P EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json
for l in open("gpurun_out/r05/train.jsonl"):
    d = json.loads(l)
    r = d["roofline"]
    print(d["config"]["precision"], round(d["ms_per_step"], 2), d["final_loss"],
          {k: (round(v["ms_per_step"], 2), round(v["frac"], 3)) for k, v in r["kernels"].items()})
PY
# the FP16 march's persistent grid on a small batch: every CU (option march_blocks) vs the default
for MB in 256; do
  timeout -k 10 300 python -u bench.py --scene train --precision mixed --steps 10 --warmup 2 --no-cpu-baseline --nrt-option march_blocks=$MB > gpurun_out/r05/train_mb$MB.json 2> gpurun_out/r05/train_mb.err
  rc=$?; echo "TRAIN mixed march_blocks=$MB EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('gpurun_out/r05/train_mb$MB.json')); print('march_blocks=$MB', round(d['ms_per_step'],2), d['final_loss'], round(d['kernel_ms_per_step']['k_intersect'],2))"
done
