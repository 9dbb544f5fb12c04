# round 6, call 8: ring32 with whole-layer chunks for 128-wide MLPs -- parity subsets + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c8
mkdir -p $O
NRT_REPORT=$O/parity.jsonl timeout -k 10 900 python -u -m pytest tests/test_gpu_ring32.py tests/test_gpu_ring_normals.py tests/test_gpu_ring_occlusion.py tests/test_gpu_callable_sdf.py tests/test_gpu_train_render.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread -m gpu > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit 11
timeout -k 10 200 python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/train32.json 2> $O/train32.err || exit 12
python -c "import json; l=json.load(open('$O/train32.json')); print(round(l['ms_per_step'],2), l['roofline']['kernel'], round(l['roofline']['frac'],3), {k: round(v,2) for k,v in l['kernel_ms_per_step'].items()})"
timeout -k 10 200 python -u bench.py --scene colocate --steps 2 --warmup 1 > $O/colocate32.json 2> $O/colocate32.err || exit 13
python -c "import json; l=json.load(open('$O/colocate32.json')); print(round(l['ms_per_step'],2), round(l['roofline']['frac'],3), l['roofline'].get('executed_frac'))"
bash tools/r06_pmc_scenes.sh colocate fp16 k_march16 800 k_march16 && bash tools/r06_pmc_scenes.sh dtu fp16 k_march16 800 k_march16 && bash tools/r06_pmc_scenes.sh colocate fp32 k_march32 800 k_march32
echo done
