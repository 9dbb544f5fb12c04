# round 6, call 2: NeRF+LE on the fused kernel -- the nerfle tests, the --envmap bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c2
mkdir -p $O
NRT_REPORT=$O/parity.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train_render.py -k "nerfle or envmap" -x -v -p no:cacheprovider --timeout 180 --timeout-method thread -m gpu > $O/tests.log 2>&1 || exit 12
timeout -k 10 200 python -u bench.py --scene nerfle --envmap --steps 3 --warmup 1 > $O/nerfle_env.json 2> $O/nerfle_env.err || exit 13
echo done
