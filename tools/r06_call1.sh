# round 6, call 1: smoke, the sharding tests, the scene benches under torchrun at N = 1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c1
mkdir -p $O
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -x -v -p no:cacheprovider --timeout 180 --timeout-method thread -m gpu > $O/rccl.log 2>&1 || exit 12
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --scene nerfle --steps 3 --warmup 1 > $O/nerfle_tr.json 2> $O/nerfle_tr.err || exit 13
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --scene dtu --precision mixed --steps 3 --warmup 1 > $O/dtu_tr.json 2> $O/dtu_tr.err || exit 14
timeout -k 10 200 python -u bench.py --scene dtu --steps 2 --warmup 1 > $O/dtu32.json 2> $O/dtu32.err || exit 15
echo done
