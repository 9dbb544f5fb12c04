# round 6, call 3: the --scene path line (batched Path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c3
mkdir -p $O
timeout -k 10 300 python -u bench.py --scene path --steps 3 --warmup 1 > $O/path.json 2> $O/path.err || exit 13
echo done
