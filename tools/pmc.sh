# PMC passes on the bench kernel (small frame).  Each pass is its own rocprofv3 run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
ARGS="--size 400 --steps 1 --warmup 0 --no-cpu-baseline --no-fp32-check"
i=0
for SET in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex k_march16 -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok: $SET"
done
