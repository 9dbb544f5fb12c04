# PMC passes on one kernel of a small bench frame.  Each pass is its own rocprofv3 run, killed
# after 60 s (an over-subscribed counter block hangs rocprofv3).
#   bash tools/pmc.sh <kernel-regex> "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
KRX=$1; shift
ARGS="${BENCH_ARGS:---size ${SIZE:-400} --steps 1 --warmup 0 --no-cpu-baseline --no-fp32-check --no-extra-legs}"
i=0
for SET in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-include-regex "$KRX" -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok: $SET"
done
