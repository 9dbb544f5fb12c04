# round 6: A/B of training-march launch shapes (FP32 step), one process per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/ab_train
mkdir -p $O
for V in "" "--nrt-option march_blocks=512" "--nrt-option march_blocks=384" "--nrt-option march_queue=1" "--nrt-option march_blocks=512 --nrt-option march_queue=1"; do
  N=$(echo "$V" | tr ' =' '__')
  timeout -k 10 200 python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline $V > $O/t$N.json 2> $O/t$N.err || exit 11
  python -c "import json,sys; l=json.load(open('$O/t$N.json')); print('$V', round(l['ms_per_step'],2), {k: round(v,2) for k,v in l['kernel_ms_per_step'].items()})"
done
echo done
