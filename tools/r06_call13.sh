# round 6 (session 2): state of the restored build -- training leg, headline leg, whole GPU suite + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c13
mkdir -p $O
timeout -k 10 200 python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/train.json 2> $O/train.err || exit 11
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra-legs > $O/head.json 2> $O/head.err || exit 12
python -c "
import json
t=json.load(open('$O/train.json')); h=json.load(open('$O/head.json'))
tm=t['roofline']['kernels']['k_march32']
print('train ms', round(t['ms_per_step'],2), 'march', round(tm['ms_per_step'],2), 'ms/Meval %.3f' % (tm['ms_per_step']/(tm['executed_evals_per_ray']*38400)*1e6), 'head k_march32', round(h['roofline']['avg_kernel_ms'],1), 'frac', round(h['roofline']['frac'],3), round(h['roofline']['executed_frac'],3))"
O=$O/tests bash tools/r06_tests.sh
