# round 6: training-march launch shape A/B -- 12-wave blocks (3 per SIMD) with the line staging
# compiled out (6 spilled VGPRs instead of 19), 8-wave without staging, shipped
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c19
mkdir -p $O
for V in base w12ns w8ns base; do
  if [ "$V" = base ]; then L=""; else L=varlib/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_$V.json 2> $O/train_$V.err || { echo "$V failed"; tail -3 $O/train_$V.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/train_$V.json')); k=d['roofline']['kernels']['k_march32']
print('$V', round(d['ms_per_step'],2), 'march', round(k['ms_per_step'],2), round(k['frac'],3))"
done
echo done
