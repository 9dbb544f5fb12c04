# round 6: k_wgrad_batch tuning A/B on the FP32 training step (group depth U, waves per EU, rows per
# split-K slice)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c20
mkdir -p $O
for V in base u16 u4 wpe2 sl512 sl128; do
  if [ "$V" = base ]; then L=""; else L=varlib/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/train_$V.json 2> $O/train_$V.err || { echo "$V failed"; tail -3 $O/train_$V.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/train_$V.json')); k=d['roofline']['kernels']
print('$V', round(d['ms_per_step'],2), 'wgrad', round(k['k_wgrad']['ms_per_step'],3), round(k['k_wgrad']['frac'],3), 'bwd', round(k['k_mlp_backward32']['ms_per_step'],3))"
done
echo done
