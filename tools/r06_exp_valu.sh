# round 6: timing-only variants of the FP32 ring march (results wrong on purpose; not shipped):
# softplus -> max(x, 0) and/or no sphere blobs -- how much of k_march32's time is VALU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/exp_valu
mkdir -p $O
for V in base spcheap nosph both; do
  if [ "$V" = base ]; then L=""; else L=build_exp/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 200 python -u bench.py --scene train --steps 6 --warmup 2 --no-cpu-baseline > $O/train_$V.json 2> $O/train_$V.err || { echo "$V train failed"; tail -3 $O/train_$V.err; exit 1; }
  NRT_LIB=$L timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra-legs > $O/head_$V.json 2> $O/head_$V.err || { echo "$V head failed"; tail -3 $O/head_$V.err; exit 1; }
  python -c "
import json
t=json.load(open('$O/train_$V.json')); h=json.load(open('$O/head_$V.json'))
print('$V', 'train march', round(t['kernel_ms_per_step']['k_march32'],2), 'head k_march32', round(h['roofline']['avg_kernel_ms'],1))"
done
echo done
