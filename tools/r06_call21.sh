# round 6: headline k_march32 launch-queue A/B -- 8-job queue chunks, 8 / 32 segmented tail rays per
# wave, against the shipped 16 / 16 (base twice, first and last)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c21
mkdir -p $O
for V in base qc8 tail8 tail32 base; do
  if [ "$V" = base ]; then L=""; else L=varlib/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra-legs > $O/head_$V.json 2> $O/head_$V.err || { echo "$V failed"; tail -3 $O/head_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$O/head_$V.json')); r=d['roofline']; print('$V', round(d['ms_per_step'],1), round(r['avg_kernel_ms'],1), round(r['frac'],3), round(r['executed_frac'],3))"
done
echo done
