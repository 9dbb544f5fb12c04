# round 6: timing-only experiment -- the fp32-split march without its guarded variant (spill-free
# registers) vs the shipped one, headline frame and DTU scene
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c18
mkdir -p $O
for V in base noguard; do
  if [ "$V" = base ]; then L=""; else L=varlib/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --precision fp32-split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-legs > $O/head_$V.json 2> $O/head_$V.err || { echo "$V head failed"; tail -3 $O/head_$V.err; exit 1; }
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --scene dtu --precision fp32-split --steps 3 --warmup 1 --no-cpu-baseline > $O/dtu_$V.json 2> $O/dtu_$V.err || { echo "$V dtu failed"; tail -3 $O/dtu_$V.err; exit 2; }
  python -c "
import json
for f in ('head','dtu'):
    d=json.loads(open('$O/'+f+'_$V.json').read().strip().split(chr(10))[-1]); r=d['roofline']
    print('$V', f, round(d['ms_per_step'],1), r.get('kernel'), r.get('avg_kernel_ms'), round(r['frac'],3))"
done
echo done
