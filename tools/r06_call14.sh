# round 6 (session 2): k_nerfle16 with two 32-sample tiles per wave (each A read feeds two MFMAs)
# -- nerfle parity tests on the shipped build (TT=2), then the --scene nerfle line per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c14
mkdir -p $O
true
true
for V in base tt1 tt2w4; do
  if [ "$V" = base ]; then L=""; else L=varlib/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --scene nerfle --precision fp16 --steps 3 --warmup 1 --no-cpu-baseline > $O/nerfle_$V.json 2> $O/nerfle_$V.err || { echo "$V failed"; tail -3 $O/nerfle_$V.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/nerfle_$V.json')); r=d['roofline']
print('$V', 'ms', round(d['ms_per_step'],2), 'kernel', r.get('avg_kernel_ms'), 'frac', round(r['frac'],3), 'exec', r.get('executed_frac'))"
done
NRT_LIB= timeout -k 10 300 python -u bench.py --scene nerfle --envmap --precision fp16 --steps 3 --warmup 1 --no-cpu-baseline > $O/nerfle_env.json 2> $O/nerfle_env.err || exit 13
python -c "import json; d=json.load(open('$O/nerfle_env.json')); print('envmap ms', round(d['ms_per_step'],2))"
echo done
