# A/B of runtime options (nrt_set_option) on the training step (FP32, mixed) and the 800^2
# frame (FP32, mixed).  Usage: bash tools/r05_ab_opt.sh base "march_queue=1" "a=1,b=2" ...
# LEGS (default "tf tm hf hm"): tf/tm = train fp32/mixed, hf/hm = headline fp32/mixed
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05/ab
LEGS=${LEGS:-"tf tm hf hm"}
for V in "$@"; do
  OPTS=""
  if [ "$V" != base ]; then for kv in ${V//,/ }; do OPTS="$OPTS --nrt-option $kv"; done; fi
  tag=$(echo "$V" | tr '=,' '__')
  for L in $LEGS; do
    case $L in
      tf) A="--scene train --precision fp32 --steps 10 --warmup 2 --no-cpu-baseline";;
      tm) A="--scene train --precision mixed --steps 10 --warmup 2 --no-cpu-baseline";;
      hf) A="--precision fp32 --steps 3 --warmup 1 --no-extra-legs --no-cpu-baseline";;
      hm) A="--precision mixed --steps 3 --warmup 1 --no-extra-legs --no-cpu-baseline";;
    esac
    timeout -k 10 300 python -u bench.py $A $OPTS > gpurun_out/r05/ab/${tag}_$L.json 2> gpurun_out/r05/ab/${tag}_$L.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$V $L failed rc=$rc"; tail -5 gpurun_out/r05/ab/${tag}_$L.err; exit 1; fi
    python - "$V" "$L" gpurun_out/r05/ab/${tag}_$L.json <<'PY'
import json, sys
v, leg, f = sys.argv[1:4]
d = json.loads(open(f).read().strip().splitlines()[-1])
r = d.get("roofline", {})
km = d.get("kernel_ms_per_step", {})
print(f"{v:24s} {leg} ms/step {d['ms_per_step']:9.2f} value {d['value']:.4g}"
      f" march {km.get('k_intersect', r.get('avg_kernel_ms', float('nan'))):.2f}"
      f" frac {r.get('frac', float('nan')):.3f} exec {r.get('executed_frac', float('nan'))}"
      f" loss {d.get('final_loss', '')}", flush=True)
PY
  done
done
