# A/B of a ring32 build variant on the FP32 training step and the colocate FP32 frame
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/ab_r32.jsonl
for V in base "$@"; do
  if [ "$V" = base ]; then L=""; else L=build_var/libnrt_hip_$V.so; fi
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/ab_train_$V.json 2>gpurun_out/r05/ab_err_$V.log || { echo "$V train failed"; tail -3 gpurun_out/r05/ab_err_$V.log; exit 1; }
  NRT_LIB=$L timeout -k 10 300 python -u bench.py --scene colocate --precision fp32 --steps 3 --warmup 1 > gpurun_out/r05/ab_coloc_$V.json 2>>gpurun_out/r05/ab_err_$V.log || { echo "$V colocate failed"; exit 1; }
  python - "$V" <<'PY'
import json, sys
v = sys.argv[1]
t = json.loads(open(f"gpurun_out/r05/ab_train_{v}.json").read().strip().splitlines()[-1])
c = json.loads(open(f"gpurun_out/r05/ab_coloc_{v}.json").read().strip().splitlines()[-1])
print(v, "train ms", round(t["ms_per_step"], 2), "march ms", round(t["kernel_ms_per_step"]["k_intersect"], 2),
      "loss", t["final_loss"], "| colocate ms", round(c["ms_per_step"], 2), "kernel", round(c["roofline"]["kernel_ms_per_step"], 2))
PY
done
