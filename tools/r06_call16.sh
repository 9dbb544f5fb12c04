# round 6: kernel time per mixed training step (rocprof stats) vs the step's wall time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c16
mkdir -p $O
rm -rf /tmp/prof_tm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_tm -o run --output-format csv -- python3 bench.py --scene train --precision mixed --steps 10 --warmup 3 --no-cpu-baseline > $O/train_mixed.json 2> $O/train_mixed.err || exit 1
find /tmp/prof_tm -name "*kernel_stats.csv" -exec cp {} $O/train_mixed_kernel_stats.csv \;
python3 - <<'PY'
import csv, json
rows = list(csv.DictReader(open("gpurun_out/r06/c16/train_mixed_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = max(int(r["Calls"]) for r in rows if "k_refine3" in r["Name"] or "k_march16" in r["Name"])
d = json.loads(open("gpurun_out/r06/c16/train_mixed.json").read().strip().split("\n")[-1])
print("march launches", n, "kernel ms per launch-step", tot / 1e6 / n, "step ms", d["ms_per_step"])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6 / n, 3))
PY
