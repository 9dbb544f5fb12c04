# round 6, call 9: NRT_MIXED flag audit + instruction mix of the training march
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c9
mkdir -p $O
timeout -k 10 400 python -u tools/mixed_audit.py 800 20000,10000,5000 > $O/mixed_audit.jsonl 2> $O/mixed_audit.err || exit 11
SET="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex "k_march32" -d $O/mix -o run --output-format csv -- python3 bench.py --scene train --steps 2 --warmup 1 --no-cpu-baseline > $O/mix.log 2>&1 || exit 12
python3 - <<'PY' > $O/train_march_instmix.txt
import csv, glob, collections
rows = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/r06/c9/mix/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[int(r["Dispatch_Id"])]["name"] = r["Kernel_Name"][:60]
for d, c in sorted(rows.items()):
    m = max(c.get("SQ_INSTS_MFMA", 1), 1)
    print(d, c["name"], "valu/mfma %.2f salu/mfma %.2f lds/mfma %.2f smem/mfma %.2f busy %.3f" % (
        c["SQ_INSTS_VALU"] / m, c["SQ_INSTS_SALU"] / m, c["SQ_INSTS_LDS"] / m, c["SQ_INSTS_SMEM"] / m,
        c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)))
PY
rm -rf $O/mix
cat $O/train_march_instmix.txt
echo done
