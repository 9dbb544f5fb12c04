# round 6 (session 2): stall breakdown + instruction mix of the headline k_march32 and the
# two-tile k_nerfle16 (one PMC pass each per counter set; SQ/GRBM counters only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c15
mkdir -p $O
STALL="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
MIX="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for K in head nerfle; do
  if [ $K = head ]; then A="--steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs"; R="k_march32"; else A="--scene nerfle --precision fp16 --steps 1 --warmup 0 --no-cpu-baseline"; R="k_nerfle16"; fi
  timeout -s KILL 150 rocprofv3 --pmc $STALL --kernel-include-regex "$R" -d $O/${K}_stall -o run --output-format csv -- python3 bench.py $A > $O/${K}_stall.log 2>&1 || { echo "stall $K failed"; tail -3 $O/${K}_stall.log; exit 11; }
  python3 tools/pmc_stall_summary.py $O/${K}_stall > $O/${K}_stall.txt || exit 12
  timeout -s KILL 150 rocprofv3 --pmc $MIX --kernel-include-regex "$R" -d $O/${K}_mix -o run --output-format csv -- python3 bench.py $A > $O/${K}_mix.log 2>&1 || { echo "mix $K failed"; tail -3 $O/${K}_mix.log; exit 13; }
  python3 - $O/${K}_mix > $O/${K}_mix.txt <<'PY' || exit 14
import csv, glob, collections, sys
rows = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[int(r["Dispatch_Id"])]["name"] = r["Kernel_Name"][:60]
for d, c in sorted(rows.items()):
    m = max(c.get("SQ_INSTS_MFMA", 1), 1)
    print(d, c["name"], "mfma %.3e valu/mfma %.2f salu/mfma %.2f lds/mfma %.2f smem/mfma %.2f vmem/mfma %.3f" % (
        m, c["SQ_INSTS_VALU"] / m, c["SQ_INSTS_SALU"] / m, c["SQ_INSTS_LDS"] / m, c["SQ_INSTS_SMEM"] / m, c["SQ_INSTS_VMEM"] / m))
PY
  rm -rf $O/${K}_stall $O/${K}_mix
  cat $O/${K}_stall.txt $O/${K}_mix.txt
done
echo done
