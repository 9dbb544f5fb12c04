# round 6 final, part A: GPU suite + smoke, k_march32 PMC (traffic, busy, stall), the default
# bench line (reads the fresh traffic file), its rocprofv3 --kernel-trace --stats summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${FINAL_DIR:-gpurun_out/r06/final}
mkdir -p $O
O=$O/tests bash tools/r06_tests.sh || exit 1
P=$O/pmc
mkdir -p $P
A="--size 800 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_march32" -d $P/$c -o run --output-format csv -- python3 bench.py $A > $P/$c.log 2>&1 || { echo "pmc $c failed"; tail -3 $P/$c.log; exit 2; }
done
python3 tools/pmc_traffic.py $P/FETCH_SIZE $P/WRITE_SIZE 800 fp32 k_march32 > $P/traffic.json || exit 3
cp profiles/pmc_k_march32.json $P/
STALL="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 150 rocprofv3 --pmc $STALL --kernel-include-regex "k_march32" -d $P/stall -o run --output-format csv -- python3 bench.py $A > $P/stall.log 2>&1 || { echo "pmc stall failed"; exit 4; }
python3 tools/pmc_stall_summary.py $P/stall > $P/stall.txt || exit 5
rm -rf $P/FETCH_SIZE $P/WRITE_SIZE $P/stall
cat $P/traffic.json $P/stall.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 6; }
tail -c 600 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra-legs > $O/prof.log 2>&1 || { echo "prof failed"; exit 7; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -delete
echo done
