# round 6: k_march32 line staging (option march_stage) -- ring tests, timing A/B, HBM traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c17
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring32.py tests/test_gpu_mixed.py -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for V in 1 0; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra-legs --nrt-option march_stage=$V > $O/head_stage$V.json 2> $O/head_stage$V.err || { echo "bench $V failed"; tail -3 $O/head_stage$V.err; exit 3; }
  python -c "import json; d=json.load(open('$O/head_stage$V.json')); r=d['roofline']; print('stage $V', round(d['ms_per_step'],1), round(r['avg_kernel_ms'],1), round(r['frac'],3), round(r['executed_frac'],3))"
done
P=$O/pmc
mkdir -p $P
A="--size 800 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_march32" -d $P/$c -o run --output-format csv -- python3 bench.py $A > $P/$c.log 2>&1 || { echo "pmc $c failed"; tail -3 $P/$c.log; exit 4; }
done
python3 tools/pmc_traffic.py $P/FETCH_SIZE $P/WRITE_SIZE 800 fp32 k_march32 > $P/traffic.json || exit 5
cp profiles/pmc_k_march32.json $P/
rm -rf $P/FETCH_SIZE $P/WRITE_SIZE
cat $P/traffic.json
echo done
