# round 3 final measurement: full GPU suite + smoke, the bench line (CPU baseline included), the
# rocprofv3 summary of the same frame, PMC passes on the headline kernel (k_march32)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/final
bash tools/run_gpu_round.sh tests || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
rc=$?; echo "BENCH EXIT $rc"; tail -c 400 gpurun_out/final/bench.json; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/final/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra-legs > gpurun_out/final/prof.log 2>&1
rc=$?; echo "PROF EXIT $rc"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/final/prof/run_kernel_stats.csv gpurun_out/final/kernel_stats.csv 2>/dev/null || find gpurun_out/final/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/final/kernel_stats.csv \;
rm -f gpurun_out/final/prof/*kernel_trace.csv
[ -n "$NOPMC" ] && exit 0
rm -rf gpurun_out/pmc
SIZE=800 BENCH_ARGS="--size 800 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs" bash tools/pmc.sh k_march32 "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" || exit 1
