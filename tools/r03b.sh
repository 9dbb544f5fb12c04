# round 3: full GPU suite + smoke + training bench (fp32, fp32-split) with its rocprof summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/run_gpu_round.sh tests || exit 1
for P in fp32 fp32-split; do
  timeout -k 10 300 python -u bench.py --scene train --precision $P --steps 10 --warmup 2 >> gpurun_out/r03b_train.jsonl 2> gpurun_out/r03b_train.err
  rc=$?; echo "TRAIN $P EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03b_prof_train.log 2>&1
rc=$?; echo "PROF TRAIN EXIT $rc"; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r03b_prof_train && find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/r03b_prof_train/ \;
