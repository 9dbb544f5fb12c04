# round 6, call 5: rocprof kernel stats of the FP32 training step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c5
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o train32 -- python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/train32_prof.json 2> $O/train32_prof.err || exit 12
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/train32_kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/train32_kernel_trace.csv \;
rm -rf $O/prof
gzip $O/train32_kernel_trace.csv
ls -la $O
echo done
