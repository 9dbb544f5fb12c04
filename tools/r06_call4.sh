# round 6, call 4: the FP32 training step -- line with the march roofline, rocprof summary, sync sites
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/c4
mkdir -p $O
timeout -k 10 300 python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline --torch-profile $O/train_sync.txt > $O/train32.json 2> $O/train32.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o train32 -- python -u bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/train32_prof.json 2> $O/train32_prof.err || exit 12
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/train32_kernel_stats.csv \;
rm -rf $O/prof
echo done
