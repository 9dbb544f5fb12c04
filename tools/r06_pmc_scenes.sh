# round 6: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of each bench --scene line's
# dominant kernel -> profiles/pmc_<scene>_<kernel>.json (bench.py reads them into roofline.traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06/pmc_scenes
mkdir -p $O
run() {  # scene precision kernel-regex size profile-name
  local sc=$1 pr=$2 kr=$3 sz=$4 pn=$5
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$kr" -d $O/${sc}_${pr}_$c -o run --output-format csv -- python3 bench.py --scene $sc --precision $pr --size $sz --steps 1 --warmup 0 --no-cpu-baseline > $O/${sc}_${pr}_$c.log 2>&1 || { echo "pass $sc $pr $c failed"; tail -3 $O/${sc}_${pr}_$c.log; return 1; }
  done
  python3 tools/pmc_traffic.py $O/${sc}_${pr}_FETCH_SIZE $O/${sc}_${pr}_WRITE_SIZE $sz $pr $kr $sc $pn || return 1
  rm -rf $O/${sc}_${pr}_FETCH_SIZE $O/${sc}_${pr}_WRITE_SIZE
}
if [ -n "$1" ]; then
  run "$@" || exit 1
else
run colocate fp16 k_march16 800 k_march16 && \
run colocate mixed k_march16 800 k_march16 && \
run colocate fp32-split k_march3 800 k_march3 && \
run colocate fp32 k_march32 800 k_march32 && \
run dtu fp16 k_march16 800 k_march16 && \
run dtu mixed k_march16 800 k_march16 && \
run dtu fp32-split k_march3 800 k_march3 && \
run dtu fp32 k_march32 800 k_march32 && \
run nerfle fp16 k_nerfle16 1600 k_nerfle && \
run path fp32 k_march32 200 k_march32 || exit 1
fi
cp profiles/pmc_*_k_*.json $O/ 2>/dev/null
echo done
