# Run one gpurun call; while the pool has no free slot / box (gpurun exit 3: nothing ran, nothing
# charged) wait and ask again, up to 20 times.  Any other outcome -- success or a failure of the
# command itself -- ends it (no retry of a GPU step that ran).
#   bash tools/gpurun_wait.sh <out-file> <timeout-s> '<command>'
OUT=$1; T=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $OUT 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "status=transient" $OUT || exit $rc
  sleep 150
done
exit 3
