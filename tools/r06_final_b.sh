# round 6 final, part B: every --scene line (colocate / dtu at four precisions, nerfle, nerfle
# --envmap, path) and the training legs, with the rocprof summaries of nerfle and training
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${FINAL_DIR:-gpurun_out/r06/final}
mkdir -p $O
rm -f $O/scenes.jsonl
for SC in colocate dtu; do
  for PREC in fp32 fp32-split mixed fp16; do
    timeout -k 10 300 python -u bench.py --scene $SC --precision $PREC --steps 3 --warmup 1 >> $O/scenes.jsonl 2> $O/scene_${SC}_$PREC.err
    rc=$?; echo "SCENE $SC $PREC EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python -u bench.py --scene nerfle --steps 3 --warmup 1 >> $O/scenes.jsonl 2> $O/scene_nerfle.err || { echo nerfle failed; exit 3; }
timeout -k 10 300 python -u bench.py --scene nerfle --envmap --steps 3 --warmup 1 >> $O/scenes.jsonl 2> $O/scene_nerfle_env.err || { echo envmap failed; exit 4; }
timeout -k 10 300 python -u bench.py --scene path --steps 3 --warmup 1 >> $O/scenes.jsonl 2> $O/scene_path.err || { echo path failed; exit 5; }
echo scenes ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_nerfle -o run --output-format csv -- python3 bench.py --scene nerfle --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_nerfle.log 2>&1 || { echo prof nerfle failed; exit 6; }
find $O/prof_nerfle -name "*kernel_stats.csv" -exec cp {} $O/nerfle_kernel_stats.csv \;
rm -rf $O/prof_nerfle
timeout -k 10 300 python -u bench.py --scene train --steps 20 --warmup 3 > $O/train.jsonl 2> $O/train.err || { echo train failed; exit 7; }
timeout -k 10 300 python -u bench.py --scene train --precision mixed --steps 20 --warmup 3 >> $O/train.jsonl 2>> $O/train.err || { echo train mixed failed; exit 8; }
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_train.log 2>&1 || { echo prof train failed; exit 9; }
find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} $O/train32_kernel_stats.csv \;
echo done
