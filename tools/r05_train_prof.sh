# rocprof kernel summary + PMC of the training step's backward kernels (mixed precision step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
PREC=${PREC:-mixed}
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --precision $PREC --steps 5 --warmup 2 --no-cpu-baseline $BENCH_EXTRA > gpurun_out/r05/prof_train.log 2>&1
rc=$?; echo "PROF EXIT $rc"; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r05/prof_train_$PREC && find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05/prof_train_$PREC/ \;
SET="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
rm -rf gpurun_out/r05/pmc_train2
timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "k_mlp_backward32|k_mlp_bwd_ring|k_wgrad_batch|k_mlp_grad_backward32|k_mlp_ring" -d gpurun_out/r05/pmc_train2 -o run --output-format csv -- python3 bench.py --scene train --precision $PREC --steps 3 --warmup 2 --no-cpu-baseline $BENCH_EXTRA > gpurun_out/r05/pmc_train2.log 2>&1
rc=$?; echo "PMC EXIT $rc"; [ $rc -eq 0 ] || exit $rc
