# Round-5 training probe: the default bench line (with its train legs), the FP32 training step's
# rocprof kernel summary, and a PMC pass over the backward kernels of 3 steady-state steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u bench.py > gpurun_out/r05/bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -c 600 gpurun_out/r05/bench.log; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --scene train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05/prof_train_fp32.log 2>&1
rc=$?; echo "PROF TRAIN EXIT $rc"; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/r05/prof_train_fp32 && find /tmp/prof_train -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05/prof_train_fp32/ \;
SET="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "k_mlp_backward32|k_wgrad_batch|k_mlp_grad_backward32|k_march32|k_mlp_ring" -d gpurun_out/r05/pmc_train -o run --output-format csv -- python3 bench.py --scene train --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r05/pmc_train.log 2>&1
rc=$?; echo "PMC EXIT $rc"; [ $rc -eq 0 ] || exit $rc
