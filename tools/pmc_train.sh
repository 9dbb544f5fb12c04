# PMC pass on the training step's MLP backward kernels (and the weight-gradient / double-backward
# kernels beside them): the column-split kernels (option
# bwd_colsplit=1, the default) and the round-3 per-wave kernels (bwd_colsplit=0), one
# rocprofv3 run per option (each killed after 90 s).  bash tools/pmc_train.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_train
mkdir -p gpurun_out/pmc_train
SET="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
for OPT in 1 0; do
  timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-include-regex "k_mlp_backward32|k_wgrad_batch|k_mlp_grad_backward32" -d gpurun_out/pmc_train/o$OPT -o run --output-format csv -- python3 bench.py --scene train --precision mixed --steps 1 --warmup 0 --nrt-option bwd_colsplit=$OPT > gpurun_out/pmc_train/o$OPT.log 2>&1 || { echo "pmc $OPT failed"; tail -5 gpurun_out/pmc_train/o$OPT.log; exit 1; }
  echo "pmc $OPT ok"
done
