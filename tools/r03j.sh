# round 3: PMC of the training step's backward kernels (k_wgrad_batch, k_mlp_backward32)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/pmc
BENCH_ARGS="--scene train --steps 1 --warmup 1 --no-cpu-baseline" bash tools/pmc.sh "k_wgrad_batch|k_mlp_backward32" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" || exit 1
