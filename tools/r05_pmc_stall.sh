# stall breakdown of the training step's ring kernels (one PMC pass, SQ counters only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
PREC=${PREC:-mixed}
SET="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
OUT=${OUT:-pmc_stall}
ARGS=${BENCH_ARGS:---scene train --precision $PREC --steps 2 --warmup 2 --no-cpu-baseline}
rm -rf gpurun_out/r05/$OUT
timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex "${KREGEX:-k_mlp_bwd_ring|k_wgrad|k_march|k_mlp_ring}" -d gpurun_out/r05/$OUT -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/r05/$OUT.log 2>&1
rc=$?; echo "PMC EXIT $rc"; exit $rc
