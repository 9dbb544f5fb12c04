# round 3: k_march16 with the SphereSDF table in LDS (two lanes per ray split the spheres):
# colocate (64 spheres) and headline fp16 frames, the march suites, PMC of the colocate k_march16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u bench.py --scene colocate --precision fp16 --steps 5 --warmup 2 > gpurun_out/r03g/colocate_fp16.json 2> gpurun_out/r03g/colocate.err
rc=$?; echo "COLOCATE EXIT $rc"; tail -c 600 gpurun_out/r03g/colocate_fp16.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --precision fp16 --no-cpu-baseline --no-extra-legs > gpurun_out/r03g/head_fp16.json 2> gpurun_out/r03g/head.err
rc=$?; echo "HEAD EXIT $rc"; tail -c 300 gpurun_out/r03g/head_fp16.json; [ $rc -eq 0 ] || exit $rc
NRT_REPORT=gpurun_out/r03g/report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_ring32.py -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03g/tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -4 gpurun_out/r03g/tests.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/pmc
BENCH_ARGS="--scene colocate --precision fp16 --steps 1 --warmup 0 --no-cpu-baseline --no-extra-legs" bash tools/pmc.sh k_march16 "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" || exit 1
