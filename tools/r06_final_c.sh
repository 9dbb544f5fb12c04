# round 6 final, part C: refresh the scene PMC traffic files the line staging changed (the plain
# k_march32 / k_march3 / k_march16 of colocate and dtu), then part B (every scene line + training)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "colocate fp16 k_march16 800 k_march16" "colocate fp32-split k_march3 800 k_march3" "colocate fp32 k_march32 800 k_march32" "dtu fp16 k_march16 800 k_march16" "dtu fp32-split k_march3 800 k_march3" "dtu fp32 k_march32 800 k_march32"; do
  bash tools/r06_pmc_scenes.sh $a > /dev/null || { echo "pmc $a failed"; exit 1; }
done
mkdir -p ${FINAL_DIR:-gpurun_out/r06/final}/pmc_scenes
cp profiles/pmc_*_k_*.json ${FINAL_DIR:-gpurun_out/r06/final}/pmc_scenes/
echo pmc ok
bash tools/r06_final_b.sh
