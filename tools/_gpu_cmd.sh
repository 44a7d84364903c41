set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
TAG=r2e STEPS="tests bench full" bash tools/gpu_r2.sh; rc=$?
cp gpurun_out/r2e_fullscale_parity.json gpurun_out/fullscale_r2e.log gpurun_out/ 2>/dev/null
exit $rc
