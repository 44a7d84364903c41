set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
TAG=r2g STEPS="tests prof bench full" bash tools/gpu_r2.sh; rc=$?
cp profiles/r2g_* gpurun_out/ 2>/dev/null
exit $rc
