set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
TAG=r2j STEPS="prof bench" bash tools/gpu_r2.sh; rc=$?
cp profiles/r2j_* gpurun_out/ 2>/dev/null
exit $rc
