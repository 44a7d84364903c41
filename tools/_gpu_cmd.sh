set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=r2n STEPS="tests bench" bash tools/gpu_r2.sh
