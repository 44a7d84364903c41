set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=r2o STEPS="tests" bash tools/gpu_r2.sh && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r2o.log 2>&1 && \
TAG=r2o STEPS="bench" bash tools/gpu_r2.sh
