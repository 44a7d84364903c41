set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out profiles
TAG=r2i STEPS="tests prof bench" bash tools/gpu_r2.sh; rc=$?
cp profiles/r2i_* gpurun_out/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r2i.log 2>&1; rc=$?; tail -1 gpurun_out/smoke_r2i.log; exit $rc
