set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 tests/test_pair_lane.py --timeout-method thread > gpurun_out/t6.log 2>&1; rc=$?; tail -5 gpurun_out/t6.log; exit $rc
