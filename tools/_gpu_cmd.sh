set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u tools/sweep.py 125000000 > gpurun_out/r2i_sweep.log 2>gpurun_out/r2i_sweep.err; rc=$?; tail -20 gpurun_out/r2i_sweep.log; exit $rc
