#!/bin/bash
# round-4 GPU call 12: the digest's GPU tests and timing (pooled scratch) with a kernel trace of it, then 1e9-row
# parity of C3 / C5 / C4 / C2 on the final kernels (tests/fullscale_parity.py: integer results bit-exact vs the C
# oracle, fp64 within 1e-12 strict of a double-double reference).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4l_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4l_pytest_quantiles.log 2>&1
rc=$?; tail -2 gpurun_out/r4l_pytest_quantiles.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4l_quantile_bench.txt 2>&1
rc=$?; tail -5 gpurun_out/r4l_quantile_bench.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4l_qprof -o q --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 2 > gpurun_out/r4l_qprof.log 2>&1 || { tail -5 gpurun_out/r4l_qprof.log; exit 5; }
timeout -k 10 800 python -u tests/fullscale_parity.py --cfg c3 c5 c4 c2 --rows 1000000000 \
  --out gpurun_out/r4z_fullscale_parity.json > gpurun_out/r4z_fullscale_parity.txt 2>&1
rc=$?; grep '^{' gpurun_out/r4z_fullscale_parity.txt | cut -c1-300 | tee -a $S; exit $rc
