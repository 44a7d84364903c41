#!/bin/bash
# round-4 GPU call 21: the digest's splitter lookup table -- quantile / digest GPU tests on the new build, then the
# 1e8-row digest timing A/B (build_variants/libprio0.so = the previous digest, in-tree = lookup table), alternating,
# and a kernel trace of the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4u_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4u_pytest_quantiles.log 2>&1
rc=$?; tail -2 gpurun_out/r4u_pytest_quantiles.log | tee $S; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for lib in build_variants/libprio0.so deequ_amd/libdqscan.so; do
    echo "== $lib" | tee -a $S
    DQ_LIB_PATH=$lib timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4u_q.txt 2>&1
    rc=$?; grep digest gpurun_out/r4u_q.txt | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4u_q.txt; exit $rc; }
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4u_qprof -o q --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 2 > gpurun_out/r4u_qprof.log 2>&1 || { tail -5 gpurun_out/r4u_qprof.log; exit 5; }
