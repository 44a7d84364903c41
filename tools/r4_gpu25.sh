#!/bin/bash
# round-4 GPU call 25: the radix select's next-iteration prefetch -- quantile / digest GPU tests on the new build, the 1e8-row
# digest timing A/B (build_variants/libprio0.so = the shipped digest, in-tree = cells), alternating, and one SQ pass
# (LDS bank conflicts / LDS waits) of the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4z2_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4z2_pytest_quantiles.log 2>&1
rc=$?; tail -2 gpurun_out/r4z2_pytest_quantiles.log | tee $S; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for lib in build_variants/libprio0.so deequ_amd/libdqscan.so; do
    echo "== $lib" | tee -a $S
    DQ_LIB_PATH=$lib timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4z2_q.txt 2>&1
    rc=$?; grep -E "digest|quantiles=" gpurun_out/r4z2_q.txt | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4z2_q.txt; exit $rc; }
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4z2_qprof -o q --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 3 > gpurun_out/r4z2_qprof.log 2>&1 || { tail -5 gpurun_out/r4z2_qprof.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d gpurun_out/r4z2_pmc -o p --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 1 > gpurun_out/r4z2_pmc.out 2>&1 || { echo "pmc fail"; exit 6; }
