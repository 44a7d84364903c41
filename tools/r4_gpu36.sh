#!/bin/bash
# round-4 GPU call 36: the radix select's equal-digit skip (AND / OR spread over copies) -- quantile GPU tests,
# then the ApproxQuantile(s) timing A/B at 1e8 rows (build_variants/libqold.so = before the skip) on the f64 column
# and on an i64 column uniform in [0, 1e6), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4q3_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4q3_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4q3_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for lib in build_variants/libqold.so deequ_amd/libdqscan.so; do
    for ir in 0 1000000; do
      echo "== $lib int-range=$ir" | tee -a $S
      DQ_LIB_PATH=$lib timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 --int-range $ir > gpurun_out/r4q3_q.txt 2>&1
      rc=$?; grep "quantiles=" gpurun_out/r4q3_q.txt | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4q3_q.txt; exit $rc; }
    done
  done
done
