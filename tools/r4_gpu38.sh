#!/bin/bash
# round-4 GPU call 38: the digest's candidate sort over the candidates' differing bits -- quantile GPU tests,
# then the ApproxQuantile(s) timing A/B at 1e8 rows (build_variants/libdold.so = before the skip) on the f64 column
# and on an i64 column uniform in [0, 1e6), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4d2_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4d2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4d2_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for lib in build_variants/libdold.so deequ_amd/libdqscan.so; do
    for ir in 0 1000000; do
      echo "== $lib int-range=$ir" | tee -a $S
      DQ_LIB_PATH=$lib timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 --int-range $ir > gpurun_out/r4d2_q.txt 2>&1
      rc=$?; grep "digest" gpurun_out/r4d2_q.txt | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4d2_q.txt; exit $rc; }
    done
  done
done
