#!/bin/bash
# round-4 GPU call: issue-rate probe, counter list, compiled-predicate-pass and quantile-digest tests, digest timing
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/issue_probe > gpurun_out/r4a_issue_probe.txt 2>&1 || exit $?
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4a_counters.txt 2>&1
timeout -k 10 120 ./tools/micro/strhash_probe > gpurun_out/r4a_strhash_probe.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_pred_jit_gpu.py tests/test_quantiles.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a_pytest_jit.log 2>&1
rc=$?; tail -5 gpurun_out/r4a_pytest_jit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 --reps 3 > gpurun_out/r4a_quantile_bench.txt 2>&1
rc=$?; cat gpurun_out/r4a_quantile_bench.txt; exit $rc
