#!/bin/bash
# round-4 GPU call 2: compiled-predicate / quantile tests, quantile timing, SQ counter passes of C5
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_pred_jit_gpu.py tests/test_quantiles.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b_pytest_jit.log 2>&1
rc=$?; tail -5 gpurun_out/r4b_pytest_jit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 --reps 3 > gpurun_out/r4b_quantile_bench.txt 2>&1 || exit $?
cat gpurun_out/r4b_quantile_bench.txt
bash tools/pmc_c5.sh r4b_pmc5
