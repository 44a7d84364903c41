#!/bin/bash
# round-4 GPU call 3: full GPU suite on the new kernels, quantile timing, A/B of the C5 headline (r3 kernels vs
# new), SQ counters of the new build
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r4c_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 --reps 3 > gpurun_out/r4c_quantile_bench.txt 2>&1 || exit $?
cat gpurun_out/r4c_quantile_bench.txt
TAG=r4c bash tools/ab_c5.sh build_variants/libbase.so deequ_amd/libdqscan.so build_variants/libbase.so deequ_amd/libdqscan.so || exit $?
bash tools/pmc_c5.sh r4c_pmc5
