#!/bin/bash
# round-4 GPU call 13: the digest's candidate pass staged in LDS (quantile GPU tests + 1e8-row timing + kernel trace),
# then the predicate JIT software-pipelined (libjpipe): JIT tests on it and a C3 A/B against the in-tree pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4m_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4m_pytest_quantiles.log 2>&1
rc=$?; tail -2 gpurun_out/r4m_pytest_quantiles.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4m_quantile_bench.txt 2>&1
rc=$?; tail -5 gpurun_out/r4m_quantile_bench.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4m_qprof -o q --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 2 > gpurun_out/r4m_qprof.log 2>&1 || { tail -5 gpurun_out/r4m_qprof.log; exit 5; }
DQ_LIB_PATH=build_variants/libjpipe.so timeout -k 10 400 python -u -m pytest tests/test_pred_jit_gpu.py tests/test_gpu_parity.py -k "pred or compliance or where or jit or ragged or configs" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4m_pytest_jpipe.log 2>&1
rc=$?; tail -2 gpurun_out/r4m_pytest_jpipe.log | tee -a $S; [ $rc -eq 0 ] || exit $rc
CFG=c3 SKIP_TESTS=1 TAG=r4m3 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libjpipe.so deequ_amd/libdqscan.so build_variants/libjpipe.so | tee -a $S
