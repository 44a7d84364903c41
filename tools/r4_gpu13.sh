#!/bin/bash
# round-4 GPU call 13: predicate JIT software-pipelined (libjpipe: row group j + 1's predicate work beside row group
# j's hashing) -- JIT tests on it, C3 A/B against the in-tree pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4m_summary.txt
DQ_LIB_PATH=build_variants/libjpipe.so timeout -k 10 400 python -u -m pytest tests/test_pred_jit_gpu.py tests/test_gpu_parity.py -k "pred or compliance or where or jit or ragged or configs" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4m_pytest_jpipe.log 2>&1
rc=$?; tail -2 gpurun_out/r4m_pytest_jpipe.log | tee $S; [ $rc -eq 0 ] || exit $rc
CFG=c3 SKIP_TESTS=1 TAG=r4m3 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libjpipe.so deequ_amd/libdqscan.so build_variants/libjpipe.so | tee -a $S
