#!/bin/bash
# round-4 GPU call 16: the compiled predicate pass with its counters reduced per workgroup in LDS and spread over 16
# accumulator copies (in-tree, 2048 workgroups; libpwg1024: 1024) vs the previous build (libr4n): JIT / predicate
# tests on the in-tree build, then the C3 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4p_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_pred_jit_gpu.py tests/test_gpu_parity.py tests/test_checks.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4p_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4p_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
CFG=c3 SKIP_TESTS=1 TAG=r4p3 bash tools/ab_c3.sh build_variants/libr4n.so deequ_amd/libdqscan.so build_variants/libpwg1024.so build_variants/libr4n.so deequ_amd/libdqscan.so build_variants/libpwg1024.so | tee -a $S
