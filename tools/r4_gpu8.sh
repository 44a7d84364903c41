#!/bin/bash
# round-4 GPU call 8: predicate-JIT variants on C3 -- in-tree (r4c: loop-ordered prologue, 8 row groups per
# wave block), jit8 (r4d: the group's hashes emitted before its register updates), jitg4 (r4d, 4 row groups:
# 72 VGPRs, 7 waves) -- JIT tests on jitg4, the A/B, and the three SQ passes over C3 on the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4h_summary.txt
DQ_LIB_PATH=build_variants/libjitg4.so timeout -k 10 400 python -u -m pytest tests/test_pred_jit_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4h_pytest_jitg4.log 2>&1
rc=$?; tail -2 gpurun_out/r4h_pytest_jitg4.log | tee $S; [ $rc -eq 0 ] || exit $rc
CFG=c3 SKIP_TESTS=1 TAG=r4h3 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libjit8.so build_variants/libjitg4.so deequ_amd/libdqscan.so build_variants/libjit8.so build_variants/libjitg4.so | tee -a $S || exit 3
bash tools/pmc_cfg.sh r4h_pmc3 c3 | tee -a $S || exit 2
