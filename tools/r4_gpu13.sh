#!/bin/bash
# round-4 GPU call 13: the Correlation ring with LDS flags instead of its per-slot barrier (libpflags) -- pair-pass
# tests and the C4 full-scale test on it, then C4 A/B against the in-tree pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4k_summary.txt
DQ_LIB_PATH=build_variants/libpflags.so timeout -k 10 300 python -u -m pytest tests/test_pair_lane.py tests/test_fullscale.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4k_pytest_pflags.log 2>&1
rc=$?; tail -2 gpurun_out/r4k_pytest_pflags.log | tee $S; [ $rc -eq 0 ] || exit $rc
CFG=c4 SKIP_TESTS=1 TAG=r4k4 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libpflags.so deequ_amd/libdqscan.so build_variants/libpflags.so | tee -a $S
