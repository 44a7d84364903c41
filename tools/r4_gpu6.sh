#!/bin/bash
# round-4 GPU call 6: full GPU suite on the in-tree build (fp64 lazy non-finite check, predicate JIT r4c with
# the loop-ordered prologue, pipelined Correlation ring), then A/B lines: C5 (r3 base / in-tree), C4 (r3 base /
# in-tree), C3 (r4c predicate JIT / in-tree).  Summary lines in gpurun_out/r4f_summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4f_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4f_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
TAG=r4f bash tools/ab_c5.sh build_variants/libbase.so deequ_amd/libdqscan.so build_variants/libbase.so deequ_amd/libdqscan.so | tee -a $S || exit 3
CFG=c4 SKIP_TESTS=1 TAG=r4f4 bash tools/ab_c3.sh build_variants/libbase.so deequ_amd/libdqscan.so build_variants/libbase.so deequ_amd/libdqscan.so | tee -a $S || exit 3
CFG=c3 SKIP_TESTS=1 TAG=r4f3 bash tools/ab_c3.sh build_variants/libprev.so deequ_amd/libdqscan.so build_variants/libprev.so deequ_amd/libdqscan.so | tee -a $S || exit 3
