#!/bin/bash
# round-4 GPU call 19: A/B of the Correlation ring's issue priority on C4 (DQ_PAIR_PRIO 0 / 1 / 2, alternating),
# then the rocprofv3 evidence of the shipped library (tools/profile_round.sh r4s).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out/r4s_profiles
export TMPDIR=/tmp
CFG=c4 SKIP_TESTS=1 TAG=r4s bash tools/ab_c3.sh build_variants/libprio0.so build_variants/libprio1.so build_variants/libprio2.so \
  build_variants/libprio0.so build_variants/libprio1.so build_variants/libprio2.so | tee gpurun_out/r4s_ab.txt
rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh r4s > gpurun_out/r4s_profile_round.log 2>&1
rc=$?; cp profiles/r4s_* gpurun_out/r4s_profiles/ 2>/dev/null; tail -3 gpurun_out/r4s_profile_round.log; [ $rc -eq 0 ] || exit $rc
