#!/bin/bash
# round-4 GPU call 12: 1e9-row parity of C3 / C5 / C4 / C2 on the final kernels (tests/fullscale_parity.py: integer
# results bit-exact vs the C oracle, fp64 within 1e-12 strict of a double-double reference), then the Correlation
# ring with LDS flags instead of its per-slot barrier (libpflags): pair-pass tests on it and a C4 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u tests/fullscale_parity.py --cfg c3 c5 c4 c2 --rows 1000000000 \
  --out gpurun_out/r4z_fullscale_parity.json > gpurun_out/r4z_fullscale_parity.txt 2>&1
rc=$?; grep '^{' gpurun_out/r4z_fullscale_parity.txt | cut -c1-300; [ $rc -eq 0 ] || exit $rc
S=gpurun_out/r4k_summary.txt
DQ_LIB_PATH=build_variants/libpflags.so timeout -k 10 300 python -u -m pytest tests/test_pair_lane.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4k_pytest_pflags.log 2>&1
rc=$?; tail -2 gpurun_out/r4k_pytest_pflags.log | tee $S; [ $rc -eq 0 ] || exit $rc
CFG=c4 SKIP_TESTS=1 TAG=r4k4 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libpflags.so deequ_amd/libdqscan.so build_variants/libpflags.so | tee -a $S
