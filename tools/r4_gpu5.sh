#!/bin/bash
# round-4 GPU call 5: the pipelined Correlation ring (build_variants/libpipe.so): pair-pass tests and the
# full-scale C2 / C4 test on it, C4 A/B against the in-tree build (round-3 ring); C3 A/B of the predicate
# JIT's row loop (libprev: 64-bit rows, in-tree: 32-bit); SQ pass over C3 and C4 with the new kernels
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
DQ_LIB_PATH=build_variants/libpipe.so timeout -k 10 600 python -u -m pytest tests/test_pair_lane.py tests/test_fullscale.py -x -v --durations=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4e_pytest_pipe.log 2>&1
rc=$?; tail -4 gpurun_out/r4e_pytest_pipe.log; [ $rc -eq 0 ] || exit $rc
CFG=c4 SKIP_TESTS=1 TAG=r4e bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libpipe.so deequ_amd/libdqscan.so build_variants/libpipe.so || exit 3
CFG=c3 SKIP_TESTS=1 TAG=r4e3 bash tools/ab_c3.sh build_variants/libprev.so deequ_amd/libdqscan.so build_variants/libprev.so deequ_amd/libdqscan.so || exit 3
CFG=c4 TAG=r4e_pmc4 bash tools/pmc_c3.sh build_variants/libpipe.so || exit 2
CFG=c3 TAG=r4e_pmc3 bash tools/pmc_c3.sh deequ_amd/libdqscan.so || exit 2
for d in gpurun_out/r4e_pmc4_libpipe gpurun_out/r4e_pmc3_libdqscan; do python3 tools/pmc_avg.py $d; done > gpurun_out/r4e_pmc.txt 2>&1; cat gpurun_out/r4e_pmc.txt
