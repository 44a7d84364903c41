#!/bin/bash
# round-4 GPU call 7: the LDS-staged UTF8 variant's per-length check (tools/stg_dbg.py), the UTF8 A/B switches
# (round-3 offsets loads / window check) on the C5 headline with the string tests on the combined variant,
# SQ passes over C3 (predicate JIT r4c) and C4 (pipelined ring).  Summary in gpurun_out/r4g_summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4g_summary.txt
DQ_LIB_PATH=build_variants/libstg.so timeout -k 10 300 python -u tools/stg_dbg.py > gpurun_out/r4g_stg_dbg.txt 2>&1
echo "stg_dbg rc=$?" | tee $S; tail -14 gpurun_out/r4g_stg_dbg.txt | tee -a $S
DQ_LIB_PATH=build_variants/libuboth.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "utf8 or profile" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g_pytest_uboth.log 2>&1
rc=$?; tail -2 gpurun_out/r4g_pytest_uboth.log | tee -a $S; [ $rc -eq 0 ] || exit $rc
TAG=r4g bash tools/ab_c5.sh deequ_amd/libdqscan.so build_variants/libusoff.so build_variants/libuwchk.so build_variants/libuboth.so deequ_amd/libdqscan.so build_variants/libusoff.so build_variants/libuwchk.so build_variants/libuboth.so | tee -a $S || exit 3
CFG=c3 TAG=r4g_pmc3 bash tools/pmc_c3.sh deequ_amd/libdqscan.so | tee -a $S || exit 2
CFG=c4 TAG=r4g_pmc4 bash tools/pmc_c3.sh deequ_amd/libdqscan.so | tee -a $S || exit 2
for d in gpurun_out/r4g_pmc3_libdqscan gpurun_out/r4g_pmc4_libdqscan; do python3 tools/pmc_avg.py $d; done > gpurun_out/r4g_pmc.txt 2>&1; cat gpurun_out/r4g_pmc.txt | tee -a $S
