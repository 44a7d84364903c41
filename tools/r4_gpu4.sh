#!/bin/bash
# round-4 GPU call 4: GPU parity tests touching the column pass (in-tree build, then the LDS-staged UTF8 variant),
# unaligned-LDS probe, A/B of the C5 headline: r3 kernels (base), the r4c build (prev), this build, staged UTF8
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullscale.py tests/test_hll_redo.py tests/test_checks.py -x -v --durations=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4d_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r4d_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/micro/lds_unaligned_probe > gpurun_out/r4d_lds_probe.txt 2>&1; cat gpurun_out/r4d_lds_probe.txt
DQ_LIB_PATH=build_variants/libstg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_hll_redo.py -x -q -k "utf8 or profile or configs or redo or string or chunked" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4d_pytest_stg.log 2>&1
rc=$?; tail -3 gpurun_out/r4d_pytest_stg.log; [ $rc -eq 0 ] || exit $rc
TAG=r4d bash tools/ab_c5.sh build_variants/libbase.so build_variants/libprev.so deequ_amd/libdqscan.so build_variants/libstg.so build_variants/libbase.so deequ_amd/libdqscan.so build_variants/libstg.so
