#!/bin/bash
# round-4 GPU call 9: full GPU suite on the in-tree build (predicate JIT r4d emission, staged UTF8 variant removed),
# smoke(), then the predicate JIT's scheduling-barrier mask on C3: in-tree (0: nothing crosses), jsb2 (VALU may
# cross), jsb1 (all ALU may cross).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4i_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4i_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4i_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4i_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r4i_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
CFG=c3 SKIP_TESTS=1 TAG=r4i3 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libjsb2.so build_variants/libjsb1.so deequ_amd/libdqscan.so build_variants/libjsb2.so build_variants/libjsb1.so | tee -a $S || exit 3
