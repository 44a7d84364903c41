#!/bin/bash
# round-4 GPU call 11 (final evidence, part 2): full GPU suite, smoke(), the quantile / digest timing at 1e8 rows, then
# bench.py with default arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4z_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4z_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4z_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4z_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r4z_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4z_quantile_bench.txt 2>&1
rc=$?; tail -5 gpurun_out/r4z_quantile_bench.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py > gpurun_out/r4z_bench.json 2> gpurun_out/r4z_bench.err
rc=$?; tail -c 600 gpurun_out/r4z_bench.json | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4z_bench.err; exit $rc; }
# diagnostic: the Correlation ring without its per-slot barrier (libnobar, results wrong) vs the in-tree pass on C4
CFG=c4 SKIP_TESTS=1 TAG=r4j4 bash tools/ab_c3.sh deequ_amd/libdqscan.so build_variants/libnobar.so deequ_amd/libdqscan.so build_variants/libnobar.so | tee gpurun_out/r4j_summary.txt
