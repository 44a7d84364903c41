#!/bin/bash
# round-4 GPU call 14 (final tree): full GPU suite, smoke(), the quantile / digest timing at 1e8 rows with its kernel
# trace, then bench.py with default arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4n_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4n_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4n_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4n_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r4n_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4n_quantile_bench.txt 2>&1
rc=$?; tail -5 gpurun_out/r4n_quantile_bench.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4n_qprof -o q --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 2 > gpurun_out/r4n_qprof.log 2>&1 || { tail -5 gpurun_out/r4n_qprof.log; exit 5; }
timeout -k 10 700 python -u bench.py > gpurun_out/r4n_bench.json 2> gpurun_out/r4n_bench.err
rc=$?; tail -c 400 gpurun_out/r4n_bench.json | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4n_bench.err; exit $rc; }
# C2 (8 x f64 moments, the stats-only column pass) against the round-3 kernels
CFG=c2 SKIP_TESTS=1 TAG=r4n2 bash tools/ab_c3.sh build_variants/libbase.so deequ_amd/libdqscan.so build_variants/libbase.so deequ_amd/libdqscan.so | tee -a $S
