#!/bin/bash
# round-4 GPU call 26 (final tree: digest cells + prefetch): full GPU suite, smoke(), quantile and
# digest timings at 1e8 rows with a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4f2_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4f2_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4f2_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r4f2_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4f2_quantile.txt 2>&1
rc=$?; cat gpurun_out/r4f2_quantile.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f2_qprof -o q -- python3 -u tools/quantile_bench.py --rows 1e8 --reps 2 > gpurun_out/r4f2_qprof.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py > gpurun_out/r4f2_bench.json 2> gpurun_out/r4f2_bench.err
rc=$?; tail -c 300 gpurun_out/r4f2_bench.json | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4f2_bench.err; exit $rc; }
