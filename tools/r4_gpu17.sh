#!/bin/bash
# round-4 GPU call 17 (final tree): full GPU suite, smoke(), 1e9-row parity of C3 (the predicate counters' new
# accumulation), bench.py with default arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4q_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4q_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4q_pytest.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4q_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r4q_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tests/fullscale_parity.py --cfg c3 --rows 1000000000 --out gpurun_out/r4q_fullscale_c3.json > gpurun_out/r4q_fullscale_c3.txt 2>&1
rc=$?; grep '^{' gpurun_out/r4q_fullscale_c3.txt | cut -c1-300 | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py > gpurun_out/r4q_bench.json 2> gpurun_out/r4q_bench.err
rc=$?; tail -c 300 gpurun_out/r4q_bench.json | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4q_bench.err; exit $rc; }
