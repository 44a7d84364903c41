#!/bin/bash
# One GPU session: parity tests, then a short bench and a rocprofv3 kernel-trace summary.
# Stops at the first fault / abort / timeout (exit codes other than 0 / 1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
ROWS=${ROWS:-100000000}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --maxfail=20 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --rows $ROWS --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
echo "bench rc=$brc"
exit $brc
