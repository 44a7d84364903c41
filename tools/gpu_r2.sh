#!/bin/bash
# Round-2 GPU session (run via gpurun): STEPS selects what runs, in order, stopping at the first
# fault / abort / timeout.  tests = pytest -m gpu; bench = bench.py (N=1, all configs);
# full = 1e9-row strict fp64 parity (tests/fullscale_parity.py); prof = tools/profile_round.sh $TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
TAG=${TAG:-r2}
for s in ${STEPS:-tests bench}; do
  case $s in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-1500} python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 400 \
        --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -40 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-900} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
      rc=$?; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"
      [ $rc -eq 0 ] || exit $rc ;;
    full)
      timeout -k 10 ${FULL_TIMEOUT:-900} python -u tests/fullscale_parity.py --rows ${FULL_ROWS:-1000000000} \
        --out gpurun_out/${TAG}_fullscale_parity.json > gpurun_out/fullscale_$TAG.log 2>&1
      rc=$?; tail -8 gpurun_out/fullscale_$TAG.log; echo "full rc=$rc"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    prof)
      bash tools/profile_round.sh $TAG || exit $? ;;
  esac
done
