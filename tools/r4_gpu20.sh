#!/bin/bash
# round-4 GPU call 20 (shipped library): the quantile / digest GPU tests (incl. the small and ragged digest sizes),
# then 1e9-row parity of C5 / C4 / C2 (tests/fullscale_parity.py; C3 was re-run in r4q after its last change).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4t_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4t_pytest_quantiles.log 2>&1
rc=$?; tail -2 gpurun_out/r4t_pytest_quantiles.log | tee $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u tests/fullscale_parity.py --cfg c5 c4 c2 --rows 1000000000 \
  --out gpurun_out/r4t_fullscale_parity.json > gpurun_out/r4t_fullscale_parity.txt 2>&1
rc=$?; grep '^{' gpurun_out/r4t_fullscale_parity.txt | cut -c1-300 | tee -a $S; exit $rc
