#!/bin/bash
# round-4 GPU call 39 (final library: + the digest candidate sort over differing bits):
# full GPU suite and smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4f6_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4f6_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4f6_pytest.log | tee $S; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4f6_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4f6_smoke.txt 2>&1
rc=$?; tail -2 gpurun_out/r4f6_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
