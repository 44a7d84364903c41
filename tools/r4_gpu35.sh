#!/bin/bash
# round-4 GPU call 35: the radix select skips the passes over digits equal in every key -- full GPU suite (incl. the
# new skip cases), smoke(), quantile timing at 1e8 rows on a small-range i64 column and the f64 column.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4q2_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4q2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4q2_pytest.log | tee $S; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4q2_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4q2_smoke.txt 2>&1
rc=$?; tail -1 gpurun_out/r4q2_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 > gpurun_out/r4q2_q.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r4q2_q.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quantile_bench.py --rows 1e8 --int-range 1000000 > gpurun_out/r4q2_qi.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r4q2_qi.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
