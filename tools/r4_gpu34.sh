#!/bin/bash
# round-4 GPU call 34: single-chunk verify_runs with the column descriptor in the kernel arguments -- full GPU suite,
# smoke(), grouping timing at 1e8 rows and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4g7_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g7_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4g7_pytest.log | tee $S; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4g7_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4g7_smoke.txt 2>&1
rc=$?; tail -1 gpurun_out/r4g7_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/group_bench.py --rows 1e8 > gpurun_out/r4g7_g.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r4g7_g.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g7_gprof -o g --output-format csv -- python3 tools/group_bench.py --rows 1e8 --reps 1 > gpurun_out/r4g7_gprof.log 2>&1 || { tail -5 gpurun_out/r4g7_gprof.log; exit 5; }
