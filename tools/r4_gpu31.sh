#!/bin/bash
# round-4 GPU call 31: grouping's radix sort over the keys' differing bits only -- full GPU suite on the new build, then the grouping
# timing A/B at 1e8 rows (build_variants/libprio0.so = the previous grouping; in-tree = group_compact) and a
# kernel trace of the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4g6_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g6_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4g6_pytest.log | tee $S; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4g6_pytest.log | head -20; exit $rc; }
for lib in build_variants/libprio0.so deequ_amd/libdqscan.so; do
  echo "== $lib" | tee -a $S
  DQ_LIB_PATH=$lib timeout -k 10 400 python -u tools/group_bench.py --rows 1e8 > gpurun_out/r4g6_g.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r4g6_g.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g6_gprof -o g --output-format csv -- python3 tools/group_bench.py --rows 1e8 --reps 1 > gpurun_out/r4g6_gprof.log 2>&1 || { tail -5 gpurun_out/r4g6_gprof.log; exit 5; }
