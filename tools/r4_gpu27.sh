#!/bin/bash
# round-4 GPU call 27: grouping analyzers' timing at 1e8 rows (tools/group_bench.py) with a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/group_bench.py --rows 1e8 > gpurun_out/r4g2_group.txt 2>&1
rc=$?; cat gpurun_out/r4g2_group.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g2_gprof -o g --output-format csv -- python3 tools/group_bench.py --rows 1e8 --reps 1 > gpurun_out/r4g2_gprof.log 2>&1 || { tail -5 gpurun_out/r4g2_gprof.log; exit 5; }
