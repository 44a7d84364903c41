#!/bin/bash
# round-4 GPU call 33: bench.py with default arguments on the final library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u bench.py > gpurun_out/r4f4_bench.json 2> gpurun_out/r4f4_bench.err
rc=$?; tail -c 300 gpurun_out/r4f4_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4f4_bench.err; exit $rc; }
