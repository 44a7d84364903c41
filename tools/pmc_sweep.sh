#!/bin/bash
# pmc_sweep.sh <label> <case-filter> <counter>... -- one rocprofv3 counter pass over tools/sweep.py
# (one case), CSV under gpurun_out/pmc_<label>; summarise locally with tools/pmc_avg.py.
set -u
L=$1; C=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$L -o pmc --output-format csv -- \
  python3 tools/sweep.py 62500000 "$C" > gpurun_out/pmc_$L.log 2>&1
