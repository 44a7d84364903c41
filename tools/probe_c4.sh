#!/bin/bash
# C4 pair-pass probe: timing (bench configs only) + one SQ counter pass of the pair kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-probe}
timeout -k 10 300 python -u bench.py --skip-headline --configs ${CFGS:-c4} --config-rows ${ROWS:-250000000} --cpu-sample 0 > gpurun_out/${TAG}_bench.json 2>gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 2; }
cat gpurun_out/${TAG}_bench.json
if [ "${PMC:-1}" = "1" ]; then
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/${TAG}_pmc -o pmc --output-format csv -- python3 bench.py --skip-headline --configs ${CFGS:-c4} --config-rows 125000000 --config-steps 1 --cpu-sample 0 > /dev/null 2>gpurun_out/${TAG}_pmc.err || { tail -5 gpurun_out/${TAG}_pmc.err; exit 3; }
python3 tools/pmc_avg.py gpurun_out/${TAG}_pmc 2>/dev/null | head -30
fi
