#!/bin/bash
# SQ counter passes over the digest kernels (diagnostic): tools/quantile_bench.py at 1e8 rows, one rep; one
# rocprofv3 run per counter set (<= 8 SQ counters each), summarised per kernel by tools/pmc_avg.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
k=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"; do
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/r4w_pmc$k -o p --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 1 > gpurun_out/r4w_pmc$k.out 2>&1 || { echo "fail $k"; tail -5 gpurun_out/r4w_pmc$k.out; exit 2; }
  python3 tools/pmc_avg.py gpurun_out/r4w_pmc$k | grep -E "digest|trampoline|quantile_hist" | cut -c1-600
done
