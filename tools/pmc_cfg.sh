#!/bin/bash
# SQ counter passes (the three of tools/pmc_c5.sh) over one config's kernels: bash tools/pmc_cfg.sh TAG CFG [lib.so]
# (CFG = c2 / c3 / c4, 250 M rows, one step), then tools/pmc_avg.py per pass into gpurun_out/TAG.txt.
set -u
TAG=${1:-pmccfg}
CFG=${2:-c3}
LIB=${3:-deequ_amd/libdqscan.so}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="bench.py --skip-headline --configs=$CFG --config-rows 250000000 --config-steps 1 --cpu-sample 0 --ingest-rows 0"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VSKIPPED"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  DQ_LIB_PATH=$LIB timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/${TAG}_p$i -o p --output-format csv -- python3 $B \
    > gpurun_out/${TAG}_p$i.out 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.out; exit 2; }
done
for i in 1 2 3; do python3 tools/pmc_avg.py gpurun_out/${TAG}_p$i; done > gpurun_out/${TAG}.txt 2>&1
grep -E "dq_pred|dq_pair|column_scan" gpurun_out/${TAG}.txt
