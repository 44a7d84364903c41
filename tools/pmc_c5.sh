#!/bin/bash
# SQ counter passes over the C5 headline kernels (2 chunks of 125 M rows), one rocprofv3 run per pass, then
# tools/pmc_avg.py per pass.  Usage (GPU box): bash tools/pmc_c5.sh TAG [lib.so]
# PASSES="ctrs;ctrs;..." replaces the three default passes (each within one pass's per-block limits).
set -u
TAG=${1:-pmc5}
LIB=${2:-deequ_amd/libdqscan.so}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="bench.py --rows 250000000 --steps 1 --warmup 0 --configs= --cpu-sample 0 --ingest-rows 0 --no-plan-timing"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VSKIPPED"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC"
IFS=';' read -r -a PL <<< "${PASSES:-$P1;$P2;$P3}"
i=0
for P in "${PL[@]}"; do
  i=$((i+1))
  DQ_LIB_PATH=$LIB timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/${TAG}_p$i -o p --output-format csv -- python3 $B \
    > gpurun_out/${TAG}_p$i.out 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.out; exit 2; }
done
for i in $(seq 1 ${#PL[@]}); do python3 tools/pmc_avg.py gpurun_out/${TAG}_p$i; done > gpurun_out/${TAG}.txt 2>&1
cat gpurun_out/${TAG}.txt
