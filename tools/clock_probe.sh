#!/bin/bash
# Effective clock and VALU issue rate of the headline kernels (MI355X_MICROARCH 'DVFS give-back'): one
# rocprofv3 pass with the kernel trace and GRBM_GUI_ACTIVE / SQ_INSTS_VALU / SQ_WAVES / SQ_BUSY_CYCLES,
# then tools/clock_summary.py.  Usage (GPU box): bash tools/clock_probe.sh TAG
set -u
TAG=${1:-clk}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES \
  -d gpurun_out/$TAG -o c --output-format csv -- \
  python3 bench.py --configs=${CFG:-} --cpu-sample 0 --ingest-rows 0 --rows ${ROWS:-500000000} --steps 3 --warmup 1 \
  > gpurun_out/$TAG.out 2>&1 || { echo "clock probe failed"; tail -5 gpurun_out/$TAG.out; exit 2; }
python3 tools/clock_summary.py gpurun_out/$TAG
