#!/bin/bash
# wg_sweep.sh -- tools/sweep.py under several column-launch workgroup targets (DQ_TARGET_WGS)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for t in 2048 4096 8192 16384; do
  DQ_TARGET_WGS=$t timeout -k 10 300 python tools/sweep.py > gpurun_out/wg_$t.log 2>&1 || exit $?
  echo "target $t"; grep -oE '"case": "[a-z0-9_]+"|"column": [0-9.]+' gpurun_out/wg_$t.log | paste - - | tr '\n' ' '; echo
done
