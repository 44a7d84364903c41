#!/bin/bash
# A/B of dq_quantile_digest: tools/quantile_bench.py against ab_libs/libold.so (the previous library) and
# the in-tree libdqscan.so, alternated, at 1e8 rows.   bash tools/digest_ab.sh TAG
set -o pipefail
T=${1:-dab}
mkdir -p gpurun_out
for k in 1 2; do
  DQ_LIB_PATH=$PWD/ab_libs/libold.so timeout -k 10 120 python3 tools/quantile_bench.py --rows 1e8 --reps 10 > gpurun_out/${T}_old$k.txt 2>&1 || exit $?
  timeout -k 10 120 python3 tools/quantile_bench.py --rows 1e8 --reps 10 > gpurun_out/${T}_new$k.txt 2>&1 || exit $?
done
