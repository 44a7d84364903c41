#!/bin/bash
# A/B of builds on one BASELINE config (diagnostic): optional GPU tests with TEST_LIB (pytest -k TEST_K over
# TEST_FILES, comma-separated), then the config's bench line (CFG, default c4) for each library given, in order.
# Stops at the first failure.  Usage (GPU box): TEST_LIB=build_variants/libX.so bash tools/ab_cfg.sh old.so new.so old.so new.so
set -u
TEST_FILES=${TEST_FILES:-tests}  # comma-separated
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
TAG=${TAG:-abcfg}
if [ -n "${TEST_LIB:-}" ]; then
  DQ_LIB_PATH=$TEST_LIB timeout -k 10 600 python -u -m pytest ${TEST_FILES//,/ } -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider ${TEST_K:+-k "$TEST_K"} > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for lib in "$@"; do
  i=$((i+1)); name=$(basename $lib .so)_$i
  DQ_LIB_PATH=$lib timeout -k 10 300 python bench.py --skip-headline --configs=${CFG:-c4} --cpu-sample 0 --ingest-rows 0 \
    --no-plan-timing > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/${TAG}_$name.err; exit 3; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_$name.json').read().strip().splitlines()[-1])
for c,v in d.get('configs',{}).items(): print('$name', c, round(v['ms_per_step'],2), round(v.get('ms_per_step_median',0),2), {k:round(x['avg_ms'],3) for k,x in v.get('kernels',{}).items()})"
done
