#!/bin/bash
# A/B of column-pass builds on the C5 headline (diagnostic): optional GPU tests with the first variant
# (DQ_LIB_PATH), then the headline for each library given, in the order given.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
TAG=${TAG:-ab5}
if [ -n "${TEST_LIB:-}" ]; then
  DQ_LIB_PATH=$TEST_LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for lib in "$@"; do
  i=$((i+1)); name=$(basename $lib .so)_$i
  DQ_LIB_PATH=$lib timeout -k 10 300 python bench.py --configs= --cpu-sample 0 --ingest-rows 0 --no-plan-timing --steps ${STEPS:-8} > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/${TAG}_$name.err; exit 3; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],2), '%.4g'%d['value'], {k[15:]:round(v['avg_ms'],3) for k,v in d['roofline']['kernels'].items()})"
done
