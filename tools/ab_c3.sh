#!/bin/bash
# A/B of the predicate pass on the C3 config (diagnostic): GPU suite on the default build, then the C3 line
# for each library given (DQ_LIB_PATH), printing the per-kernel averages.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in "$@"; do
  name=$(basename $lib .so)
  DQ_LIB_PATH=$lib timeout -k 10 300 python bench.py --skip-headline --configs=${CFG:-c3} --cpu-sample 0 --ingest-rows 0 > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/${TAG}_$name.err; exit 3; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${TAG}_$name.json').read().strip().splitlines()[-1])
for c,v in d.get('configs',{}).items(): print('$name', c, round(v['ms_per_step'],2), round(v.get('ms_per_step_median',0),2), {k:round(x['avg_ms'],3) for k,x in v.get('kernels',{}).items()})"
done
