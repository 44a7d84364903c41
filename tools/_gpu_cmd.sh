set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --configs= --cpu-sample 0 --ingest-rows 0 --steps 8"
for s in 2 3 4 1 2 3; do
  DQ_STR_RANGE_SCALE=$s timeout -k 10 200 $B > gpurun_out/rs_$s.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/rs_$s.json').read().strip().splitlines()[-1])
print('$s', round(d['value']/1e10,4), round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],4))"
done
