set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --configs= --cpu-sample 0 --ingest-rows 0 --steps 8"
for t in 8192 4096 12288 16384 8192; do
  DQ_TARGET_WGS=$t timeout -k 10 200 $B > gpurun_out/tw_$t.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/tw_$t.json').read().strip().splitlines()[-1])
k=d['roofline']['kernels']
print('$t', round(d['value']/1e10,4), round(d['ms_per_step'],2), {n[15:]:round(v['avg_ms'],3) for n,v in k.items() if 'column' in n})"
done
