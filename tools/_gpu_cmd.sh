set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --skip-headline --configs c3 --cpu-sample 0 --ingest-rows 0 --config-steps 6"
for w in 2048 1024 4096 8192 16384 2048; do
  DQ_PRED_WGS=$w timeout -k 10 200 $B > gpurun_out/pw_$w.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/pw_$w.json').read().strip().splitlines()[-1])['configs']['c3']
print('$w', round(d['ms_per_step_median'],2), {k:round(x['avg_ms'],3) for k,x in d['kernels'].items()})"
done
