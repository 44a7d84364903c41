set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests > gpurun_out/t15.log 2>&1; rc=$?; tail -2 gpurun_out/t15.log; [ $rc -eq 0 ] || exit $rc
for t in 0 1 0 1; do
  DQ_VARIANT_RANGES=$t timeout -k 10 300 python -u bench.py --configs= --cpu-sample 0 --ingest-rows 0 > gpurun_out/h_vr$t.json 2>gpurun_out/h_vr$t.err || { tail gpurun_out/h_vr$t.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/h_vr$t.json')); k=d['roofline']['kernels']; print('vr$t', round(d['value']/1e10,4), round(d['ms_per_step'],3), {n: round(e['avg_ms'],4) for n,e in k.items()})"
done
