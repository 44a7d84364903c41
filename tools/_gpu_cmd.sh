set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_distributed.py -k "pred or compliance or Compliance or where or config or pattern or string or hll" > gpurun_out/t9.log 2>&1; rc=$?; tail -2 gpurun_out/t9.log; [ $rc -eq 0 ] || exit $rc
for v in S C; do
  E="DQ_PRED_CONCURRENT=1"; if [ $v = S ]; then E="DQ_PRED_CONCURRENT=0"; fi
  env $E timeout -k 10 300 python -u bench.py --skip-headline --configs c3 --cpu-sample 0 --ingest-rows 0 > gpurun_out/c3_$v.json 2>gpurun_out/c3_$v.err || { tail gpurun_out/c3_$v.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/c3_$v.json')); c=d['configs']['c3']; print('$v', c['ms_per_step'], c['rows_per_s'], {n: round(e['avg_ms'],4) for n,e in c['kernels'].items()})"
done
