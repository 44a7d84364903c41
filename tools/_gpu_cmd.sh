set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "deferred or edge_lengths" > gpurun_out/t10.log 2>&1; rc=$?; tail -3 gpurun_out/t10.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --skip-headline --configs c3 --cpu-sample 0 --ingest-rows 0 > gpurun_out/c3_serial.json 2>gpurun_out/c3_serial.err || exit 2
python3 -c "import json,sys; d=json.load(open('gpurun_out/c3_serial.json')); c=d['configs']['c3']; print('c3', c['ms_per_step'], c['rows_per_s'], {n: round(e['avg_ms'],4) for n,e in c['kernels'].items()})"
