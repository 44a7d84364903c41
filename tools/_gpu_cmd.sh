set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > gpurun_out/t13.log 2>&1; rc=$?; tail -3 gpurun_out/t13.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke2.log 2>&1; rc=$?; tail -1 gpurun_out/smoke2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --skip-headline --configs c4 --cpu-sample 0 --ingest-rows 0 > gpurun_out/c4_final.json 2>gpurun_out/c4_final.err || exit 2
python3 -c "import json,sys; d=json.load(open('gpurun_out/c4_final.json')); c=d['configs']['c4']; print('c4', c['ms_per_step'], c['rows_per_s'], c['roofline'])"
