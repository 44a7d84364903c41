set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pred or compliance or Compliance or where or config or pattern or string" > gpurun_out/t11.log 2>&1; rc=$?; tail -2 gpurun_out/t11.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c3_fs -o fs --output-format csv -- python3 bench.py --skip-headline --configs c3 --config-rows 125000000 --config-steps 1 --cpu-sample 0 --ingest-rows 0 > /dev/null 2> gpurun_out/c3_fs.err || { tail -5 gpurun_out/c3_fs.err; exit 4; }
python3 tools/pmc_avg.py gpurun_out/c3_fs | grep pred
timeout -k 10 600 python -u bench.py --skip-headline --configs c3 --cpu-sample 0 --ingest-rows 0 > gpurun_out/c3_reuse.json 2>gpurun_out/c3_reuse.err || exit 2
python3 -c "import json,sys; d=json.load(open('gpurun_out/c3_reuse.json')); c=d['configs']['c3']; print('c3', c['ms_per_step'], c['rows_per_s'], {n: round(e['avg_ms'],4) for n,e in c['kernels'].items()})"
