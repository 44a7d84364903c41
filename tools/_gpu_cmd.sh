set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fullscale.py > gpurun_out/t7.log 2>&1; rc=$?; tail -3 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
DQ_LIB_PATH=$PWD/build_variants/libW6.so timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "infinit or nan or profile" > gpurun_out/t7w.log 2>&1; rc=$?; tail -2 gpurun_out/t7w.log; [ $rc -eq 0 ] || exit $rc
for v in A W6 B; do
  L=""
  if [ $v != B ]; then L=$PWD/build_variants/lib$v.so; fi
  DQ_LIB_PATH=$L timeout -k 10 300 python -u bench.py --configs=c2 --cpu-sample 0 --ingest-rows 0 > gpurun_out/h_$v.json 2>gpurun_out/h_$v.err || { tail gpurun_out/h_$v.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/h_$v.json')); k=d['roofline']['kernels']; print('$v', d['value'], d['ms_per_step'], {n: round(e['avg_ms'],4) for n,e in k.items()}, 'c2', d['configs']['c2']['ms_per_step'])"
done
