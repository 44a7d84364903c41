set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "hll or utf8 or deferred or datatype or profile or nan or infinit or config or kat" > gpurun_out/t14.log 2>&1; rc=$?; tail -1 gpurun_out/t14.log; [ $rc -eq 0 ] || exit $rc
for v in A B; do
  L=""; if [ $v = A ]; then L=$PWD/build_variants/libA.so; fi
  DQ_LIB_PATH=$L timeout -k 10 300 python -u bench.py --configs= --cpu-sample 0 --ingest-rows 0 > gpurun_out/h_$v.json 2>gpurun_out/h_$v.err || { tail gpurun_out/h_$v.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/h_$v.json')); k=d['roofline']['kernels']; print('$v', round(d['value']/1e10,4), round(d['ms_per_step'],3), {n: round(e['avg_ms'],4) for n,e in k.items()})"
done
