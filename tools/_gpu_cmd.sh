set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
DQ_LIB_PATH=$PWD/build_variants/libP4.so timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_pair_lane.py -k "all_f64" > gpurun_out/t12.log 2>&1; rc=$?; tail -1 gpurun_out/t12.log; [ $rc -eq 0 ] || exit $rc
for v in B P4 B2; do
  L=""; if [ $v = P4 ]; then L=$PWD/build_variants/libP4.so; fi
  DQ_LIB_PATH=$L timeout -k 10 300 python -u bench.py --skip-headline --configs c4 --cpu-sample 0 --ingest-rows 0 > gpurun_out/c4_$v.json 2>gpurun_out/c4_$v.err || { tail gpurun_out/c4_$v.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/c4_$v.json')); c=d['configs']['c4']; print('$v', c['ms_per_step'], c['roofline']['avg_launch_ms'])"
done
