set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
for v in A B C; do
  if [ $v = B ]; then L=""; else L=$PWD/build_variants/lib$v.so; fi
  DQ_LIB_PATH=$L timeout -k 10 200 python -u tools/sweep.py 125000000 utf8x4_hll > gpurun_out/sw_$v.log 2>&1 || exit $?
  echo "$v: $(tail -1 gpurun_out/sw_$v.log)"
done
