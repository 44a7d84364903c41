# long_ab.sh TAG -- the LONG string pass: its GPU tests, then str_len_bench.py --path long for the row-order build
# (build_variants/libl0.so: DQ_LONG_PHASED=0) and the in-tree library, twice each (diagnostic A/B)
set -e
TAG=${1:-r6l}
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_utf8_hll.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${TAG}_utf8_tests.log 2>&1
for rep in 1 2; do
for lib in build_variants/libl0.so deequ_amd/libdqscan.so; do
  echo "== $lib" >> gpurun_out/${TAG}_strlen.txt
  DQ_LIB_PATH=$lib timeout -k 10 300 python -u tools/str_len_bench.py --path long --bands 8:24,16:48,24:100,0:120 >> gpurun_out/${TAG}_strlen.txt 2>&1
done
done
