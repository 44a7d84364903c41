#!/bin/bash
# round-4 GPU call 40: the numeric grouping compaction with the next tile's loads in flight -- full GPU suite, smoke(),
# then the grouping timing A/B at 1e8 rows (build_variants/libgold.so = before), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4g8_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g8_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4g8_pytest.log | tee $S; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4g8_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4g8_smoke.txt 2>&1
rc=$?; tail -1 gpurun_out/r4g8_smoke.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  for lib in build_variants/libgold.so deequ_amd/libdqscan.so; do
    echo "== $lib" | tee -a $S
    DQ_LIB_PATH=$lib timeout -k 10 400 python -u tools/group_bench.py --rows 1e8 > gpurun_out/r4g8_g.txt 2>&1
    rc=$?; grep "freq_build" gpurun_out/r4g8_g.txt | tee -a $S; [ $rc -eq 0 ] || exit $rc
  done
done
