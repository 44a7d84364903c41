#!/bin/bash
# round-4 GPU call 22: digest pass variants (diagnostic A/B at 1e8 rows): libprio0 = the shipped digest (4096
# workgroups per chunk, 11-step search, one LDS atomic per ballot); dg1 = 1024 workgroups; dg2 = + one LDS atomic
# per wave and iteration; dg3 = + the splitter lookup table (the in-tree defaults); dg4 = dg2 with 512 workgroups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export TMPDIR=/tmp
S=gpurun_out/r4v_summary.txt
timeout -k 10 300 python -u -m pytest tests/test_quantiles.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4v_pytest_quantiles.log 2>&1
rc=$?; tail -2 gpurun_out/r4v_pytest_quantiles.log | tee $S; [ $rc -eq 0 ] || exit $rc
for lib in prio0 dg1 dg2 dg3 dg4; do
  echo "== $lib" | tee -a $S
  DQ_LIB_PATH=build_variants/lib$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4v_$lib -o q --output-format csv -- python3 tools/quantile_bench.py --rows 1e8 --reps 3 > gpurun_out/r4v_$lib.txt 2>&1
  rc=$?; grep digest gpurun_out/r4v_$lib.txt | tee -a $S; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4v_$lib.txt; exit $rc; }
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/r4v_$lib/**/q_kernel_stats.csv',recursive=True)[0])):
    if 'digest' in r['Name'] or 'trampoline' in r['Name']: print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" | tee -a $S
done
